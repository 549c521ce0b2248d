"""Config 1 of BASELINE.json on the host: `Mjlab-Velocity-Flat-Unitree-G1`, num_envs = 1,
zero actions (`--agent zero`), the whole env on the CPU -- the torch managers on CPU tensors
and the fp64 oracle behind the physics boundary (tests/oracle_sim.py; the product itself has
no CPU path).  A plumbing test, as SURVEY.md section 8d defines config 1."""

import torch

from oracle_sim import make_cpu_env


def test_config1_cpu_env_plumbing():
  env = make_cpu_env("Mjlab-Velocity-Flat-Unitree-G1", num_envs=1, seed=42)
  obs, extras = env.reset()
  assert obs["policy"].shape == (1, 99) and obs["critic"].shape == (1, 111)
  z = torch.zeros(1, env.action_manager.total_action_dim)
  for _ in range(40):
    obs, rew, term, trunc, extras = env.step(z)
    assert torch.isfinite(obs["policy"]).all() and torch.isfinite(rew).all()
  # zero action holds the knees-bent default pose: the pelvis stays up, nothing terminates
  robot = env.scene["robot"]
  assert float(robot.data.root_link_pos_w[0, 2]) > 0.6
  assert not bool(term.any())
  assert env.sim.overflow_events().tolist() == [0, 0, 0]
  # feet on the ground: the contact sensor sees both feet, the air-time clock runs
  fc = env.scene["feet_ground_contact"].data
  assert (fc.found > 0).all()
  assert int(env.common_step_counter) == 40
