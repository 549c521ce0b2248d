"""Fused HIP managers on the jump task (mjlab_amd/fused.py FusedJumpStep, the jump branch of
csrc/velocity_task.hip) against the torch manager path of mjlab_amd/jump.py on identical
state: rewards (stateful jump height / landing balance included), per-term step rewards,
terminations (root height, excessive landing force), JumpCommand state, the jump
observation layout, the per-step metrics and the reset path.

Randomness is neutralised so both paths are deterministic: observation corruption off,
reset pose / joint offsets zero (the fused kernels draw from a
counter-based hash, the torch path from Philox).
Tolerances: fp32 with different operation order: rewards rtol 1e-4 atol 1e-5 (the
explosive-takeoff power sum and the joint-velocity variance reduce over 29 joints in a
different order: step rewards atol 1e-4); observations atol 1e-4; flags exact."""

import pytest
import torch

pytestmark = pytest.mark.gpu

TASKS = ["Mjlab-Jump-Flat-Unitree-G1", "Mjlab-Jump-Hfield-Unitree-G1"]


def _env(task, n, device, fused, zero_reset=False):
  from mjlab_amd.envs import ManagerBasedRlEnv, load_env_cfg
  cfg = load_env_cfg(task, False)
  cfg.scene.num_envs = n
  cfg.seed = 3
  cfg.observations["policy"].enable_corruption = False
  if zero_reset:
    cfg.events["reset_base"].params["pose_range"] = {}
    cfg.events["reset_robot_joints"].params["position_range"] = (0.0, 0.0)
  env = ManagerBasedRlEnv(cfg, device=device)
  env.reset()
  env.enable_graph(capture=False, fused=fused)
  assert (env._fused is not None) == fused, getattr(env, "_fused_unsupported", "")
  return env


def _close(a, b, **kw):
  torch.testing.assert_close(torch.as_tensor(a).float(), torch.as_tensor(b).float(), **kw)


def _stateful(env):
  rm = env.reward_manager
  jh = rm._term_cfgs[rm._term_names.index("jump_height")].func
  lb = rm._term_cfgs[rm._term_names.index("landing_stability")].func
  return jh, lb


@pytest.mark.parametrize("task", TASKS)
def test_fused_jump_step_matches_torch(task, gpu_device):
  n = 128
  # zero reset ranges: on the heightfield some envs terminate within these steps
  et = _env(task, n, gpu_device, fused=False, zero_reset=True)
  ef = _env(task, n, gpu_device, fused=True, zero_reset=True)
  g = torch.Generator(device=gpu_device).manual_seed(0)
  nact = et.action_manager.total_action_dim
  for step in range(8):
    a = 0.5 * (2 * torch.rand(n, nact, device=gpu_device, generator=g) - 1)
    ot, rt, tt, ut, _ = et.step(a)
    of, rf, tf, uf, _ = ef.step(a)
    torch.cuda.synchronize()
    assert torch.equal(tt, tf) and torch.equal(ut, uf)
    _close(rt, rf, rtol=1e-4, atol=1e-5)
    _close(et.reward_manager._step_reward, ef.reward_manager._step_reward, rtol=1e-4, atol=1e-4)
    for k in ("policy", "critic"):
      _close(ot[k], of[k], rtol=1e-4, atol=1e-4)
    _close(et.command_manager.get_command("jump"), ef.command_manager.get_command("jump"))
    _close(et.sim.data.qpos, ef.sim.data.qpos, rtol=1e-4, atol=1e-4)
    for st, sf in zip(_stateful(et), _stateful(ef)):
      for attr in ("peak_heights", "initial_heights", "stability_timer"):
        if hasattr(st, attr):
          _close(getattr(st, attr), getattr(sf, attr), rtol=1e-5, atol=1e-5)
      for attr in ("initialized", "was_in_air"):
        if hasattr(st, attr):
          assert torch.equal(getattr(st, attr), getattr(sf, attr))
    log_t, log_f = et.extras["log"], ef.extras["log"]
    for k in ("Metrics/peak_jump_height", "Metrics/jump_height", "Metrics/landing_success_rate",
              "Metrics/air_time_mean", "Metrics/angular_momentum_mean"):
      assert k in log_f, k
      _close(log_t[k], log_f[k].reshape(()), rtol=1e-4, atol=1e-5)
  for name in et.reward_manager._term_names:
    _close(et.reward_manager._episode_sums[name], ef.reward_manager._episode_sums[name],
           rtol=1e-4, atol=1e-5)
  assert torch.equal(et.episode_length_buf, ef.episode_length_buf)


def test_fused_jump_reset_path_matches_torch(gpu_device):
  task = TASKS[0]
  n = 64
  et = _env(task, n, gpu_device, fused=False, zero_reset=True)
  ef = _env(task, n, gpu_device, fused=True, zero_reset=True)
  maxlen = et.max_episode_length
  for e in (et, ef):
    e.episode_length_buf[::3] = maxlen - 1  # these envs time out on the next step
  a = torch.zeros(n, et.action_manager.total_action_dim, device=gpu_device)
  ot, rt, tt, ut, _ = et.step(a)
  of, rf, tf, uf, _ = ef.step(a)
  torch.cuda.synchronize()
  assert torch.equal(ut, uf) and ut[::3].all()
  assert torch.equal(et.episode_length_buf, ef.episode_length_buf)
  mask = ut.clone()
  _close(et.sim.data.qpos[mask], ef.sim.data.qpos[mask], rtol=1e-5, atol=1e-5)
  _close(et.sim.data.qvel[mask], ef.sim.data.qvel[mask], rtol=0, atol=1e-6)
  assert (ef.action_manager.action[mask] == 0).all()
  for k in ("policy", "critic"):
    _close(ot[k], of[k], rtol=1e-4, atol=1e-4)
  ct, cf = et.command_manager.get_term("jump"), ef.command_manager.get_term("jump")
  assert torch.equal(ct.command_counter, cf.command_counter)
  _close(ct.time_left, cf.time_left, rtol=1e-6, atol=0)
  log_t, log_f = et.extras["log"], ef.extras["log"]
  for k, v in log_t.items():
    if k.startswith(("Episode_Reward/", "Episode_Termination/", "Metrics/jump/")):
      assert k in log_f, k
      _close(torch.as_tensor(v, device=gpu_device).reshape(()), log_f[k].reshape(()),
             rtol=1e-4, atol=1e-6)
