"""GPU behaviour of the Simulation / Entity boundary, mirroring the reference's own tests:
  tests/test_sim.py:89-135 (reset restores state, zeroes warmstart; selective reset);
  tests/test_entity_data.py:44-135 (root velocity write/read round trips, frames);
plus engine contracts: masked forward touches only masked worlds, stepping is
deterministic, step(n) equals n single steps, and the sync-free/graph env path runs."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sim(scene, n, device):
  from mjlab_amd.scenes import load_scene
  from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
  m = load_scene(scene)
  sim = Simulation(n, SimulationCfg(nconmax=48, njmax=160,
                                    mujoco=MujocoCfg(timestep=m.timestep, iterations=10,
                                                     ls_iterations=20)), m, device)
  return m, sim


def _keyframe(sim, m, device, jitter=0.0, seed=0):
  n = sim.num_envs
  g = torch.Generator(device="cpu").manual_seed(seed)
  q = torch.tensor(np.tile(m.key_qpos, (n, 1)), dtype=torch.float32)
  q[:, 7:] += jitter * (torch.rand(n, m.nq - 7, generator=g) - 0.5)
  sim.data.qpos[:] = q.to(device)
  jq = torch.tensor([m.jnt_qposadr[j] for j in m.actuator_trnid], device=device)
  sim.data.ctrl[:] = sim.data.qpos[:, jq]


def test_reset_restores_initial_state(gpu_device):
  m, sim = _sim("go1_velocity", 4, gpu_device)
  q0 = sim.data.qpos.clone()
  v0 = sim.data.qvel.clone()
  _keyframe(sim, m, gpu_device, jitter=0.2)
  for _ in range(10):
    sim.step()
  torch.cuda.synchronize()
  assert not torch.allclose(sim.data.qpos, q0)
  sim.reset()
  torch.testing.assert_close(sim.data.qpos[:], q0)
  torch.testing.assert_close(sim.data.qvel[:], v0)
  assert (sim.data.qacc_warmstart == 0).all()


def test_reset_selective(gpu_device):
  m, sim = _sim("go1_velocity", 4, gpu_device)
  q0 = sim.data.qpos.clone()
  _keyframe(sim, m, gpu_device, jitter=0.2)
  for _ in range(10):
    sim.step()
  after = sim.data.qpos.clone()
  sim.reset(torch.tensor([1, 3], device=gpu_device))
  torch.testing.assert_close(sim.data.qpos[1], q0[1])
  torch.testing.assert_close(sim.data.qpos[3], q0[3])
  torch.testing.assert_close(sim.data.qpos[0], after[0])
  torch.testing.assert_close(sim.data.qpos[2], after[2])


def test_masked_forward_only_touches_masked_worlds(gpu_device):
  m, sim = _sim("g1_velocity", 6, gpu_device)
  _keyframe(sim, m, gpu_device, jitter=0.1)
  sim.forward()
  xpos = sim.data.xpos.clone()
  sim.data.qpos[:, 2] += 0.25
  mask = torch.tensor([1, 0, 1, 0, 0, 1], dtype=torch.bool, device=gpu_device)
  sim.forward(mask)
  torch.cuda.synchronize()
  root = int(m.jnt_bodyid[0])  # body of the free joint (body 1 is the static terrain)
  moved = (sim.data.xpos[:, root, 2] - xpos[:, root, 2]).abs() > 0.2
  assert moved.tolist() == mask.tolist()


def test_overflow_counted_on_every_fused_substep(gpu_device):
  """The engine's per-world overflow counters (engine_counters[:, 2:5]) and the event
  totals must count the events of every substep of a fused multi-substep step, not only
  the last: with 8 constraint rows per world the standing G1's foot contacts overflow the
  rows on every substep, so one step(nsubstep=4) must count what four step() calls count."""
  from mjlab_amd.scenes import load_scene
  from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
  m = load_scene("g1_velocity")
  counts = []
  for fused in (True, False):
    sim = Simulation(16, SimulationCfg(nconmax=48, njmax=8, mujoco=MujocoCfg(
      timestep=m.timestep, iterations=10, ls_iterations=20)), m, gpu_device)
    _keyframe(sim, m, gpu_device, jitter=0.05)
    ev0 = sim.overflow_events().clone()
    if fused:
      sim.step(nsubstep=4)
    else:
      for _ in range(4):
        sim.step()
    torch.cuda.synchronize()
    counts.append((sim.engine_counters[:, 2:5].cpu().clone(), (sim.overflow_events() - ev0).cpu()))
  (wf, tf), (ws, ts) = counts
  assert int(ws[:, 1].max()) == 4, "expected a row overflow on each of the 4 substeps"
  assert torch.equal(wf, ws)
  assert torch.equal(tf, ts)


def test_step_is_deterministic(gpu_device):
  outs = []
  for _ in range(2):
    m, sim = _sim("g1_velocity", 64, gpu_device)
    _keyframe(sim, m, gpu_device, jitter=0.3, seed=5)
    for _ in range(8):
      sim.step()
    torch.cuda.synchronize()
    outs.append((sim.data.qpos.clone(), sim.data.qvel.clone(), sim.data.sensordata.clone()))
  for a, b in zip(*outs):
    assert torch.equal(a, b)


def test_multi_substep_equals_single_steps(gpu_device):
  res = []
  for fused in (True, False):
    m, sim = _sim("go1_velocity", 32, gpu_device)
    _keyframe(sim, m, gpu_device, jitter=0.3, seed=7)
    if fused:
      sim.step(4)
    else:
      for _ in range(4):
        sim.step()
    torch.cuda.synchronize()
    res.append((sim.data.qpos.clone(), sim.data.qvel.clone(), sim.data.time.clone()))
  for a, b in zip(*res):
    assert torch.equal(a, b)


@pytest.fixture()
def go1_env(gpu_device):
  from mjlab_amd.envs import make_env
  env = make_env("Mjlab-Velocity-Flat-Unitree-Go1", num_envs=2, device=gpu_device, seed=0)
  env.reset()
  return env


def test_root_velocity_world_frame_roundtrip(go1_env, gpu_device):
  """test_entity_data.py:44-70."""
  ent, sim = go1_env.scene["robot"], go1_env.sim
  pose = torch.tensor([0.0, 0.0, 1.0, 0.6, 0.2, 0.3, 0.7141], device=gpu_device).repeat(2, 1)
  ent.write_root_link_pose_to_sim(pose)
  vel = torch.tensor([1.0, 0.5, 0.0, 0.0, 0.3, 0.1], device=gpu_device).repeat(2, 1)
  ent.write_root_link_velocity_to_sim(vel)
  sim.forward()
  read = ent.data.root_link_vel_w.clone()
  assert torch.allclose(read, vel, atol=1e-4)
  ent.write_root_link_velocity_to_sim(read)
  sim.forward()
  assert torch.allclose(ent.data.root_link_vel_w, read, atol=1e-4)


def test_root_velocity_frame_conversion(go1_env, gpu_device):
  """test_entity_data.py:73-102: angular velocity stored in the body frame in qvel."""
  from mjlab_amd.math_utils import quat_apply_inverse
  ent, sim = go1_env.scene["robot"], go1_env.sim
  quat = torch.tensor([0.6, 0.2, 0.3, 0.7141], device=gpu_device).repeat(2, 1)
  ent.write_root_link_pose_to_sim(torch.cat([torch.zeros(2, 3, device=gpu_device), quat], -1))
  lin = torch.tensor([1.0, 0.5, 0.2], device=gpu_device).repeat(2, 1)
  ang = torch.tensor([0.1, 0.2, 0.3], device=gpu_device).repeat(2, 1)
  ent.write_root_link_velocity_to_sim(torch.cat([lin, ang], -1))
  qvel = sim.data.qvel[:, :6]
  assert torch.allclose(qvel[:, :3], lin, atol=1e-5)
  assert torch.allclose(qvel[:, 3:], quat_apply_inverse(quat, ang), atol=1e-5)


def test_write_velocity_uses_qpos_not_xquat(go1_env, gpu_device):
  """test_entity_data.py:105-132."""
  ent, sim = go1_env.scene["robot"], go1_env.sim
  ent.write_root_link_pose_to_sim(torch.tensor([0, 0, 1.0, 1, 0, 0, 0], device=gpu_device).repeat(2, 1))
  sim.forward()
  vel = torch.tensor([1.0, 0.0, 0.0, 0.0, 1.0, 0.0], device=gpu_device).repeat(2, 1)
  ent.write_root_link_pose_to_sim(torch.tensor([0, 0, 1.0, 0.707, 0, 0.707, 0], device=gpu_device).repeat(2, 1))
  ent.write_root_link_velocity_to_sim(vel)
  sim.forward()
  assert torch.allclose(ent.data.root_link_vel_w, vel, atol=1e-4)


@pytest.mark.parametrize("task", ["Mjlab-Velocity-Flat-Unitree-G1", "Mjlab-Velocity-Flat-Unitree-Go1"])
def test_env_graph_step(task, gpu_device):
  """Sync-free env step captured in a HIP graph: observations finite, rewards finite,
  resets happen through the masked path, episode counters advance."""
  from mjlab_amd.envs import make_env
  env = make_env(task, num_envs=256, device=gpu_device, seed=1)
  env.reset()
  env.enable_graph(capture=True)
  g = torch.Generator(device=gpu_device).manual_seed(0)
  nact = env.action_manager.total_action_dim
  for _ in range(30):
    obs, rew, term, trunc, extras = env.step(2 * torch.rand(256, nact, device=gpu_device, generator=g) - 1)
  torch.cuda.synchronize()
  for v in obs.values():
    assert torch.isfinite(v).all()
  assert torch.isfinite(rew).all()
  assert env.sim.stats()["unsupported"] == 0


def test_overflow_event_total_matches_world_counters(gpu_device):
  """engine_events (one atomic per overflow event) equals the per-world cumulative
  counters summed over worlds; an 8-row capacity forces row overflow."""
  from mjlab_amd.scenes import load_scene
  from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
  m = load_scene("g1_velocity")
  sim = Simulation(16, SimulationCfg(nconmax=48, njmax=8, mujoco=MujocoCfg(timestep=m.timestep)),
                   m, gpu_device)
  _keyframe(sim, m, gpu_device, jitter=0.1)
  for _ in range(6):
    sim.step()
  torch.cuda.synchronize()
  per_world = sim.engine_counters[:, 2:5].sum(dim=0)
  total = sim.overflow_events()
  assert total.tolist() == per_world.tolist()
  assert int(total[1]) > 0
