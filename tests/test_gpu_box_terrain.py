"""Box-stair rough terrain on the GPU: the terrain broadphase (chunk and
box AABB culls over 3564 static boxes) and the box narrowphase against the fp64 oracle, and
the `Mjlab-Velocity-Rough-Unitree-G1` task with its terrain-level curriculum.

  - one mj_step with robots across stair edges of random stair patches matches the oracle
    (tolerances of tests/test_gpu_parity.py);
  - robots on the flat box patches reproduce the plane scene's step;
  - robots far above the terrain make no contacts (no box block survives the culls);
  - the rough task runs through the fused, graph-captured step: env origins follow the
    terrain levels, levels move only for resetting envs, the mean level is logged.
"""

import numpy as np
import pytest
import torch

from parity_util import oracle_step

pytestmark = pytest.mark.gpu


def _sim(m, n, device):
  from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
  cfg = SimulationCfg(nconmax=48, njmax=160,
                      mujoco=MujocoCfg(timestep=m.timestep, iterations=10, ls_iterations=20))
  return Simulation(n, cfg, m, device)


def _terrain_top(m, x, y):
  """Highest static box top under (x, y)."""
  st = (m.geom_type == 6) & (m.body_weldid[m.geom_bodyid] == 0)
  p, s = m.geom_pos[st], m.geom_size[st]
  inside = (np.abs(x - p[:, 0]) <= s[:, 0]) & (np.abs(y - p[:, 1]) <= s[:, 1])
  return float((p[inside, 2] + s[inside, 2]).max())


def _states(m, n, seed, cols, spread, dz=(-0.03, 0.02), height=0.74, tilt=0.0, flip=False):
  rng = np.random.default_rng(seed)
  o = m.arrays["terrain_origins"]
  q = np.tile(m.key_qpos, (n, 1))
  for i in range(n):
    r, c = rng.integers(0, o.shape[0]), rng.choice(cols)
    q[i, :2] = o[r, c, :2] + rng.uniform(-spread, spread, 2)
    q[i, 2] = _terrain_top(m, *q[i, :2]) + height + rng.uniform(*dz)
    if tilt > 0:  # random roll / pitch of the root
      ax = rng.normal(size=3)
      ax[2] = 0.0
      ax /= np.linalg.norm(ax)
      a = rng.uniform(-tilt, tilt)
      qt = np.array([np.cos(a / 2), *(np.sin(a / 2) * ax)])
      if flip:  # upside down (roll pi) before the tilt
        qt = np.array([-qt[1], qt[0], qt[3], -qt[2]])
      q[i, 3:7] = qt
  q[:, 7:] += rng.uniform(-0.1, 0.1, (n, m.nq - 7))
  qv = rng.normal(0, 0.3, (n, m.nv))
  qv[:, :3] *= 0.3
  jq = np.array([m.jnt_qposadr[j] for j in m.actuator_trnid])
  ctrl = q[:, jq] + rng.uniform(-0.2, 0.2, (n, m.nu))
  return q, qv, ctrl


def _load(sim, q, qv, ctrl):
  d = sim.data
  d.qpos[:] = torch.as_tensor(q, dtype=torch.float32)
  d.qvel[:] = torch.as_tensor(qv, dtype=torch.float32)
  d.ctrl[:] = torch.as_tensor(ctrl, dtype=torch.float32)
  d.qacc_warmstart[:] = 0


def test_rough_step_parity_across_stair_edges(gpu_device):
  from mjlab_amd.scenes import load_scene
  m = load_scene("g1_velocity_rough")
  n = 48
  sim = _sim(m, n, gpu_device)
  q, qv, ctrl = _states(m, n, seed=11, cols=range(8, 20), spread=2.6, dz=(-0.01, 0.03))
  _load(sim, q, qv, ctrl)
  sim.step()
  torch.cuda.synchronize()
  ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=True, nconmax=64)
  # worlds at the 160-row capacity drop rows by design (row_overflow), each side its own
  # way: skipped
  keep = [i for i, r in enumerate(ref) if r["nefc"] < 160]
  assert len(keep) >= n - 4
  d = sim.data
  ncon, qacc = d.ncon.cpu().numpy(), d.qacc.cpu().numpy()
  qpos, qvel = d.qpos.cpu().numpy(), d.qvel.cpu().numpy()
  sens = d.sensordata.cpu().numpy()
  # 5e-3 (test_gpu_parity.py: 2e-3): a sphere centre just outside a box edge gives an fp32
  # normal (nearest point - centre) / distance whose error grows as eps * |x| / distance, and
  # the stair patches sit up to 80 m from the origin
  for i in keep:
    r = ref[i]
    assert ncon[i] == r["ncon"], f"world {i}: ncon {ncon[i]} vs {r['ncon']}"
    sc = max(1.0, np.abs(r["qacc"]).max())
    np.testing.assert_allclose(qacc[i], r["qacc"], atol=5e-3 * sc, err_msg=f"qacc world {i}")
    np.testing.assert_allclose(qvel[i], r["qvel"], atol=5e-3 * sc * m.timestep + 1e-5)
    np.testing.assert_allclose(qpos[i], r["qpos"], atol=5e-3 * sc * m.timestep ** 2 + 1e-5)
    ssc = max(1.0, np.abs(r["sensordata"]).max())
    np.testing.assert_allclose(sens[i], r["sensordata"], atol=3e-3 * ssc, err_msg=f"sens {i}")
  assert sum(ref[i]["ncon"] > 0 for i in keep) >= n // 2
  assert sim.stats()["unsupported"] == 0


def test_go1_trunk_on_stairs_parity(gpu_device):
  """Go1 upside down on the stairs, trunk tilted: its trunk box meets the step boxes' faces
  and edges (box-box narrowphase)."""
  from mjlab_amd.scenes import load_scene
  m = load_scene("go1_velocity_rough")
  n = 48
  sim = _sim(m, n, gpu_device)
  q, qv, ctrl = _states(m, n, seed=21, cols=range(8, 20), spread=2.6, dz=(-0.02, 0.01),
                        height=0.05, tilt=0.4, flip=True)
  _load(sim, q, qv, ctrl)
  sim.step()
  torch.cuda.synchronize()
  ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=True, nconmax=64)
  keep = [i for i, r in enumerate(ref) if r["nefc"] < 160]
  assert len(keep) >= n - 8
  trunk = m.names["geom"].index("robot/trunk_collision")
  boxbox = sum(int(((r["contact"][:, 1] == trunk) | (r["contact"][:, 0] == trunk)).any()) for r in ref)
  assert boxbox >= n // 4
  d = sim.data
  ncon, qacc = d.ncon.cpu().numpy(), d.qacc.cpu().numpy()
  qpos, qvel = d.qpos.cpu().numpy(), d.qvel.cpu().numpy()
  for i in keep:
    r = ref[i]
    assert ncon[i] == r["ncon"], f"world {i}: ncon {ncon[i]} vs {r['ncon']}"
    sc = max(1.0, np.abs(r["qacc"]).max())
    np.testing.assert_allclose(qacc[i], r["qacc"], atol=5e-3 * sc, err_msg=f"qacc world {i}")
    np.testing.assert_allclose(qvel[i], r["qvel"], atol=5e-3 * sc * m.timestep + 1e-5)
    np.testing.assert_allclose(qpos[i], r["qpos"], atol=5e-3 * sc * m.timestep ** 2 + 1e-5)
  assert sim.stats()["unsupported"] == 0


def test_flat_box_patches_match_the_plane_on_gpu(gpu_device):
  from mjlab_amd.scenes import load_scene
  mr, mp = load_scene("g1_velocity_rough"), load_scene("g1_velocity")
  n = 16
  q, qv, ctrl = _states(mr, n, seed=12, cols=range(0, 8), spread=3.0)
  outs = []
  for m in (mr, mp):
    sim = _sim(m, n, gpu_device)
    _load(sim, q, qv, ctrl)
    sim.step()
    torch.cuda.synchronize()
    outs.append((sim.data.ncon.cpu().numpy(), sim.data.qacc.cpu().numpy(),
                 sim.data.qpos.cpu().numpy(), sim.data.sensordata.cpu().numpy()))
  np.testing.assert_array_equal(outs[0][0], outs[1][0])
  assert (outs[0][0] > 0).sum() >= n // 2
  for i in range(n):
    sc = max(1.0, np.abs(outs[1][1][i]).max())
    np.testing.assert_allclose(outs[0][1][i], outs[1][1][i], atol=1e-3 * sc)
    ssc = max(1.0, np.abs(outs[1][3][i]).max())
    np.testing.assert_allclose(outs[0][3][i], outs[1][3][i], atol=2e-3 * ssc)
  np.testing.assert_allclose(outs[0][2], outs[1][2], atol=1e-5)


def test_rough_cull_far_above(gpu_device):
  from mjlab_amd.scenes import load_scene
  m = load_scene("g1_velocity_rough")
  n = 8
  sim = _sim(m, n, gpu_device)
  q, qv, ctrl = _states(m, n, seed=13, cols=range(20), spread=3.0)
  q[:, 2] += 5.0
  _load(sim, q, qv, ctrl)
  sim.forward()
  torch.cuda.synchronize()
  ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=False, nconmax=64)
  assert list(sim.data.ncon.cpu().numpy()) == [r["ncon"] for r in ref]
  assert sim.stats()["unsupported"] == 0
  gx = sim.data.geom_xpos.cpu().numpy()
  st = np.where((m.geom_type == 6) & (m.body_weldid[m.geom_bodyid] == 0))[0]
  np.testing.assert_allclose(gx[:, st], np.broadcast_to(m.geom_pos[st], gx[:, st].shape), atol=1e-5)


@pytest.mark.parametrize("task,z0", [("Mjlab-Velocity-Rough-Unitree-G1", 0.76),
                                     ("Mjlab-Velocity-Rough-Unitree-Go1", 0.278)])
def test_rough_task_graph_step_and_terrain_levels(task, z0, gpu_device):
  from mjlab_amd.envs import make_env
  n = 256
  env = make_env(task, num_envs=n, device=gpu_device, seed=3)
  env.reset()
  terrain = env.scene.terrain
  # initial levels 0..5 (max_init_terrain_level); the reset's own curriculum pass moves
  # every env one level up (the default pose sits far from its origin), as the reference
  assert terrain is not None and int(terrain.terrain_levels.max()) <= 6
  z = env.scene["robot"].data.root_link_pos_w[:, 2] - env.scene.env_origins[:, 2]
  assert (z - z0).abs().max() < 0.05  # spawned on the sub-terrain origins
  env.enable_graph(capture=True)
  assert env._fused is not None, getattr(env, "_fused_unsupported", "")
  g = torch.Generator(device=gpu_device).manual_seed(0)
  nact = env.action_manager.total_action_dim
  moved = 0
  for _ in range(80):
    before = terrain.terrain_levels.clone()
    obs, rew, term, trunc, extras = env.step(2 * torch.rand(n, nact, device=gpu_device, generator=g) - 1)
    changed = terrain.terrain_levels != before
    assert not (changed & ~env.reset_buf).any()  # only resetting envs move
    moved += int(changed.sum())
    assert torch.equal(env.scene.env_origins,
                       terrain.terrain_origins[terrain.terrain_levels, terrain.terrain_types])
  torch.cuda.synchronize()
  assert moved > 0 and int(env.reset_buf.numel()) == n
  assert 0 <= int(terrain.terrain_levels.min()) and int(terrain.terrain_levels.max()) <= 9
  lvl = extras["log"]["Curriculum/terrain_levels"]
  assert float(lvl) == pytest.approx(float(terrain.terrain_levels.float().mean()))
  for v in obs.values():
    assert torch.isfinite(v).all()
  assert torch.isfinite(rew).all()
  assert env.sim.stats()["unsupported"] == 0


def test_rough_task_eager_step(gpu_device):
  from mjlab_amd.envs import make_env
  n = 64
  env = make_env("Mjlab-Velocity-Rough-Unitree-G1", num_envs=n, device=gpu_device, seed=4)
  env.reset()
  g = torch.Generator(device=gpu_device).manual_seed(1)
  nact = env.action_manager.total_action_dim
  for _ in range(40):
    obs, rew, term, trunc, extras = env.step(2 * torch.rand(n, nact, device=gpu_device, generator=g) - 1)
  terrain = env.scene.terrain
  assert torch.equal(env.scene.env_origins,
                     terrain.terrain_origins[terrain.terrain_levels, terrain.terrain_types])
  assert torch.isfinite(obs["policy"]).all() and torch.isfinite(rew).all()


def test_native_terrain_update_matches_the_torch_rule(gpu_device):
  """mjx_terrain_levels (the fused curriculum kernel) against the torch form of the same
  rule on one state: levels, origins and the mean level; wrap-around draws excepted."""
  from mjlab_amd import mdp
  from mjlab_amd.envs import make_env
  n = 512
  env = make_env("Mjlab-Velocity-Rough-Unitree-G1", num_envs=n, device=gpu_device, seed=5)
  env.reset()
  terrain = env.scene.terrain
  g = torch.Generator(device=gpu_device).manual_seed(0)
  root = int(env.scene["robot"].indexing.root_body_id)
  xpos = env.sim.data.xpos
  xpos[:, root, :2] = env.scene.env_origins[:, :2] + 12.0 * torch.rand(n, 2, device=gpu_device, generator=g) - 6.0
  mask = torch.rand(n, device=gpu_device, generator=g) < 0.5
  up, down = mdp._terrain_moves(env, slice(None), "twist")
  lv0 = terrain.terrain_levels.clone()
  want = lv0 + up.long() - down.long()
  wrap = mask & (want >= terrain.max_terrain_level)
  want = torch.where(mask, want.clamp(min=0), lv0)
  cmd = env.command_manager.get_command("twist")
  terrain.update_env_origins_native(mask, xpos, root, cmd, env.max_episode_length_s)
  torch.cuda.synchronize()
  assert torch.equal(terrain.terrain_levels[~wrap], want[~wrap])
  assert ((terrain.terrain_levels[wrap] >= 0) & (terrain.terrain_levels[wrap] < terrain.max_terrain_level)).all()
  assert int(mask.sum()) > 100 and int((up & mask).sum()) > 10 and int((down & mask).sum()) > 10
  assert torch.equal(env.scene.env_origins[mask],
                     terrain.terrain_origins[terrain.terrain_levels, terrain.terrain_types][mask])
  assert float(terrain.mean_level) == pytest.approx(float(terrain.terrain_levels.float().mean()), abs=1e-5)
