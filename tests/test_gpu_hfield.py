"""Heightfield collision on the GPU and the jump task (row a29).

  - one mj_step on the config-5 terrain (200 heightfield patches) matches the fp64 oracle
    (same tolerances as tests/test_gpu_parity.py), robots spread over random patches;
  - a flattened heightfield terrain reproduces the plane scene's step on the GPU;
  - robots far above the terrain make no contacts and raise no unsupported-pair flag
    (the AABB cull leaves no hfield block active);
  - the jump task (flat and heightfield) runs through the sync-free graph-captured step.
"""

import copy

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


def _states(m, n, seed, dz=(-0.04, 0.02)):
  rng = np.random.default_rng(seed)
  o = m.arrays["terrain_origins"]
  q = np.tile(m.key_qpos, (n, 1))
  for i in range(n):
    r, c = rng.integers(0, o.shape[0]), rng.integers(0, o.shape[1])
    q[i, :2] = o[r, c, :2] + rng.uniform(-0.6, 0.6, 2)  # on the spawn platform
    q[i, 2] = o[r, c, 2] + 0.55 + rng.uniform(*dz)
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


def _check_step(m, sim, q, qv, ctrl, min_contact_worlds=1):
  ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=True, nconmax=64)
  d = sim.data
  ncon, qacc = d.ncon.cpu().numpy(), d.qacc.cpu().numpy()
  qpos, qvel = d.qpos.cpu().numpy(), d.qvel.cpu().numpy()
  sens = d.sensordata.cpu().numpy()
  hit = 0
  for i, r in enumerate(ref):
    assert ncon[i] == r["ncon"], f"world {i}: ncon {ncon[i]} vs {r['ncon']}"
    hit += r["ncon"] > 0
    sc = max(1.0, np.abs(r["qacc"]).max())
    np.testing.assert_allclose(qacc[i], r["qacc"], atol=2e-3 * sc, err_msg=f"qacc world {i}")
    np.testing.assert_allclose(qvel[i], r["qvel"], atol=2e-3 * sc * m.timestep + 1e-5)
    np.testing.assert_allclose(qpos[i], r["qpos"], atol=2e-3 * sc * m.timestep ** 2 + 1e-5)  # h x the qvel bound
    ssc = max(1.0, np.abs(r["sensordata"]).max())
    np.testing.assert_allclose(sens[i], r["sensordata"], atol=3e-3 * ssc, err_msg=f"sens {i}")
  assert hit >= min_contact_worlds
  assert sim.stats()["unsupported"] == 0


def test_hfield_step_parity(gpu_device):
  from mjlab_amd.scenes import load_scene
  m = load_scene("g1_jump_hfield")
  n = 48
  sim = _sim(m, n, gpu_device)
  q, qv, ctrl = _states(m, n, seed=4)
  _load(sim, q, qv, ctrl)
  sim.step()
  torch.cuda.synchronize()
  _check_step(m, sim, q, qv, ctrl, min_contact_worlds=n // 2)


def test_flat_hfield_matches_plane_on_gpu(gpu_device):
  from mjlab_amd.scenes import load_scene
  mh = copy.deepcopy(load_scene("g1_jump_hfield"))
  mh.arrays["hfield_data"] = np.zeros_like(mh.arrays["hfield_data"])
  gp = mh.arrays["geom_pos"].copy()
  gp[mh.geom_type == 1, 2] = 0.0
  mh.arrays["geom_pos"] = gp
  mp = load_scene("g1_jump")
  n = 16
  q, qv, ctrl = _states(mh, n, seed=5)
  q[:, 2] = 0.55 + np.random.default_rng(6).uniform(-0.03, 0.01, n)
  outs = []
  for m in (mh, mp):
    sim = _sim(m, n, gpu_device)
    _load(sim, q, qv, ctrl)
    sim.step()
    torch.cuda.synchronize()
    outs.append((sim.data.ncon.cpu().numpy(), sim.data.qacc.cpu().numpy(),
                 sim.data.qpos.cpu().numpy()))
  np.testing.assert_array_equal(outs[0][0], outs[1][0])
  assert outs[0][0].min() > 0
  for i in range(n):
    sc = max(1.0, np.abs(outs[1][1][i]).max())
    np.testing.assert_allclose(outs[0][1][i], outs[1][1][i], atol=1e-3 * sc)
  np.testing.assert_allclose(outs[0][2], outs[1][2], atol=1e-5)


def test_hfield_cull_far_above(gpu_device):
  from mjlab_amd.scenes import load_scene
  m = load_scene("g1_jump_hfield")
  n = 8
  sim = _sim(m, n, gpu_device)
  q, qv, ctrl = _states(m, n, seed=7)
  q[:, 2] += 5.0
  _load(sim, q, qv, ctrl)
  sim.forward()
  torch.cuda.synchronize()
  ncon = sim.data.ncon.cpu().numpy()
  ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=False, nconmax=64)
  assert list(ncon) == [r["ncon"] for r in ref]
  assert sim.stats()["unsupported"] == 0
  # static heightfield frames are published for every world
  gx = sim.data.geom_xpos.cpu().numpy()
  hid = np.where(m.geom_type == 1)[0]
  np.testing.assert_allclose(gx[:, hid], np.broadcast_to(m.geom_pos[hid], gx[:, hid].shape), atol=1e-5)


@pytest.mark.parametrize("task", ["Mjlab-Jump-Flat-Unitree-G1", "Mjlab-Jump-Hfield-Unitree-G1"])
def test_jump_graph_step(task, gpu_device):
  from mjlab_amd.envs import make_env
  n = 128
  env = make_env(task, num_envs=n, device=gpu_device, seed=2)
  env.reset()
  if task.endswith("Hfield-Unitree-G1"):
    # spawn on the sub-terrain origins (reset_base adds env_origins)
    z = env.scene["robot"].data.root_link_pos_w[:, 2] - env.scene.env_origins[:, 2]
    assert (z - 0.55).abs().max() < 0.02
  env.enable_graph(capture=True)
  g = torch.Generator(device=gpu_device).manual_seed(0)
  nact = env.action_manager.total_action_dim
  for _ in range(20):
    obs, rew, term, trunc, _ = env.step(2 * torch.rand(n, nact, device=gpu_device, generator=g) - 1)
  torch.cuda.synchronize()
  assert obs["policy"].shape == (n, 3 + 3 + 3 + 29 + 29 + 29 + 1 + 1 + 2 + 2 + 1)
  for v in obs.values():
    assert torch.isfinite(v).all()
  assert torch.isfinite(rew).all()
  assert env.sim.stats()["unsupported"] == 0
