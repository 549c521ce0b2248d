"""Capsule-capsule on the GPU against the oracle (MuJoCo's mjc_CapsuleCapsule,
engine_collision_primitive.c; engine_impl.h capsule_capsule, oracle.c col_capsule_capsule):
crossed, exactly parallel (two contacts from the segment ends), anti-parallel, collinear
end-to-end (MuJoCo's duplicate contact) and random general poses -- contact count, depth,
point and normal, then the stepped state."""

import numpy as np
import pytest
import torch

from parity_util import oracle_step
from test_capsule_capsule import state, two_capsules

pytestmark = pytest.mark.gpu


def _states(n, seed):
  rng = np.random.default_rng(seed)
  qs = [state((0, 0, 0), (1, 0, 0), (0.05, 0.02, 0.09), (0, 1, 0)),
        state((0, 0, 0), (1, 0, 0), (0.1, 0, 0.09), (1, 0, 0)),
        state((0, 0, 0), (1, 0, 0), (0.0, 0, 0.095), (-1, 0, 0)),
        state((0, 0, 0), (1, 0, 0), (0.45, 0, 0.0), (1, 0, 0))]
  while len(qs) < n:
    pa = rng.uniform(-0.05, 0.05, 3)
    ax = rng.normal(size=3)
    if len(qs) % 2:  # exactly parallel, offset along and across the axis
      u = ax / np.linalg.norm(ax)
      side = np.cross(u, rng.normal(size=3))
      side *= rng.uniform(0.085, 0.099) / np.linalg.norm(side)
      pb = pa + side + u * rng.uniform(-0.35, 0.35)
      qs.append(state(pa, ax, pb, ax if rng.uniform() < 0.5 else -ax))
    else:
      qs.append(state(pa, ax, pa + rng.uniform(-0.12, 0.12, 3), rng.normal(size=3)))
  return np.array(qs[:n])


def test_capsule_capsule_contacts_and_step(gpu_device):
  from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
  m = two_capsules()
  n = 64
  q = _states(n, seed=4)
  qv = np.zeros((n, m.nv))
  ctrl = np.zeros((n, m.nu))
  cfg = SimulationCfg(nconmax=8, njmax=40,
                      mujoco=MujocoCfg(timestep=m.timestep, iterations=10, ls_iterations=20))
  sim = Simulation(n, cfg, m, gpu_device)
  d = sim.data
  d.qpos[:] = torch.as_tensor(q, dtype=torch.float32)
  d.qvel.zero_()
  d.qacc_warmstart.zero_()
  sim.forward()
  torch.cuda.synchronize()
  ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=False, nconmax=8, njmax=40)
  ncon = d.ncon.cpu().numpy()
  dist = d.contact_dist.reshape(n, -1).cpu().numpy()
  pos = d.contact_pos.reshape(n, -1, 3).cpu().numpy()
  frame = d.contact_frame.reshape(n, -1, 9).cpu().numpy()
  two = 0
  for i, r in enumerate(ref):
    assert ncon[i] == r["ncon"], f"world {i}: ncon {ncon[i]} vs {r['ncon']}"
    two += r["ncon"] == 2
    c = r["contact"]
    k = int(ncon[i])
    np.testing.assert_allclose(dist[i, :k], c[:, 2], atol=2e-6, err_msg=f"dist {i}")
    np.testing.assert_allclose(pos[i, :k], c[:, 3:6], atol=2e-6, err_msg=f"pos {i}")
    np.testing.assert_allclose(frame[i, :k, :3], c[:, 6:9], atol=2e-5, err_msg=f"normal {i}")
  assert two >= n // 3  # the parallel cases touch at both ends
  # one step from there
  d.qpos[:] = torch.as_tensor(q, dtype=torch.float32)
  d.qvel.zero_()
  d.qacc_warmstart.zero_()
  sim.step()
  torch.cuda.synchronize()
  ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=True, nconmax=8, njmax=40)
  qacc = d.qacc.cpu().numpy()
  for i, r in enumerate(ref):
    sc = max(1.0, np.abs(r["qacc"]).max())
    np.testing.assert_allclose(qacc[i], r["qacc"], atol=2e-3 * sc, err_msg=f"qacc world {i}")
  assert sim.stats()["unsupported"] == 0
