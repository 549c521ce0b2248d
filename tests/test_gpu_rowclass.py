"""Newton row classes: worlds whose constraint-row count fits a
class capacity run the Newton phase in a smaller LDS carve, concurrently with the
full-capacity class.  The per-world arithmetic is the same code at other LDS offsets, so
every class split must give results bit-identical to the single-class run, and each
class must match the fp64 oracle (tolerances of tests/test_gpu_parity.py).

MJX355_ROW_CLASSES (read at Simulation creation) pins the class capacities: "" = none,
"8" = one class of <= 8 rows, "8,24" = two classes; unset = the automatic choice.
"""

import os

import numpy as np
import pytest
import torch

from parity_util import g1_states, oracle_step

pytestmark = pytest.mark.gpu


def _run(classes, q, qv, ctrl, device, nsteps=2):
  from mjlab_amd.scenes import load_scene
  from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
  old = os.environ.get("MJX355_ROW_CLASSES")
  if classes is None:
    os.environ.pop("MJX355_ROW_CLASSES", None)
  else:
    os.environ["MJX355_ROW_CLASSES"] = classes
  try:
    m = load_scene("g1_velocity")
    cfg = SimulationCfg(nconmax=48, njmax=160,
                        mujoco=MujocoCfg(timestep=m.timestep, iterations=10, ls_iterations=20))
    sim = Simulation(q.shape[0], cfg, m, device)
  finally:
    if old is None:
      os.environ.pop("MJX355_ROW_CLASSES", None)
    else:
      os.environ["MJX355_ROW_CLASSES"] = old
  d = sim.data
  d.qpos[:] = torch.as_tensor(q, dtype=torch.float32)
  d.qvel[:] = torch.as_tensor(qv, dtype=torch.float32)
  d.ctrl[:] = torch.as_tensor(ctrl, dtype=torch.float32)
  d.qacc_warmstart[:] = 0
  out = []
  for _ in range(nsteps):
    sim.step()
    torch.cuda.synchronize()
    out.append({k: getattr(d, k).cpu().numpy().copy()
                for k in ("qpos", "qvel", "qacc", "qfrc_constraint", "nefc", "solver_niter")})
  return m, out


def test_row_classes_bit_identical(gpu_device):
  n = 96
  from mjlab_amd.scenes import load_scene
  q, qv, ctrl = g1_states(load_scene("g1_velocity"), n, seed=11)
  _, base = _run("", q, qv, ctrl, gpu_device)
  nefc = base[0]["nefc"].reshape(-1)
  # the splits below must put worlds on both sides of each capacity
  assert (nefc <= 8).any() and (nefc > 24).any(), nefc
  for classes in ("8", "8,24", "24,40", None):
    _, got = _run(classes, q, qv, ctrl, gpu_device)
    for a, b in zip(base, got):
      for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=f"classes={classes!r} field {k}")


def test_row_classes_oracle(gpu_device):
  n = 48
  from mjlab_amd.scenes import load_scene
  m = load_scene("g1_velocity")
  q, qv, ctrl = g1_states(m, n, seed=12)
  _, got = _run("8,24", q, qv, ctrl, gpu_device, nsteps=1)
  ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=True)
  g = got[0]
  classes = {0: 0, 1: 0, 2: 0}
  for i, r in enumerate(ref):
    ne = int(g["nefc"].reshape(-1)[i])
    classes[1 if ne <= 8 else 2 if ne <= 24 else 0] += 1
    sc = max(1.0, np.abs(r["qacc"]).max())
    np.testing.assert_allclose(g["qacc"][i], r["qacc"], atol=2e-3 * sc)
    np.testing.assert_allclose(g["qvel"][i], r["qvel"], atol=2e-3 * sc * m.timestep + 1e-5)
  assert all(v > 0 for v in classes.values()), classes
