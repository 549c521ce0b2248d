"""Developer probe for the tree-form SPD factors: one step of a few worlds per scene, NaN /
zero counts of the smooth and constrained accelerations and their error vs the oracle (not
a test)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import numpy as np
import torch
from parity_util import g1_states, oracle_step
from mjlab_amd.scenes import load_scene
from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg

for scene in sys.argv[1:] or ["g1_velocity"]:
  m = load_scene(scene)
  n = 16
  sim = Simulation(n, SimulationCfg(nconmax=48, njmax=160, mujoco=MujocoCfg(
      timestep=m.timestep, iterations=10, ls_iterations=20)), m, "cuda:0")
  q, qv, ctrl = g1_states(m, n, seed=2)
  d = sim.data
  d.qpos[:] = torch.tensor(q, dtype=torch.float32)
  d.qvel[:] = torch.tensor(qv, dtype=torch.float32)
  d.ctrl[:] = torch.tensor(ctrl, dtype=torch.float32)
  d.qacc_warmstart[:] = 0
  sim.forward()
  torch.cuda.synchronize()
  ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=False)
  print(scene, "spec", getattr(sim, "spec", None))
  for f in ("qacc_smooth", "qacc", "qfrc_smooth"):
    g = getattr(d, f).cpu().numpy()
    e = max(np.abs(g[i] - ref[i][f]).max() for i in range(n)) if f in ref[0] else float("nan")
    print(f"  {f:12s} nan {int(np.isnan(g).sum())} zero-rows {int((np.abs(g).max(1) == 0).sum())}"
          f" maxerr {e:.3e} scale {max(np.abs(r[f]).max() for r in ref) if f in ref[0] else 0:.3e}")
  print("  ncon", d.ncon.cpu().numpy()[:8], "nefc", d.nefc.cpu().numpy()[:8],
        "niter", d.solver_niter.cpu().numpy()[:8])
