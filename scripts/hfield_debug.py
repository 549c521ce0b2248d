"""Developer probe: GPU vs oracle contact lists on the heightfield scene (not a test)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import numpy as np, torch
from test_gpu_hfield import _sim, _states, _load
from parity_util import oracle_step
from mjlab_amd.scenes import load_scene
m = load_scene("g1_jump_hfield")
n = 48
sim = _sim(m, n, "cuda:0")
q, qv, ctrl = _states(m, n, seed=4)
_load(sim, q, qv, ctrl)
sim.forward(); torch.cuda.synchronize()
ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=False, nconmax=64)
ncon = sim.data.ncon.cpu().numpy(); cg = sim.data.contact_geom.cpu().numpy(); cd = sim.data.contact_dist.cpu().numpy()
for i in range(n):
  if ncon[i] != ref[i]["ncon"]:
    go = sorted((int(a), int(b), round(float(c), 5)) for (a, b), c in zip(cg[i][:ncon[i]], cd[i][:ncon[i]]))
    ro = sorted((int(r[0]), int(r[1]), round(float(r[2]), 5)) for r in ref[i]["contact"])
    print("world", i, "gpu", ncon[i], "ref", ref[i]["ncon"], "q", q[i, :3])
    print("  only gpu:", sorted(set(go) - set(ro)))
    print("  only ref:", sorted(set(ro) - set(go)))
print(sim.stats())
