"""Developer probe: GPU vs oracle contact lists on the box-stair scene (not a test)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import numpy as np, torch
from test_gpu_box_terrain import _sim, _states, _load
from parity_util import oracle_step
from mjlab_amd.scenes import load_scene
m = load_scene("g1_velocity_rough")
n = 48
sim = _sim(m, n, "cuda:0")
q, qv, ctrl = _states(m, n, seed=11, cols=range(8, 20), spread=2.6, dz=(-0.01, 0.03))
_load(sim, q, qv, ctrl)
sim.forward(); torch.cuda.synchronize()
ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=False, nconmax=64)
d = sim.data
ncon = d.ncon.cpu().numpy(); cg = d.contact_geom.cpu().numpy(); cd = d.contact_dist.cpu().numpy()
cp = d.contact_pos.cpu().numpy(); cf = d.contact_frame.cpu().numpy(); qacc = d.qacc.cpu().numpy()
bad = 0
for i in range(n):
  r = ref[i]
  k = min(ncon[i], r["ncon"])
  rc = r["contact"]
  geq = ncon[i] == r["ncon"] and np.array_equal(cg[i][:k], rc[:k, :2].astype(int))
  dd = np.abs(cd[i][:k] - rc[:k, 2]).max() if k else 0
  pd = np.abs(cp[i][:k] - rc[:k, 3:6]).max() if k else 0
  nd = np.abs(cf[i][:k, :3] - rc[:k, 6:9]).max() if k else 0
  qd = np.abs(qacc[i] - r["qacc"]).max() / max(1, np.abs(r["qacc"]).max())
  if not geq or dd > 1e-4 or pd > 1e-4 or nd > 1e-3 or qd > 2e-3:
    bad += 1
    print(f"world {i}: ncon {ncon[i]}/{r['ncon']} geoms_eq {geq} dist {dd:.2e} pos {pd:.2e} normal {nd:.2e} qacc_rel {qd:.2e} nefc {r['nefc']} q {q[i,:3]}")
    if bad <= 2:
      for j in range(max(ncon[i], r["ncon"])):
        g = (cg[i][j].tolist(), round(float(cd[i][j]), 5), np.round(cp[i][j], 4).tolist(), np.round(cf[i][j][:3], 3).tolist()) if j < ncon[i] else None
        o = (rc[j, :2].astype(int).tolist(), round(float(rc[j, 2]), 5), np.round(rc[j, 3:6], 4).tolist(), np.round(rc[j, 6:9], 3).tolist()) if j < r["ncon"] else None
        print("   ", g, "|", o)
print("bad", bad, sim.stats())
