"""Inputs of scripts/chol_bench: a G1-shaped Newton Hessian H = M + J^T D J (tree-sparse M,
foot contact rows on leg chains + root) in the natural dof order and in a leaves-first
block order (the order the dropped block-parallel factor used), padded to 36, plus a
right-hand side."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd"))
from mjlab_amd.scenes import load_scene  # noqa: E402


NR = 36
m = load_scene("g1_velocity")
par = [int(p) for p in m.dof_parentid]
nv = len(par)
rng = np.random.default_rng(0)


def chain(i):
  out = []
  while i >= 0:
    out.append(i)
    i = par[i]
  return out


H = np.zeros((nv, nv))
for i in range(nv):  # M: cliques on ancestor chains
  c = chain(i)
  u = np.zeros(nv)
  u[c] = rng.normal(size=len(c))
  H += np.outer(u, u)
H += np.diag(rng.uniform(0.05, 0.5, nv))
for foot in (11, 17, 27, 34):  # contact rows on the foot / hand chains
  for _ in range(4):
    c = chain(foot)
    u = np.zeros(nv)
    u[c] = rng.normal(size=len(c))
    H += 30.0 * np.outer(u, u)
# leaves first: the four chain ends level by level, then waist and root (G1 dof tree)
perm = [27, 34, 11, 17, 26, 33, 10, 16, 25, 32, 9, 15, 24, 31, 8, 14, 23, 30, 7, 13, 22, 29, 6, 12,
        21, 28, -1, 20, 19, 18, 5, 4, 3, 2, 1, 0]
Hn = np.eye(NR)
Hn[:nv, :nv] = H
Hp = np.eye(NR)
for a, pa in enumerate(perm):
  for b, pb in enumerate(perm):
    if pa >= 0 and pb >= 0:
      Hp[a, b] = H[pa, pb]
b = rng.normal(size=NR)
b[nv:] = 0
bp = np.array([b[p] if p >= 0 else 0.0 for p in perm])
out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
os.makedirs(out, exist_ok=True)
Hn.astype(np.float32).tofile(os.path.join(out, "H_nat.bin"))
b.astype(np.float32).tofile(os.path.join(out, "b_nat.bin"))
Hp.astype(np.float32).tofile(os.path.join(out, "H_perm.bin"))
bp.astype(np.float32).tofile(os.path.join(out, "b_perm.bin"))
x = np.linalg.solve(Hn, b)
print("perm", perm)
print("x[0..3] natural", x[:4], " permuted", [x[p] for p in perm[:4]])
