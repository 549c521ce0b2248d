"""Leaves-first dof order for the engine's register-row Cholesky.

The Newton Hessian H = M + J^T D J of a tree has MuJoCo's branch-induced sparsity: M couples
a dof only with its ancestors and descendants, and a contact against a static geom couples
the dofs on one body's ancestor chain.  Eliminated leaves first, such a matrix factors
without fill (MuJoCo's mj_factorM runs backwards over the tree order for the same reason),
and dofs whose descendants have all been eliminated are mutually uncoupled.  The engine
factors in 4-column blocks; `block_order` fills the blocks by Hu's list schedule (ready dofs
with the longest remaining chain to the root first), so as many blocks as possible hold 4
mutually uncoupled pivots, which the kernel factors side by side (`rows_chol_blk`).

The order only changes the elimination order of an SPD solve: any permutation is exact in
exact arithmetic, and the kernel checks each block's independence at run time.
"""

from __future__ import annotations

from typing import Sequence


def block_order(parent: Sequence[int], nvp: int) -> list[int]:
  """Position -> dof index (-1 = identity padding), length `nvp` (a multiple of 4, >= nv).

  `parent[i]` is dof i's parent dof (-1 for a root), parents before children (MuJoCo's
  dof_parentid).  Padding slots fill blocks that would otherwise have to take a dof
  coupled with a pivot of the same block.
  """
  nv = len(parent)
  if nvp < nv or nvp % 4:
    raise ValueError(f"nvp {nvp} must be a multiple of 4 and >= nv {nv}")
  depth = [0] * nv
  for i in range(nv):
    p = int(parent[i])
    if p >= i:
      raise ValueError("dof_parentid must list parents before children")
    depth[i] = depth[p] + 1 if p >= 0 else 1
  nchild = [0] * nv
  for i in range(nv):
    if parent[i] >= 0:
      nchild[int(parent[i])] += 1
  ready = {i for i in range(nv) if nchild[i] == 0}
  pads = nvp - nv
  order: list[int] = []

  def place(i: int) -> None:
    order.append(i)
    ready.discard(i)
    p = int(parent[i])
    if p >= 0:
      nchild[p] -= 1
      if nchild[p] == 0:
        ready.add(p)

  while len([o for o in order if o >= 0]) < nv:
    # the dofs ready at the block's start are mutually uncoupled
    pick = sorted(ready, key=lambda i: (-depth[i], i))[:4]
    for i in pick:
      place(i)
    need = 4 - len(pick)
    while need and pads:
      order.append(-1)
      pads -= 1
      need -= 1
    while need and ready:  # no padding left: a chained block
      place(min(ready, key=lambda i: (-depth[i], i)))
      need -= 1
    if need:  # every dof placed
      break
  order.extend([-1] * (nvp - len(order)))
  return order


def independent_blocks(parent: Sequence[int], order: Sequence[int]) -> list[bool]:
  """Per 4-block of `order`: are its pivots mutually uncoupled for a tree-sparse H (no
  pivot an ancestor of another)?  The kernel decides this per matrix at run time; this is
  the structural answer, for tests and DESIGN numbers."""
  def anc(i):
    out = set()
    i = int(parent[i])
    while i >= 0:
      out.add(i)
      i = int(parent[i])
    return out
  res = []
  for b in range(0, len(order), 4):
    blk = [i for i in order[b:b + 4] if i >= 0]
    res.append(all(j not in anc(i) for i in blk for j in blk if i != j))
  return res
