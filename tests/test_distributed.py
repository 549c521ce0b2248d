"""World-size-2 gloo checks of the multi-process path (mjlab_amd/distributed.py), on CPU."""

import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _worker(rank, world, port, q):
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                    RANK=str(rank), LOCAL_RANK=str(rank))
  from mjlab_amd import distributed as d
  d.init("gloo")
  try:
    w, r, lr = d.world_info()
    mx = d.max_over_ranks(1.5 + rank)
    stats = torch.arange(2 + rank, dtype=torch.float32) + 10 * rank  # ragged lengths
    g = d.gather_stats(stats)
    q.put((rank, w, r, mx, g.tolist(), d.rank_seed(42, r)))
  finally:
    import torch.distributed as dist
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_gloo():
  world, port = 2, _free_port()
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
  for p in procs:
    p.start()
  res = sorted(q.get(timeout=90) for _ in range(world))
  for p in procs:
    p.join(timeout=30)
    assert p.exitcode == 0
  for rank, w, r, mx, g, seed in res:
    assert (w, r) == (2, rank)
    assert mx == 2.5                       # max over ranks
    assert g == [[0.0, 1.0, 0.0], [10.0, 11.0, 12.0]]  # zero-padded all-gather
    assert seed == 42 + rank


def test_single_process_passthrough():
  from mjlab_amd import distributed as d
  assert d.max_over_ranks(3.0) == 3.0
  assert d.gather_stats(torch.ones(3)).shape == (1, 3)
