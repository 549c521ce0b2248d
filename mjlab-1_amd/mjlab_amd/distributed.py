"""Multi-GPU plumbing: one process per GPU, worlds sharded by rank.

Worlds never interact, so the data path has no collective: each rank steps its own
`num_envs` worlds (reference semantics, docs/api/distributed_training.md:43-92) with seed
base + rank (scripts/train.py:59).  The only cross-rank traffic is bookkeeping:
  - the timed region's MAX over ranks (bench), and
  - one packed fp32 all-gather of episode statistics per report (~30 scalars per rank),
over RCCL (backend "nccl") on the GPU box, gloo on CPU for tests.
"""

from __future__ import annotations

import os

import torch
import torch.distributed as dist


def world_info() -> tuple[int, int, int]:
  """(world_size, rank, local_rank) from the torch.distributed.run environment."""
  return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
          int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str = "nccl", device: torch.device | None = None) -> None:
  """Initialise the process group (127.0.0.1 rendezvous comes from MASTER_ADDR)."""
  os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
  if dist.is_initialized():
    return
  if backend == "nccl" and device is not None:
    dist.init_process_group("nccl", device_id=device)
  else:
    dist.init_process_group(backend)


def rank_seed(base: int, rank: int) -> int:
  return int(base) + int(rank)


def max_over_ranks(value: float, device: torch.device | str = "cpu") -> float:
  """Max of a host scalar over ranks (the driver's timing rule: slowest rank wins)."""
  if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
    return float(value)
  t = torch.tensor([float(value)], dtype=torch.float64, device=device)
  dist.all_reduce(t, op=dist.ReduceOp.MAX)
  return float(t.item())


def gather_stats(stats: torch.Tensor) -> torch.Tensor:
  """All-gather a packed fp32 statistics vector: [world_size, n] on every rank.
  Vectors of different length are zero-padded to the longest."""
  if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
    return stats.reshape(1, -1)
  n = torch.tensor([stats.numel()], device=stats.device)
  dist.all_reduce(n, op=dist.ReduceOp.MAX)
  buf = torch.zeros(int(n.item()), dtype=torch.float32, device=stats.device)
  buf[:stats.numel()] = stats.reshape(-1).to(torch.float32)
  out = [torch.zeros_like(buf) for _ in range(dist.get_world_size())]
  dist.all_gather(out, buf)
  return torch.stack(out)
