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


def sum_over_ranks(values, device: torch.device | str = "cpu") -> list[float]:
  """Element-wise sum of a short host vector over ranks (e.g. per-rank event counts)."""
  vals = [float(v) for v in values]
  if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
    return vals
  t = torch.tensor(vals, dtype=torch.float64, device=device)
  dist.all_reduce(t, op=dist.ReduceOp.SUM)
  return [float(v) for v in t.tolist()]


def gather_stats(stats: torch.Tensor, capacity: int | None = None) -> torch.Tensor:
  """All-gather a packed fp32 statistics vector: [world_size, capacity] on every rank.
  Each rank's vector is zero-padded to `capacity` (default: its own length, which must then
  be equal on every rank).  No host synchronisation: the lengths are fixed by the caller."""
  cap = stats.numel() if capacity is None else int(capacity)
  if stats.numel() > cap:
    raise ValueError(f"stats vector of {stats.numel()} values exceeds capacity {cap}")
  buf = torch.zeros(cap, dtype=torch.float32, device=stats.device)
  buf[:stats.numel()] = stats.reshape(-1).to(torch.float32)
  if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
    return buf.reshape(1, -1)
  out = [torch.zeros_like(buf) for _ in range(dist.get_world_size())]
  dist.all_gather(out, buf)
  return torch.stack(out)


class StatsGather:
  """Episode-statistics all-gather off the critical path: a
  fixed-capacity fp32 send buffer and per-rank receive buffers allocated once; `start`
  packs the values on a side stream and issues an asynchronous all-gather (RCCL on the GPU,
  gloo on CPU); `wait` returns the [world_size, capacity] result after making the caller's
  stream wait for it.  Nothing reads back to the host, so a runner can start the gather
  after its rollout and collect it after the PPO update."""

  def __init__(self, capacity: int, device: torch.device | str = "cpu") -> None:
    self.capacity = int(capacity)
    self.device = torch.device(device)
    self.active = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    self.world = dist.get_world_size() if self.active else 1
    self.send = torch.zeros(self.capacity, dtype=torch.float32, device=self.device)
    self.recv = [torch.zeros_like(self.send) for _ in range(self.world)]
    self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
    self._work = None

  def start(self, values: torch.Tensor) -> None:
    if values.numel() > self.capacity:
      raise ValueError(f"{values.numel()} statistics exceed the capacity {self.capacity}")
    cur = torch.cuda.current_stream(self.device) if self.stream is not None else None
    ctx = torch.cuda.stream(self.stream) if self.stream is not None else _null()
    if self.stream is not None:
      self.stream.wait_stream(cur)
    with ctx:
      self.send.zero_()
      self.send[:values.numel()].copy_(values.reshape(-1).to(torch.float32))
      if self.active:
        self._work = dist.all_gather(self.recv, self.send, async_op=True)
      else:
        self.recv[0].copy_(self.send)
    if self.stream is not None:
      values.record_stream(self.stream)

  def wait(self) -> torch.Tensor:
    if self._work is not None:
      self._work.wait()
      self._work = None
    if self.stream is not None:
      torch.cuda.current_stream(self.device).wait_stream(self.stream)
    return torch.stack(self.recv)


class _null:
  def __enter__(self):
    return self

  def __exit__(self, *a):
    return False
