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
    g = d.gather_stats(stats, capacity=3)
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
  g = d.StatsGather(4)
  g.start(torch.tensor([1.0, 2.0]))
  assert g.wait().tolist() == [[1.0, 2.0, 0.0, 0.0]]


class _ToyEnv:
  """Vectorised one-step task (act = target), with an extras["log"] entry that differs per
  rank, for the runner's cross-rank statistics path."""

  def __init__(self, n, rank, ragged_keys=False):
    self.ragged_keys = ragged_keys
    self.num_envs, self.num_actions, self.device = n, 2, torch.device("cpu")
    self.max_episode_length = 1
    self.episode_length_buf = torch.zeros(n, dtype=torch.long)
    self.g = torch.Generator().manual_seed(rank)
    self.rank = rank
    self.extras = {"log": {"Episode_Termination/time_out": torch.tensor(float(rank + 1)),
                           "Metrics/constant": 5.0}}
    self.unwrapped = self
    self._new()

  def _new(self):
    self.target = 2 * torch.rand(self.num_envs, 2, generator=self.g) - 1
    self.obs = {"policy": self.target.clone(), "critic": self.target.clone()}

  def get_observations(self):
    return self.obs

  def step(self, a):
    r = -((a - self.target) ** 2).sum(-1) + 10.0 * self.rank
    self._new()
    self.calls = getattr(self, "calls", 0) + 1
    if self.ragged_keys:
      # the ranks' key sets differ: one key only rank 0 holds, and one that rank 1 starts
      # reporting after the first iteration (4 env steps)
      if self.rank == 0:
        self.extras["log"]["Metrics/only_rank0"] = 3.0
      elif self.calls > 4:
        self.extras["log"]["Metrics/late_rank1"] = torch.tensor(7.0)
    return self.obs, r, torch.ones(self.num_envs, dtype=torch.long), {"time_outs": torch.zeros(self.num_envs)}


def _runner_worker(rank, world, port, q, ragged_keys=False):
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                    RANK=str(rank), LOCAL_RANK=str(rank))
  from mjlab_amd import distributed as d
  from mjlab_amd.rl import OnPolicyRunner, RslRlOnPolicyRunnerCfg, RslRlPpoActorCriticCfg, RslRlPpoAlgorithmCfg
  d.init("gloo")
  try:
    torch.manual_seed(0)
    cfg = RslRlOnPolicyRunnerCfg(
      policy=RslRlPpoActorCriticCfg(actor_hidden_dims=(8,), critic_hidden_dims=(8,)),
      algorithm=RslRlPpoAlgorithmCfg(), num_steps_per_env=4)
    env = _ToyEnv(32 * (rank + 1), rank, ragged_keys)  # different env counts: episode-weighted means
    runner = OnPolicyRunner(env, cfg, device="cpu")
    hist = runner.learn(3 if ragged_keys else 2)
    q.put((rank, hist))
  finally:
    import torch.distributed as dist
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_two_rank_runner_stats_gather():
  """rl/runner.py gathers each rollout's episode statistics and extras["log"] across ranks
  (StatsGather, asynchronous, overlapped with the update); rank 0 logs the world values."""
  world, port = 2, _free_port()
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  procs = [ctx.Process(target=_runner_worker, args=(r, world, port, q)) for r in range(world)]
  for p in procs:
    p.start()
  res = dict(q.get(timeout=150) for _ in range(world))
  for p in procs:
    p.join(timeout=30)
    assert p.exitcode == 0
  h0, h1 = res[0], res[1]
  assert all("world/mean_reward" not in r for r in h1)  # only rank 0 logs world values
  for r0, r1 in zip(h0, h1):
    n0, n1 = r0["episodes"], r1["episodes"]
    assert r0["world/episodes"] == n0 + n1
    want = (r0["mean_reward"] * n0 + r1["mean_reward"] * n1) / (n0 + n1)
    assert abs(r0["world/mean_reward"] - want) < 1e-4 * max(1.0, abs(want))
    assert r0["world/Episode_Termination/time_out"] == 1.5   # (1 + 2) / 2
    assert r0["world/Metrics/constant"] == 5.0


@pytest.mark.timeout(180)
def test_two_rank_runner_ragged_log_keys():
  """ranks whose extras["log"] key sets differ (and keys that first appear after
  the first iteration) must still gather into one layout: the union of keys, agreed every
  iteration, with per-key presence so a missing key is not averaged as zero."""
  world, port = 2, _free_port()
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  procs = [ctx.Process(target=_runner_worker, args=(r, world, port, q, True)) for r in range(world)]
  for p in procs:
    p.start()
  res = dict(q.get(timeout=150) for _ in range(world))
  for p in procs:
    p.join(timeout=30)
    assert p.exitcode == 0
  h0 = res[0]
  assert len(h0) == 3
  for it, r0 in enumerate(h0):
    assert r0["world/Episode_Termination/time_out"] == 1.5
    assert r0["world/Metrics/only_rank0"] == 3.0  # rank 0's value, not (3 + 0) / 2
    if it == 0:
      assert "world/Metrics/late_rank1" not in r0
    else:
      assert r0["world/Metrics/late_rank1"] == 7.0


def _bench_worker(rank, world, port, q):
  """bench.py's rank logic on a CPU stand-in (gloo): per-rank seed, MAX of the elapsed
  time, SUM of the dropped-contact events, the packed episode-statistics all-gather."""
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                    RANK=str(rank), LOCAL_RANK=str(rank))
  import sys
  sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
  import bench
  from mjlab_amd import distributed as d
  d.init("gloo")
  try:
    seed = d.rank_seed(42, rank)
    el, dropped, g = bench.reduce_over_ranks(1.0 + 0.5 * rank, [rank, 0, 2 * rank],
                                             torch.tensor([float(seed), 1.0 + rank]), "cpu")
    q.put((rank, seed, el, dropped, g.tolist()))
  finally:
    import torch.distributed as dist
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_bench_reduction():
  world, port = 2, _free_port()
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
  for p in procs:
    p.start()
  res = sorted(q.get(timeout=90) for _ in range(world))
  for p in procs:
    p.join(timeout=30)
    assert p.exitcode == 0
  for rank, seed, el, dropped, g in res:
    assert seed == 42 + rank
    assert el == 1.5                      # the slowest rank's time
    assert dropped == [1, 0, 2]           # summed: every rank exits the same way
    assert g == [[42.0, 1.0], [43.0, 2.0]]


def test_bench_refuses_gpus_world_mismatch():
  """`--gpus N` must match the launcher's WORLD_SIZE (checked before any GPU call)."""
  import subprocess
  import sys
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
  r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "1"], env=env,
                     capture_output=True, text=True, timeout=120)
  assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr
