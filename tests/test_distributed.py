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

  def __init__(self, n, rank):
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
    return self.obs, r, torch.ones(self.num_envs, dtype=torch.long), {"time_outs": torch.zeros(self.num_envs)}


def _runner_worker(rank, world, port, q):
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
    env = _ToyEnv(32 * (rank + 1), rank)  # different env counts: episode-weighted means
    runner = OnPolicyRunner(env, cfg, device="cpu")
    hist = runner.learn(2)
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
