"""The learner side (mjlab_amd/rl, restating rsl-rl-lib 3.1.0 as the reference trains with
it, `src/mjlab/rl/*`): GAE against a plain-numpy restatement, the running observation
normaliser against batch statistics, rsl_rl's adaptive learning-rate rule, a PPO run that
learns a toy task on CPU, and the world-size-2 gradient all-reduce (gloo).  rsl_rl itself is
not installed here: parity with it is by formula restatement (parity unpinned)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from mjlab_amd.rl import PPO, ActorCritic, EmpiricalNormalization, OnPolicyRunner, RslRlOnPolicyRunnerCfg
from mjlab_amd.rl.config import RslRlPpoActorCriticCfg, RslRlPpoAlgorithmCfg, load_rl_cfg
from mjlab_amd.rl.ppo import RolloutStorage


def _gae_numpy(rew, val, done, last, gamma, lam):
  T = rew.shape[0]
  ret = np.zeros_like(rew)
  adv = 0.0
  for t in reversed(range(T)):
    nv = last if t == T - 1 else val[t + 1]
    nt = 1.0 - done[t]
    delta = rew[t] + nt * gamma * nv - val[t]
    adv = delta + nt * gamma * lam * adv
    ret[t] = adv + val[t]
  return ret


def test_gae_matches_numpy():
  rng = np.random.default_rng(0)
  T, N = 24, 16
  obs = {"policy": torch.zeros(N, 3), "critic": torch.zeros(N, 5)}
  s = RolloutStorage(N, T, obs, 2, "cpu")
  rew = rng.normal(size=(T, N, 1)).astype(np.float32)
  val = rng.normal(size=(T, N, 1)).astype(np.float32)
  done = (rng.random((T, N, 1)) < 0.1).astype(np.float32)
  last = rng.normal(size=(N, 1)).astype(np.float32)
  s.rewards[:] = torch.from_numpy(rew)
  s.values[:] = torch.from_numpy(val)
  s.dones[:] = torch.from_numpy(done)
  s.compute_returns(torch.from_numpy(last), 0.99, 0.95, normalize_advantage=False)
  ref = _gae_numpy(rew, val, done, last, 0.99, 0.95)
  np.testing.assert_allclose(s.returns.numpy(), ref, rtol=1e-5, atol=1e-5)
  np.testing.assert_allclose(s.advantages.numpy(), ref - val, rtol=1e-5, atol=1e-5)
  s.compute_returns(torch.from_numpy(last), 0.99, 0.95, normalize_advantage=True)
  a = s.advantages.numpy()
  assert abs(a.mean()) < 1e-5 and abs(a.std(ddof=1) - 1.0) < 1e-4


def test_empirical_normalization_tracks_all_samples():
  torch.manual_seed(0)
  n = EmpiricalNormalization(4)
  n.train()
  xs = [torch.randn(37, 4) * torch.tensor([1.0, 2.0, 0.5, 3.0]) + torch.tensor([0.0, 1.0, -2.0, 5.0])
        for _ in range(6)]
  for x in xs:
    n.update(x)
  allx = torch.cat(xs).double()
  torch.testing.assert_close(n.mean.double(), allx.mean(0), rtol=1e-5, atol=1e-5)
  torch.testing.assert_close(n.std.double(), allx.std(0, unbiased=False), rtol=1e-4, atol=1e-5)
  y = n(xs[0])
  torch.testing.assert_close(y, (xs[0] - n.mean) / (n.std + 1e-2))
  n.eval()
  c = int(n.count)
  n.update(xs[0])  # eval mode: frozen
  assert int(n.count) == c


def test_adaptive_learning_rate_rule():
  f = PPO._adapt_lr
  assert f(0.05, 1e-3, 0.01) == pytest.approx(1e-3 / 1.5)   # kl > 2 * desired
  assert f(0.001, 1e-3, 0.01) == pytest.approx(1.5e-3)      # 0 < kl < desired / 2
  assert f(0.0, 1e-3, 0.01) == 1e-3                         # kl == 0: unchanged
  assert f(0.01, 1e-3, 0.01) == 1e-3                        # in band
  assert f(1.0, 1.2e-5, 0.01) == 1e-5                       # floor
  assert f(1e-4, 9e-3, 0.01) == 1e-2                        # ceiling


def test_task_rl_configs_follow_the_reference():
  g1 = load_rl_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  assert g1.policy.actor_hidden_dims == (512, 256, 128) and g1.policy.actor_obs_normalization
  assert (g1.algorithm.entropy_coef, g1.algorithm.learning_rate, g1.num_steps_per_env) == (0.01, 1e-3, 24)
  go1 = load_rl_cfg("Mjlab-Velocity-Flat-Unitree-Go1")
  assert not go1.policy.actor_obs_normalization and go1.max_iterations == 10_000
  jump = load_rl_cfg("Mjlab-Jump-Flat-Unitree-G1")
  assert jump.policy.actor_hidden_dims == (256, 128, 64) and jump.algorithm.gamma == 0.98
  assert jump.algorithm.num_learning_epochs == 6 and jump.algorithm.value_loss_coef == 2.0


class _ReachEnv:
  """Toy vectorised task (one-step episodes): act = target.  Reward -|a - target|^2."""

  def __init__(self, n, seed=0):
    self.num_envs, self.num_actions, self.device = n, 2, torch.device("cpu")
    self.max_episode_length = 1
    self.episode_length_buf = torch.zeros(n, dtype=torch.long)
    self.g = torch.Generator().manual_seed(seed)
    self._new()
    self.unwrapped = self

  def _new(self):
    self.target = 2 * torch.rand(self.num_envs, 2, generator=self.g) - 1
    self.obs = {"policy": self.target.clone(), "critic": self.target.clone()}

  def get_observations(self):
    return self.obs

  def step(self, a):
    r = -((a - self.target) ** 2).sum(-1)
    self._new()
    return self.obs, r, torch.ones(self.num_envs, dtype=torch.long), {"time_outs": torch.zeros(self.num_envs)}


def test_ppo_learns_a_toy_task():
  torch.manual_seed(0)
  cfg = RslRlOnPolicyRunnerCfg(
    policy=RslRlPpoActorCriticCfg(init_noise_std=0.5, actor_hidden_dims=(32, 32),
                                  critic_hidden_dims=(32, 32), actor_obs_normalization=True,
                                  critic_obs_normalization=True),
    algorithm=RslRlPpoAlgorithmCfg(learning_rate=3e-3, entropy_coef=0.0),
    num_steps_per_env=8)
  env = _ReachEnv(256)
  runner = OnPolicyRunner(env, cfg, device="cpu")
  hist = runner.learn(40)
  first, last = hist[0]["mean_reward"], np.mean([h["mean_reward"] for h in hist[-5:]])
  assert first < -0.5 and last > 0.5 * first  # error at least halved
  assert all(np.isfinite(h["value_function"]) and np.isfinite(h["surrogate"]) for h in hist)
  assert runner.tot_timesteps == 40 * 8 * 256


def _free_port():
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _grad_worker(rank, world, port, q):
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                    RANK=str(rank), LOCAL_RANK=str(rank))
  import torch.distributed as dist
  dist.init_process_group("gloo")
  try:
    torch.manual_seed(100 + rank)  # different init per rank: broadcast must equalise it
    obs = {"policy": torch.zeros(4, 3), "critic": torch.zeros(4, 3)}
    pol = ActorCritic(obs, {"policy": ("policy",), "critic": ("critic",)}, 2, actor_hidden_dims=(8,),
                      critic_hidden_dims=(8,))
    alg = PPO(pol, multi_gpu=True)
    alg.broadcast_parameters()
    x = torch.full((4, 3), float(rank + 1))
    loss = alg.policy.actor(x).sum() + alg.policy.critic(x).sum()
    loss.backward()
    local = [p.grad.clone() for p in alg.policy.parameters() if p.grad is not None]
    alg.reduce_parameters()
    red = [p.grad.clone() for p in alg.policy.parameters() if p.grad is not None]
    q.put((rank, [t.tolist() for t in local], [t.tolist() for t in red],
           [p.detach().tolist() for p in alg.policy.parameters()]))
  finally:
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_gradient_all_reduce():
  world, port = 2, _free_port()
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  procs = [ctx.Process(target=_grad_worker, args=(r, world, port, q)) for r in range(world)]
  for p in procs:
    p.start()
  res = sorted(q.get(timeout=90) for _ in range(world))
  for p in procs:
    p.join(timeout=30)
    assert p.exitcode == 0
  (_, l0, r0, p0), (_, l1, r1, p1) = res
  for a, b in zip(p0, p1):  # rank 0's parameters everywhere
    np.testing.assert_array_equal(np.array(a), np.array(b))
  for a, b, c, d in zip(l0, l1, r0, r1):
    mean = (np.array(a) + np.array(b)) / 2
    np.testing.assert_allclose(np.array(c), mean, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(np.array(d), mean, rtol=1e-6, atol=1e-6)
