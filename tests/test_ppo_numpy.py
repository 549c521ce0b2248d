"""One PPO iteration of `mjlab_amd.rl.PPO` against a numpy restatement of rsl-rl-lib
3.1.0's update (the reference's learner, `uv.lock:2532-2547`, configured by
`src/mjlab/tasks/velocity/config/g1/rl_cfg.py:10-39`; the library itself is not installed).

The numpy side shares no code with the torch side: hand-written forward and backward
passes of the ELU MLPs and of the Gaussian policy, the clipped surrogate and clipped value
losses with their sub-gradients, the entropy bonus, the KL-adaptive learning rate applied
before each optimizer step, global-norm gradient clipping (`clip_grad_norm_`: coefficient
max_norm / (norm + 1e-6), clamped at 1) and Adam with PyTorch's bias correction.  Both run
in float64 from the same initial weights, rollout data and mini-batch permutation; after
the iteration every parameter, the learning rate and the logged losses must agree to
float64 rounding.  Parity here is by restatement of the published algorithm (rsl_rl's
source is absent): what it pins is that the torch learner computes that algorithm.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from mjlab_amd.rl.ppo import PPO, ActorCritic

NA_OBS, NC_OBS, NACT = 5, 7, 3
HID = (8, 6)
T, N = 6, 4
EPOCHS, MB = 3, 2


def _elu(z):
  return np.where(z > 0, z, np.expm1(np.minimum(z, 0.0)))


def _delu(z):
  return np.where(z > 0, 1.0, np.exp(np.minimum(z, 0.0)))


def _mlp_fwd(layers, x):
  acts, zs = [x], []
  h = x
  for i, (W, b) in enumerate(layers):
    z = h @ W.T + b
    zs.append(z)
    h = _elu(z) if i < len(layers) - 1 else z
    acts.append(h)
  return h, (acts, zs)


def _mlp_bwd(layers, cache, gout):
  acts, zs = cache
  grads = [None] * len(layers)
  g = gout
  for i in reversed(range(len(layers))):
    W, _ = layers[i]
    if i < len(layers) - 1:
      g = g * _delu(zs[i])
    grads[i] = (g.T @ acts[i], g.sum(0))
    g = g @ W
  return grads


def _layers(seq):
  lin = [m for m in seq if isinstance(m, torch.nn.Linear)]
  return [(m.weight.detach().numpy().copy(), m.bias.detach().numpy().copy()) for m in lin]


class NumpyPPO:
  """rsl_rl 3.1.0 PPO.update for an MLP ActorCritic with a scalar-type std."""

  def __init__(self, policy: ActorCritic, cfg: dict, norm_a, norm_c):
    self.actor = _layers(policy.actor)
    self.critic = _layers(policy.critic)
    self.std = policy.std.detach().numpy().copy()
    self.cfg = cfg
    self.lr = cfg["learning_rate"]
    self.norm_a, self.norm_c = norm_a, norm_c  # (mean, std, eps): fixed during the update
    self.t = 0
    self.m = self._zeros()
    self.v = self._zeros()

  def _params(self):
    out = []
    for W, b in self.actor + self.critic:
      out += [W, b]
    return out + [self.std]

  def _zeros(self):
    return [np.zeros_like(p) for p in self._params()]

  def _norm(self, x, nm):
    mean, std, eps = nm
    return (x - mean) / (std + eps)

  def step(self, obs_a, obs_c, act, target_v, adv, ret, old_logp, old_mu, old_sigma):
    c = self.cfg
    B = act.shape[0]
    xa, xc = self._norm(obs_a, self.norm_a), self._norm(obs_c, self.norm_c)
    mu, acache = _mlp_fwd(self.actor, xa)
    value, ccache = _mlp_fwd(self.critic, xc)
    value = value[:, 0]
    sig = np.broadcast_to(self.std, mu.shape)
    logp = np.sum(-((act - mu) ** 2) / (2 * sig ** 2) - np.log(sig) - 0.5 * np.log(2 * np.pi), axis=1)
    ent = np.sum(0.5 + 0.5 * np.log(2 * np.pi) + np.log(sig), axis=1)
    # adaptive learning rate from the KL to the rollout-time policy (before the step)
    kl = np.sum(np.log(sig / old_sigma + 1e-5) + (old_sigma ** 2 + (old_mu - mu) ** 2) / (2 * sig ** 2) - 0.5,
                axis=1).mean()
    if kl > c["desired_kl"] * 2.0:
      self.lr = max(1e-5, self.lr / 1.5)
    elif 0.0 < kl < c["desired_kl"] / 2.0:
      self.lr = min(1e-2, self.lr * 1.5)
    # clipped surrogate
    ratio = np.exp(logp - old_logp)
    eps_c = c["clip_param"]
    rc = np.clip(ratio, 1 - eps_c, 1 + eps_c)
    s1, s2 = -adv * ratio, -adv * rc
    surr = np.maximum(s1, s2).mean()
    inside = (ratio > 1 - eps_c) & (ratio < 1 + eps_c)
    d_ratio = np.where(s1 >= s2, -adv, np.where(inside, -adv, 0.0)) / B
    d_logp = d_ratio * ratio
    # clipped value loss
    vc = target_v + np.clip(value - target_v, -eps_c, eps_c)
    l1, l2 = (value - ret) ** 2, (vc - ret) ** 2
    vloss = np.maximum(l1, l2).mean()
    vin = np.abs(value - target_v) < eps_c
    d_value = np.where(l1 >= l2, 2 * (value - ret), np.where(vin, 2 * (vc - ret), 0.0)) / B
    d_value *= c["value_loss_coef"]
    loss_ent = ent.mean()
    # policy gradients: logp and entropy through mu and the std parameter
    d_mu = d_logp[:, None] * (act - mu) / sig ** 2
    d_sig = d_logp[:, None] * ((act - mu) ** 2 / sig ** 3 - 1.0 / sig)
    d_std = d_sig.sum(0) - c["entropy_coef"] * (1.0 / self.std)
    ga = _mlp_bwd(self.actor, acache, d_mu)
    gc = _mlp_bwd(self.critic, ccache, d_value[:, None])
    grads = []
    for gW, gb in ga + gc:
      grads += [gW, gb]
    grads.append(d_std)
    # clip_grad_norm_
    total = np.sqrt(sum(float(np.sum(g * g)) for g in grads))
    coef = min(1.0, c["max_grad_norm"] / (total + 1e-6))
    grads = [g * coef for g in grads]
    # Adam (torch defaults: betas 0.9 / 0.999, eps 1e-8)
    self.t += 1
    b1, b2, eps = 0.9, 0.999, 1e-8
    bc1, bc2 = 1 - b1 ** self.t, 1 - b2 ** self.t
    params = self._params()
    for i, (p, g) in enumerate(zip(params, grads)):
      self.m[i] = b1 * self.m[i] + (1 - b1) * g
      self.v[i] = b2 * self.v[i] + (1 - b2) * g * g
      denom = np.sqrt(self.v[i]) / np.sqrt(bc2) + eps
      p -= (self.lr / bc1) * self.m[i] / denom
    return vloss, surr, loss_ent


@pytest.mark.parametrize("seed", [0, 1])
def test_one_ppo_iteration_matches_numpy(seed):
  prev = torch.get_default_dtype()
  torch.set_default_dtype(torch.float64)
  try:
    torch.manual_seed(seed)
    rng = np.random.default_rng(seed)
    obs0 = {"policy": torch.zeros(N, NA_OBS), "critic": torch.zeros(N, NC_OBS)}
    policy = ActorCritic(obs0, {"policy": ["policy"], "critic": ["critic"]}, NACT,
                         actor_obs_normalization=True, critic_obs_normalization=True,
                         actor_hidden_dims=HID, critic_hidden_dims=HID, activation="elu",
                         init_noise_std=0.8)
    cfg = dict(num_learning_epochs=EPOCHS, num_mini_batches=MB, clip_param=0.2, gamma=0.99, lam=0.95,
               value_loss_coef=1.0, entropy_coef=0.01, learning_rate=1e-3, max_grad_norm=1.0,
               use_clipped_value_loss=True, schedule="adaptive", desired_kl=0.01)
    ppo = PPO(policy, device="cpu", **cfg)
    ppo.graph_act = False
    ppo.init_storage(N, T, obs0, NACT)
    # a rollout: the policy acts on random observations (normalisers updated as in
    # process_env_step), random rewards, some dones and time-outs
    for _ in range(T):
      obs = {"policy": torch.as_tensor(rng.normal(0, 2, (N, NA_OBS))),
             "critic": torch.as_tensor(rng.normal(1, 1.5, (N, NC_OBS)))}
      ppo.act(obs)
      rew = torch.as_tensor(rng.normal(0, 1, N))
      dones = torch.as_tensor(rng.random(N) < 0.2)
      ppo.process_env_step(obs, rew, dones, {"time_outs": torch.as_tensor(rng.random(N) < 0.1)})
    last = {"policy": torch.as_tensor(rng.normal(0, 2, (N, NA_OBS))),
            "critic": torch.as_tensor(rng.normal(1, 1.5, (N, NC_OBS)))}
    ppo.compute_returns(last)
    s = ppo.storage
    nm = lambda n: (n._mean.numpy().copy(), n._std.numpy().copy(), n.eps)
    ref = NumpyPPO(policy, cfg, nm(policy.actor_obs_normalizer), nm(policy.critic_obs_normalizer))
    flat = lambda t: t.detach().flatten(0, 1).numpy().copy()
    data = dict(oa=flat(s.observations["policy"]), oc=flat(s.observations["critic"]), act=flat(s.actions),
                tv=flat(s.values)[:, 0], adv=flat(s.advantages)[:, 0], ret=flat(s.returns)[:, 0],
                logp=flat(s.actions_log_prob)[:, 0], mu=flat(s.mu), sig=flat(s.sigma))
    # the mini-batch permutation update() draws first (one randperm for all epochs)
    torch.manual_seed(1000 + seed)
    mb = T * N // MB
    idx = torch.randperm(MB * mb).numpy()
    torch.manual_seed(1000 + seed)
    out = ppo.update()
    losses = []
    for _ in range(EPOCHS):
      for i in range(MB):
        b = idx[i * mb:(i + 1) * mb]
        losses.append(ref.step(data["oa"][b], data["oc"][b], data["act"][b], data["tv"][b], data["adv"][b],
                               data["ret"][b], data["logp"][b], data["mu"][b], data["sig"][b]))
    lv, ls, le = np.mean(np.array(losses), axis=0)
    assert out["value_function"] == pytest.approx(lv, rel=1e-10, abs=1e-12)
    assert out["surrogate"] == pytest.approx(ls, rel=1e-10, abs=1e-12)
    assert out["entropy"] == pytest.approx(le, rel=1e-10, abs=1e-12)
    assert ppo.learning_rate == pytest.approx(ref.lr, rel=1e-12)
    for (W, b), (Wr, br) in zip(_layers(policy.actor) + _layers(policy.critic), ref.actor + ref.critic):
      np.testing.assert_allclose(W, Wr, rtol=0, atol=1e-11)
      np.testing.assert_allclose(b, br, rtol=0, atol=1e-11)
    np.testing.assert_allclose(policy.std.detach().numpy(), ref.std, rtol=0, atol=1e-11)
    # and the update moved the parameters (the comparison is not of two untouched copies)
    assert ref.t == EPOCHS * MB
  finally:
    torch.set_default_dtype(prev)
