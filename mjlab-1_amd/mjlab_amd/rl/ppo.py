"""PPO learner restating rsl-rl-lib 3.1.0 (the reference's pinned dependency,
`uv.lock:2532-2547`; used through `src/mjlab/rl/*` and `scripts/train.py`), which is not
present here: same networks, normalisation, storage, GAE, clipped losses, adaptive learning
rate and multi-GPU reductions.

Differences that matter on MI355X, none of which changes the arithmetic:
  - observations are written into the rollout storage when the policy acts, because the
    graph-captured env step returns the same output tensors every step;
  - episode bookkeeping stays on the device (sums and counts of finished episodes), with
    one host read per iteration for logging, instead of a `nonzero` + host copy per step;
  - gradients are all-reduced as one flat fp32 bucket over RCCL (backend "nccl").
"""

from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn
from torch.distributions import Normal

_ACT = {"elu": nn.ELU, "relu": nn.ReLU, "selu": nn.SELU, "tanh": nn.Tanh, "lrelu": nn.LeakyReLU,
        "sigmoid": nn.Sigmoid, "softplus": nn.Softplus, "gelu": nn.GELU, "silu": nn.SiLU}


def mlp(input_dim: int, output_dim: int, hidden_dims, activation: str) -> nn.Sequential:
  """rsl_rl.networks.MLP: Linear + activation per hidden layer, linear output."""
  layers, d = [], input_dim
  for h in hidden_dims:
    layers += [nn.Linear(d, h), _ACT[activation.lower()]()]
    d = h
  layers.append(nn.Linear(d, output_dim))
  return nn.Sequential(*layers)


class EmpiricalNormalization(nn.Module):
  """rsl_rl.modules.normalizer.EmpiricalNormalization: running mean / variance over every
  sample seen (training mode only), y = (x - mean) / (std + eps)."""

  def __init__(self, shape: int, eps: float = 1e-2, until: int | None = None):
    super().__init__()
    self.eps, self.until = eps, until
    self.register_buffer("_mean", torch.zeros(shape).unsqueeze(0))
    self.register_buffer("_var", torch.ones(shape).unsqueeze(0))
    self.register_buffer("_std", torch.ones(shape).unsqueeze(0))
    self.register_buffer("count", torch.tensor(0, dtype=torch.long))

  @property
  def mean(self):
    return self._mean.squeeze(0).clone()

  @property
  def std(self):
    return self._std.squeeze(0).clone()

  def forward(self, x: torch.Tensor) -> torch.Tensor:
    return (x - self._mean) / (self._std + self.eps)

  @torch.jit.unused
  def update(self, x: torch.Tensor) -> None:
    if not self.training:
      return
    if self.until is not None and int(self.count) >= self.until:
      return
    n = x.shape[0]
    self.count += n
    rate = n / self.count
    var_x = torch.var(x, dim=0, unbiased=False, keepdim=True)
    mean_x = torch.mean(x, dim=0, keepdim=True)
    delta = mean_x - self._mean
    self._mean += rate * delta
    self._var += rate * (var_x - self._var + delta * (mean_x - self._mean))
    self._std.copy_(torch.sqrt(self._var))


class ActorCritic(nn.Module):
  """rsl_rl.modules.ActorCritic (3.x): Gaussian policy with a state-independent std."""

  is_recurrent = False

  def __init__(self, obs: dict, obs_groups: dict, num_actions: int,
               actor_obs_normalization=False, critic_obs_normalization=False,
               actor_hidden_dims=(256, 256, 256), critic_hidden_dims=(256, 256, 256),
               activation="elu", init_noise_std=1.0, noise_std_type="scalar", **_):
    super().__init__()
    self.obs_groups = obs_groups
    na = sum(obs[g].shape[-1] for g in obs_groups["policy"])
    nc = sum(obs[g].shape[-1] for g in obs_groups["critic"])
    self.actor = mlp(na, num_actions, actor_hidden_dims, activation)
    self.critic = mlp(nc, 1, critic_hidden_dims, activation)
    self.actor_obs_normalization = actor_obs_normalization
    self.critic_obs_normalization = critic_obs_normalization
    self.actor_obs_normalizer = EmpiricalNormalization(na) if actor_obs_normalization else nn.Identity()
    self.critic_obs_normalizer = EmpiricalNormalization(nc) if critic_obs_normalization else nn.Identity()
    self.noise_std_type = noise_std_type
    if noise_std_type == "scalar":
      self.std = nn.Parameter(init_noise_std * torch.ones(num_actions))
    elif noise_std_type == "log":
      self.log_std = nn.Parameter(torch.log(init_noise_std * torch.ones(num_actions)))
    else:
      raise ValueError(f"unknown noise_std_type {noise_std_type!r}")
    self.distribution = None
    Normal.set_default_validate_args(False)

  def reset(self, dones=None):
    pass

  def get_actor_obs(self, obs: dict) -> torch.Tensor:
    return torch.cat([obs[g] for g in self.obs_groups["policy"]], dim=-1)

  def get_critic_obs(self, obs: dict) -> torch.Tensor:
    return torch.cat([obs[g] for g in self.obs_groups["critic"]], dim=-1)

  @property
  def action_mean(self):
    return self.distribution.mean

  @property
  def action_std(self):
    return self.distribution.stddev

  @property
  def entropy(self):
    return self.distribution.entropy().sum(dim=-1)

  def _update_distribution(self, x: torch.Tensor) -> None:
    mean = self.actor(x)
    std = self.std.expand_as(mean) if self.noise_std_type == "scalar" else torch.exp(self.log_std).expand_as(mean)
    self.distribution = Normal(mean, std)

  def act(self, obs: dict, sample: bool = True) -> torch.Tensor | None:
    self._update_distribution(self.actor_obs_normalizer(self.get_actor_obs(obs)))
    return self.distribution.sample() if sample else None

  def act_inference(self, obs: dict) -> torch.Tensor:
    return self.actor(self.actor_obs_normalizer(self.get_actor_obs(obs)))

  def evaluate(self, obs: dict) -> torch.Tensor:
    return self.critic(self.critic_obs_normalizer(self.get_critic_obs(obs)))

  def get_actions_log_prob(self, actions: torch.Tensor) -> torch.Tensor:
    return self.distribution.log_prob(actions).sum(dim=-1)

  def update_normalization(self, obs: dict) -> None:
    if self.actor_obs_normalization:
      self.actor_obs_normalizer.update(self.get_actor_obs(obs))
    if self.critic_obs_normalization:
      self.critic_obs_normalizer.update(self.get_critic_obs(obs))


class RolloutStorage:
  """rsl_rl.storage.RolloutStorage ("rl" training type), observation groups as a dict."""

  def __init__(self, num_envs: int, num_transitions: int, obs: dict, num_actions: int, device):
    T, N = num_transitions, num_envs
    self.T, self.N, self.device = T, N, device
    self.observations = {k: torch.zeros(T, N, *v.shape[1:], device=device) for k, v in obs.items()}
    z = lambda *s: torch.zeros(T, N, *s, device=device)
    self.actions, self.rewards, self.dones = z(num_actions), z(1), z(1)
    self.values, self.actions_log_prob = z(1), z(1)
    self.mu, self.sigma = z(num_actions), z(num_actions)
    self.returns, self.advantages = z(1), z(1)
    self.step = 0

  def clear(self):
    self.step = 0

  def compute_returns(self, last_values, gamma, lam, normalize_advantage: bool = True):
    advantage = 0
    for step in reversed(range(self.T)):
      next_values = last_values if step == self.T - 1 else self.values[step + 1]
      not_terminal = 1.0 - self.dones[step].float()
      delta = self.rewards[step] + not_terminal * gamma * next_values - self.values[step]
      advantage = delta + not_terminal * gamma * lam * advantage
      self.returns[step] = advantage + self.values[step]
    self.advantages = self.returns - self.values
    if normalize_advantage:
      self.advantages = (self.advantages - self.advantages.mean()) / (self.advantages.std() + 1e-8)

  def mini_batch_generator(self, num_mini_batches: int, num_epochs: int):
    batch = self.T * self.N
    mb = batch // num_mini_batches
    flat = lambda t: t.flatten(0, 1)
    obs = {k: flat(v) for k, v in self.observations.items()}
    actions, values, returns = flat(self.actions), flat(self.values), flat(self.returns)
    logp, adv = flat(self.actions_log_prob), flat(self.advantages)
    mu, sigma = flat(self.mu), flat(self.sigma)
    # rsl_rl 3.1.0 RolloutStorage.mini_batch_generator: one permutation drawn before the
    # epoch loop, reused by every epoch
    idx = torch.randperm(num_mini_batches * mb, device=self.device)
    for _ in range(num_epochs):
      for i in range(num_mini_batches):
        b = idx[i * mb:(i + 1) * mb]
        yield ({k: v[b] for k, v in obs.items()}, actions[b], values[b], adv[b], returns[b],
               logp[b], mu[b], sigma[b])


class PPO:
  """rsl_rl.algorithms.PPO (3.1.0)."""

  def __init__(self, policy: ActorCritic, num_learning_epochs=5, num_mini_batches=4, clip_param=0.2,
               gamma=0.99, lam=0.95, value_loss_coef=1.0, entropy_coef=0.01, learning_rate=1e-3,
               max_grad_norm=1.0, use_clipped_value_loss=True, schedule="adaptive", desired_kl=0.01,
               device="cpu", normalize_advantage_per_mini_batch=False, multi_gpu=False, **_):
    self.device = device
    self.policy = policy.to(device)
    self.learning_rate = learning_rate
    # fused Adam on the GPU: one kernel per step instead of one per parameter tensor
    fused = torch.device(device).type == "cuda"
    self.optimizer = torch.optim.Adam(self.policy.parameters(), lr=learning_rate, fused=fused)
    self.clip_param, self.num_learning_epochs, self.num_mini_batches = clip_param, num_learning_epochs, num_mini_batches
    self.value_loss_coef, self.entropy_coef = value_loss_coef, entropy_coef
    self.gamma, self.lam, self.max_grad_norm = gamma, lam, max_grad_norm
    self.use_clipped_value_loss, self.schedule, self.desired_kl = use_clipped_value_loss, schedule, desired_kl
    self.normalize_advantage_per_mini_batch = normalize_advantage_per_mini_batch
    self.multi_gpu = multi_gpu and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    self.storage: RolloutStorage | None = None
    self.graph_act = True  # GPU: rollout-time policy evaluation as one graph replay
    self._act_graph = self._act_key = self._gobs = self._gout = None

  def init_storage(self, num_envs: int, num_transitions: int, obs: dict, num_actions: int):
    self.storage = RolloutStorage(num_envs, num_transitions, obs, num_actions, self.device)

  def _act_core(self, obs: dict, eps: torch.Tensor | None = None):
    if eps is None:
      actions = self.policy.act(obs).detach()
    else:  # reparameterised draw from given standard normals (the graphed path)
      self.policy.act(obs, sample=False)
      actions = (self.policy.action_mean + self.policy.action_std * eps).detach()
    return (actions, self.policy.evaluate(obs).detach(),
            self.policy.get_actions_log_prob(actions).detach().unsqueeze(-1),
            self.policy.action_mean.detach(), self.policy.action_std.detach())

  def act(self, obs: dict) -> torch.Tensor:
    s, t = self.storage, self.storage.step
    for k, v in obs.items():  # the env's graph outputs are overwritten by the next step
      s.observations[k][t].copy_(v)
    if self.graph_act and torch.device(self.device).type == "cuda":
      out = self._act_graphed(obs)
    else:
      out = self._act_core(obs)
    for dst, src in zip((s.actions, s.values, s.actions_log_prob, s.mu, s.sigma), out):
      dst[t].copy_(src)
    return out[0]

  def _act_graphed(self, obs: dict):
    """The rollout-time policy evaluation (actor + critic MLPs, action draw, log-prob) as
    one HIP graph replay on static input / output buffers: ~40 small launches per env step
    become one.  The standard normals are drawn outside the graph (one launch) and the
    action is mean + std * eps inside it -- the same distribution as Normal.sample().
    Re-recorded when the observation groups change shape."""
    key = tuple((k, tuple(v.shape)) for k, v in obs.items())
    if self._act_graph is None or self._act_key != key:
      self._record_act(obs, key)
    for k, v in obs.items():
      self._gobs[k].copy_(v)
    self._geps.normal_()
    self._act_graph.replay()
    return self._gout

  @torch.inference_mode(False)
  @torch.no_grad()
  def _record_act(self, obs: dict, key) -> None:
    # recorded outside inference mode: the first capture of a process registers the CUDA
    # generator's graph state tensors, and inference tensors there break every later
    # capture made outside inference mode (e.g. the env's own step graph)
    self._gobs = {k: v.detach().clone() for k, v in obs.items()}
    na = self.storage.actions.shape[-1]
    self._geps = torch.zeros(self.storage.N, na, device=self.device)
    side = torch.cuda.Stream(device=self.device)
    side.wait_stream(torch.cuda.current_stream(self.device))
    with torch.cuda.stream(side):
      for _ in range(2):  # warm-up (allocator, lazy init) before recording
        self._act_core(self._gobs, self._geps)
    torch.cuda.current_stream(self.device).wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
      self._gout = self._act_core(self._gobs, self._geps)
    self._act_graph, self._act_key = g, key

  def process_env_step(self, obs: dict, rewards: torch.Tensor, dones: torch.Tensor, extras: dict):
    s, t = self.storage, self.storage.step
    self.policy.update_normalization(obs)
    r = rewards.reshape(-1, 1).clone()
    if "time_outs" in extras:  # bootstrap on time-outs
      r += self.gamma * s.values[t] * extras["time_outs"].reshape(-1, 1).to(self.device).float()
    s.rewards[t].copy_(r)
    s.dones[t].copy_(dones.reshape(-1, 1).float())
    s.step += 1
    self.policy.reset(dones)

  def compute_returns(self, obs: dict):
    last_values = self.policy.evaluate(obs).detach()
    self.storage.compute_returns(last_values, self.gamma, self.lam,
                                 normalize_advantage=not self.normalize_advantage_per_mini_batch)

  def update(self) -> dict:
    mean_value = mean_surr = mean_ent = 0.0
    vals = []
    gen = self.storage.mini_batch_generator(self.num_mini_batches, self.num_learning_epochs)
    for obs_b, act_b, target_v, adv_b, ret_b, old_logp, old_mu, old_sigma in gen:
      if self.normalize_advantage_per_mini_batch:
        with torch.no_grad():
          adv_b = (adv_b - adv_b.mean()) / (adv_b.std() + 1e-8)
      self.policy.act(obs_b)
      logp = self.policy.get_actions_log_prob(act_b)
      value = self.policy.evaluate(obs_b)
      mu, sigma, entropy = self.policy.action_mean, self.policy.action_std, self.policy.entropy
      if self.desired_kl is not None and self.schedule == "adaptive":
        with torch.inference_mode():
          kl = torch.sum(torch.log(sigma / old_sigma + 1e-5)
                         + (old_sigma.pow(2) + (old_mu - mu).pow(2)) / (2.0 * sigma.pow(2)) - 0.5, dim=-1)
          kl_mean = kl.mean()
          if self.multi_gpu:
            dist.all_reduce(kl_mean, op=dist.ReduceOp.SUM)
            kl_mean /= dist.get_world_size()
          self.learning_rate = self._adapt_lr(float(kl_mean), self.learning_rate, self.desired_kl)
          if self.multi_gpu:
            lr = torch.tensor(self.learning_rate, device=self.device)
            dist.broadcast(lr, src=0)
            self.learning_rate = float(lr)
          for g in self.optimizer.param_groups:
            g["lr"] = self.learning_rate
      ratio = torch.exp(logp - old_logp.squeeze(-1))
      a = adv_b.squeeze(-1)
      surrogate = -a * ratio
      surrogate_clipped = -a * torch.clamp(ratio, 1.0 - self.clip_param, 1.0 + self.clip_param)
      surrogate_loss = torch.max(surrogate, surrogate_clipped).mean()
      if self.use_clipped_value_loss:
        v_clipped = target_v + (value - target_v).clamp(-self.clip_param, self.clip_param)
        value_loss = torch.max((value - ret_b).pow(2), (v_clipped - ret_b).pow(2)).mean()
      else:
        value_loss = (ret_b - value).pow(2).mean()
      loss = surrogate_loss + self.value_loss_coef * value_loss - self.entropy_coef * entropy.mean()
      self.optimizer.zero_grad()
      loss.backward()
      if self.multi_gpu:
        self.reduce_parameters()
      nn.utils.clip_grad_norm_(self.policy.parameters(), self.max_grad_norm)
      self.optimizer.step()
      vals.append(torch.stack([value_loss.detach(), surrogate_loss.detach(), entropy.mean().detach()]))
    n = self.num_learning_epochs * self.num_mini_batches
    mean_value, mean_surr, mean_ent = (torch.stack(vals).sum(0) / n).tolist()  # one host read
    self.storage.clear()
    return {"value_function": mean_value, "surrogate": mean_surr, "entropy": mean_ent}

  @staticmethod
  def _adapt_lr(kl_mean: float, lr: float, desired_kl: float) -> float:
    """rsl_rl's adaptive schedule (rank 0 decides, then broadcasts)."""
    if dist.is_available() and dist.is_initialized() and dist.get_rank() != 0:
      return lr
    if kl_mean > desired_kl * 2.0:
      return max(1e-5, lr / 1.5)
    if 0.0 < kl_mean < desired_kl / 2.0:
      return min(1e-2, lr * 1.5)
    return lr

  def broadcast_parameters(self):
    """Rank 0's model (and normaliser) state to every rank."""
    state = [self.policy.state_dict()]
    dist.broadcast_object_list(state, src=0)
    self.policy.load_state_dict(state[0])

  def reduce_parameters(self):
    """All-reduce the gradients as one flat bucket (mean over ranks)."""
    grads = [p.grad.view(-1) for p in self.policy.parameters() if p.grad is not None]
    flat = torch.cat(grads)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    flat /= dist.get_world_size()
    off = 0
    for p in self.policy.parameters():
      if p.grad is not None:
        n = p.numel()
        p.grad.data.copy_(flat[off:off + n].view_as(p.grad.data))
        off += n
