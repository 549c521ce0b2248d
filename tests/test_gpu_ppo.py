"""One PPO iteration of `mjlab_amd.rl.PPO` in fp32 on the GPU -- the policy, the rollout
storage, the mini-batch permutation and the fused Adam on `cuda:0`, as `scripts/train.py` runs
them -- against the float64 numpy restatement of rsl-rl-lib 3.1.0's update in
`test_ppo_numpy.py` (the reference's learner, `uv.lock:2532-2547`, configured by
`src/mjlab/tasks/velocity/config/g1/rl_cfg.py:10-39`; rsl_rl itself is not installed, so
parity is by restatement of the published algorithm).

The numpy side starts from the GPU run's own initial weights, normaliser statistics, rollout
data and permutation (all fp32 values, read exactly into float64).  The fp32 tolerance:
  - the learning rate: equal (the adaptive rule's branch taken at every mini-batch must be the
    same; the run logs the KL so a tie would show);
  - the mean losses: within 1e-5 relative (fp32 sums over a 12-sample mini-batch);
  - every parameter: |p_gpu - p_np| <= 1e-6 |p| + UPDATE_REL |p_np - p_0| + 1e-7 with
    UPDATE_REL = 2e-3 -- Adam normalises each gradient element by its running RMS, so an
    element's update carries the *relative* fp32 error of its gradient (|g| against the
    magnitude of the terms summed into it), which reaches ~1e-4 for elements whose gradient
    is a small difference of per-sample terms; the bound scales with the update itself, not
    with lr, so a learner that did not move would fail it.
The same check runs in fp32 on the CPU (non-GPU suite), which pins the tolerance model
without a GPU; the GPU test adds the device path (cuda randperm, fused Adam kernels).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from mjlab_amd.rl.ppo import PPO, ActorCritic
from test_ppo_numpy import EPOCHS, HID, MB, N, NA_OBS, NACT, NC_OBS, T, NumpyPPO

UPDATE_REL = 2e-3


def _layers64(seq):
  lin = [m for m in seq if isinstance(m, torch.nn.Linear)]
  return [(m.weight.detach().double().cpu().numpy(), m.bias.detach().double().cpu().numpy()) for m in lin]


class _View:
  """NumpyPPO reads the policy's layers / std through `.actor`, `.critic`, `.std`."""

  def __init__(self, policy):
    self.actor, self.critic, self.std = policy.actor, policy.critic, policy.std


def run_iteration(seed: int, device: str):
  torch.manual_seed(seed)
  rng = np.random.default_rng(seed)
  f32 = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float32), device=device)
  obs0 = {"policy": torch.zeros(N, NA_OBS, device=device), "critic": torch.zeros(N, NC_OBS, device=device)}
  policy = ActorCritic(obs0, {"policy": ["policy"], "critic": ["critic"]}, NACT,
                       actor_obs_normalization=True, critic_obs_normalization=True,
                       actor_hidden_dims=HID, critic_hidden_dims=HID, activation="elu",
                       init_noise_std=0.8).to(device)
  cfg = dict(num_learning_epochs=EPOCHS, num_mini_batches=MB, clip_param=0.2, gamma=0.99, lam=0.95,
             value_loss_coef=1.0, entropy_coef=0.01, learning_rate=1e-3, max_grad_norm=1.0,
             use_clipped_value_loss=True, schedule="adaptive", desired_kl=0.01)
  ppo = PPO(policy, device=device, **cfg)
  ppo.init_storage(N, T, obs0, NACT)
  for _ in range(T):
    obs = {"policy": f32(rng.normal(0, 2, (N, NA_OBS))), "critic": f32(rng.normal(1, 1.5, (N, NC_OBS)))}
    ppo.act(obs)
    rew = f32(rng.normal(0, 1, N))
    dones = torch.as_tensor(rng.random(N) < 0.2, device=device)
    ppo.process_env_step(obs, rew, dones, {"time_outs": torch.as_tensor(rng.random(N) < 0.1, device=device)})
  last = {"policy": f32(rng.normal(0, 2, (N, NA_OBS))), "critic": f32(rng.normal(1, 1.5, (N, NC_OBS)))}
  ppo.compute_returns(last)
  s = ppo.storage
  nm = lambda n: (n._mean.double().cpu().numpy(), n._std.double().cpu().numpy(), n.eps)
  view = _View(policy)
  ref = NumpyPPO.__new__(NumpyPPO)
  ref.actor, ref.critic = _layers64(view.actor), _layers64(view.critic)
  ref.std = view.std.detach().double().cpu().numpy()
  ref.cfg, ref.lr = cfg, cfg["learning_rate"]
  ref.norm_a, ref.norm_c = nm(policy.actor_obs_normalizer), nm(policy.critic_obs_normalizer)
  ref.t = 0
  ref.m, ref.v = ref._zeros(), ref._zeros()
  p0 = [(W.copy(), b.copy()) for W, b in ref.actor + ref.critic] + [ref.std.copy()]
  flat = lambda t: t.detach().flatten(0, 1).double().cpu().numpy()
  data = dict(oa=flat(s.observations["policy"]), oc=flat(s.observations["critic"]), act=flat(s.actions),
              tv=flat(s.values)[:, 0], adv=flat(s.advantages)[:, 0], ret=flat(s.returns)[:, 0],
              logp=flat(s.actions_log_prob)[:, 0], mu=flat(s.mu), sig=flat(s.sigma))
  # the mini-batch permutation update() draws first (one randperm on the storage's device)
  torch.manual_seed(1000 + seed)
  mb = T * N // MB
  idx = torch.randperm(MB * mb, device=device).cpu().numpy()
  torch.manual_seed(1000 + seed)
  out = ppo.update()
  losses = []
  for _ in range(EPOCHS):
    for i in range(MB):
      b = idx[i * mb:(i + 1) * mb]
      losses.append(ref.step(data["oa"][b], data["oc"][b], data["act"][b], data["tv"][b], data["adv"][b],
                             data["ret"][b], data["logp"][b], data["mu"][b], data["sig"][b]))
  return out, ppo, policy, ref, losses, p0


def check_iteration(seed: int, device: str) -> dict:
  out, ppo, policy, ref, losses, p0 = run_iteration(seed, device)
  lv, ls, le = np.mean(np.array(losses), axis=0)
  assert out["value_function"] == pytest.approx(lv, rel=1e-5, abs=1e-7)
  assert out["surrogate"] == pytest.approx(ls, rel=1e-5, abs=1e-6)
  assert out["entropy"] == pytest.approx(le, rel=1e-5, abs=1e-7)
  assert ppo.learning_rate == pytest.approx(ref.lr, rel=1e-6)
  got = _layers64(policy.actor) + _layers64(policy.critic)
  worst = 0.0
  moved = 0.0
  pairs = []
  for (W, b), (Wr, br), (W0, b0) in zip(got, ref.actor + ref.critic, p0[:-1]):
    pairs += [(W, Wr, W0), (b, br, b0)]
  pairs.append((policy.std.detach().double().cpu().numpy(), ref.std, p0[-1]))
  for g, r, z in pairs:
    tol = 1e-6 * np.abs(r) + UPDATE_REL * np.abs(r - z) + 1e-7
    worst = max(worst, float((np.abs(g - r) / tol).max()))
    moved = max(moved, float(np.abs(r - z).max()))
    np.testing.assert_array_less(np.abs(g - r), tol)
  assert ref.t == EPOCHS * MB and moved > 1e-4  # the update moved the parameters
  return dict(worst_ratio=worst, moved=moved)


@pytest.mark.parametrize("seed", [0, 1])
def test_ppo_iteration_fp32_cpu(seed):
  """The fp32 tolerance model on the CPU (no GPU needed)."""
  check_iteration(seed, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_ppo_iteration_fp32_gpu(seed, gpu_device):
  """The learner's update on the MI355X: policy, storage, randperm and fused Adam on the GPU."""
  st = check_iteration(seed, gpu_device)
  print("ppo fp32 gpu", seed, st)
