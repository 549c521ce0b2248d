"""On-policy runner restating rsl_rl.runners.OnPolicyRunner (rsl-rl-lib 3.1.0) as the
reference drives it (`scripts/train.py`, `tasks/velocity/rl/runner.py`): rollouts of
`num_steps_per_env` env steps under inference mode, returns, PPO update, logging and
checkpoints.  Multi-GPU follows rsl_rl's scheme: one process per GPU, each with its own
envs (seed + rank), rank 0's parameters broadcast at start, gradients all-reduced (RCCL).

Episode statistics stay on the device during the rollout (sums and counts of finished
episodes); the iteration's log reads them once, together with the env's extras["log"].
With several ranks, the rollout's statistics (finished-episode reward / length sums and
counts, and the numeric extras["log"] entries) are packed into one fixed-size vector and
all-gathered asynchronously on a side stream (distributed.StatsGather) while the PPO update
runs; rank 0's record then carries the world-wide values under "world/..." (episode means
over every rank's finished episodes, extras["log"] averaged over the ranks that report each
key; the key set is the union over ranks, agreed on every iteration).  rsl_rl logs rank
0's local statistics only (docs/api/distributed_training.md:68-100); those stay in the
record as before.
"""

from __future__ import annotations

import os
import time
from dataclasses import asdict

import torch
import torch.distributed as dist

from ..distributed import StatsGather
from .config import RslRlOnPolicyRunnerCfg
from .ppo import PPO, ActorCritic


class OnPolicyRunner:
  def __init__(self, env, train_cfg: RslRlOnPolicyRunnerCfg | dict, log_dir: str | None = None,
               device: str = "cpu"):
    cfg = asdict(train_cfg) if not isinstance(train_cfg, dict) else train_cfg
    self.cfg, self.alg_cfg, self.policy_cfg = cfg, dict(cfg["algorithm"]), dict(cfg["policy"])
    self.device = device
    self.env = env
    self.distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    self.rank = dist.get_rank() if self.distributed else 0
    self.world_size = dist.get_world_size() if self.distributed else 1
    obs = self.env.get_observations()
    self.obs_groups = cfg["obs_groups"]
    for group in ("policy", "critic"):
      for g in self.obs_groups[group]:
        if g not in obs:
          raise KeyError(f"observation group {g!r} (obs_groups[{group!r}]) not produced by the env")
    pc = {k: v for k, v in self.policy_cfg.items() if k != "class_name"}
    policy = ActorCritic(obs, self.obs_groups, self.env.num_actions, **pc).to(device)
    ac = {k: v for k, v in self.alg_cfg.items() if k != "class_name"}
    self.alg = PPO(policy, device=device, multi_gpu=self.distributed, **ac)
    self.num_steps_per_env = cfg["num_steps_per_env"]
    self.save_interval = cfg["save_interval"]
    self.alg.init_storage(self.env.num_envs, self.num_steps_per_env, obs, self.env.num_actions)
    if self.distributed:
      self.alg.broadcast_parameters()
    self.log_dir = log_dir
    self.current_learning_iteration = 0
    self.tot_timesteps = 0
    self.tot_time = 0.0
    self.history: list[dict] = []
    self._gather = None
    self._log_keys: list[str] | None = None

  @staticmethod
  def _numeric_log(log: dict) -> dict:
    out = {}
    for k, v in log.items():
      if isinstance(v, torch.Tensor) and v.numel() == 1:
        out[k] = v.reshape(())
      elif isinstance(v, (int, float)) and not isinstance(v, bool):
        out[k] = v
    return out

  def _agree_keys(self, local: list[str]) -> list[str]:
    """The union of every rank's extras["log"] keys (sorted), agreed on with one small host
    all-gather per iteration: ranks can hold different key sets (a rank whose envs did not
    reset yet, eager `_reset_idx` replacing the dict), and the packed all-gather needs one
    layout on every rank."""
    lists = [None] * self.world_size
    dist.all_gather_object(lists, sorted(local))
    return sorted(set().union(*[set(x) for x in lists]))

  def _start_gather(self, done_rew, done_len, done_cnt, log: dict) -> None:
    """Pack [reward sum, length sum, episode count, the agreed extras["log"] keys' values,
    and per key a presence flag (1 where this rank has the key)] and start the all-gather (no
    device sync).  The key list is re-agreed every iteration; the buffers are rebuilt only
    when it changes (on every rank at once, since every rank sees the same union)."""
    num = self._numeric_log(log)
    keys = self._agree_keys(list(num))
    if keys != self._log_keys or self._gather is None:
      self._log_keys = keys
      self._gather = StatsGather(3 + 2 * len(keys), torch.device(self.device))
    dev = done_rew.device
    vals = [done_rew, done_len, done_cnt]
    for k in self._log_keys:
      v = num.get(k, 0.0)
      vals.append(v.to(dev, torch.float32) if isinstance(v, torch.Tensor)
                  else torch.tensor(float(v), device=dev))
    vals += [torch.tensor(1.0 if k in num else 0.0, device=dev) for k in self._log_keys]
    self._gather.start(torch.stack([v.reshape(()).float() for v in vals]))

  def _finish_gather(self, rec: dict) -> None:
    g = self._gather.wait()  # [world, 3 + 2 nkeys]
    if self.rank != 0:
      return
    g = g.double().cpu()
    cnt = float(g[:, 2].sum())
    rec["world/episodes"] = cnt
    rec["world/mean_reward"] = float(g[:, 0].sum()) / cnt if cnt > 0 else None
    rec["world/mean_episode_length"] = float(g[:, 1].sum()) / cnt if cnt > 0 else None
    nk = len(self._log_keys)
    for i, k in enumerate(self._log_keys):
      have = g[:, 3 + nk + i]
      n = float(have.sum())
      # mean over the ranks that reported the key (missing values are padding, not zeros)
      rec[f"world/{k}"] = float((g[:, 3 + i] * have).sum()) / n if n > 0 else None

  def learn(self, num_learning_iterations: int, init_at_random_ep_len: bool = False) -> list[dict]:
    env, alg = self.env, self.alg
    if init_at_random_ep_len:
      env.episode_length_buf = torch.randint_like(env.episode_length_buf, high=int(env.max_episode_length))
    obs = env.get_observations()
    alg.policy.train()
    dev = torch.device(self.device)
    cur_rew = torch.zeros(env.num_envs, device=dev)
    cur_len = torch.zeros(env.num_envs, device=dev)
    start = self.current_learning_iteration
    for it in range(start, start + num_learning_iterations):
      t0 = time.perf_counter()
      done_rew = torch.zeros((), device=dev)
      done_len = torch.zeros((), device=dev)
      done_cnt = torch.zeros((), device=dev)
      with torch.inference_mode():
        for _ in range(self.num_steps_per_env):
          actions = alg.act(obs)
          obs, rewards, dones, extras = env.step(actions.to(env.device))
          alg.process_env_step(obs, rewards, dones, extras)
          cur_rew += rewards
          cur_len += 1
          d = dones.to(cur_rew.dtype)
          done_rew += (cur_rew * d).sum()
          done_len += (cur_len * d).sum()
          done_cnt += d.sum()
          cur_rew *= 1.0 - d
          cur_len *= 1.0 - d
        alg.compute_returns(obs)
      log = getattr(env.unwrapped, "extras", {}).get("log", {})
      if self.distributed:
        self._start_gather(done_rew, done_len, done_cnt, log)  # overlaps the update
      if dev.type == "cuda":
        torch.cuda.synchronize(dev)
      t1 = time.perf_counter()
      losses = alg.update()
      t2 = time.perf_counter()
      self.current_learning_iteration = it + 1
      steps = self.num_steps_per_env * env.num_envs * self.world_size
      self.tot_timesteps += steps
      self.tot_time += t2 - t0
      n = float(done_cnt)
      rec = {"iteration": it, "collection_time": t1 - t0, "learn_time": t2 - t1,
             "fps": steps / (t2 - t0), "learning_rate": alg.learning_rate,
             "mean_action_noise_std": float(alg.policy.std.detach().mean()) if hasattr(alg.policy, "std") else None,
             "episodes": n, "mean_reward": float(done_rew) / n if n > 0 else None,
             "mean_episode_length": float(done_len) / n if n > 0 else None, **losses}
      for k, v in log.items():
        try:
          rec[k] = float(v)
        except (TypeError, ValueError):
          pass
      if self.distributed:
        self._finish_gather(rec)
      self.history.append(rec)
      if self.log_dir and self.rank == 0 and self.save_interval and (it + 1) % self.save_interval == 0:
        self.save(os.path.join(self.log_dir, f"model_{it + 1}.pt"))
    if self.log_dir and self.rank == 0:
      self.save(os.path.join(self.log_dir, f"model_{self.current_learning_iteration}.pt"))
    return self.history

  def save(self, path: str) -> None:
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    torch.save({"model_state_dict": self.alg.policy.state_dict(),
                "optimizer_state_dict": self.alg.optimizer.state_dict(),
                "iter": self.current_learning_iteration, "infos": None}, path)

  def load(self, path: str, load_optimizer: bool = True) -> None:
    d = torch.load(path, map_location=self.device, weights_only=True)
    self.alg.policy.load_state_dict(d["model_state_dict"])
    if load_optimizer:
      self.alg.optimizer.load_state_dict(d["optimizer_state_dict"])
    self.current_learning_iteration = int(d["iter"])

  def get_inference_policy(self, device: str | None = None):
    self.alg.policy.eval()
    if device is not None:
      self.alg.policy.to(device)
    return self.alg.policy.act_inference
