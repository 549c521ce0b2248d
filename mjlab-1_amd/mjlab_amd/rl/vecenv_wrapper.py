"""`src/mjlab/rl/vecenv_wrapper.py:1-111`: the rsl_rl VecEnv view of a ManagerBasedRlEnv.
Observations are a dict of group tensors (rsl_rl 3.x passes a TensorDict; `tensordict` is
not installed here and the learner only indexes it by group name)."""

from __future__ import annotations

import torch


class RslRlVecEnvWrapper:
  def __init__(self, env, clip_actions: float | None = None):
    self.env = env
    self.clip_actions = clip_actions
    self.num_envs = env.num_envs
    self.device = torch.device(env.device)
    self.max_episode_length = env.max_episode_length
    self.num_actions = env.action_manager.total_action_dim
    # reset at the start since rsl_rl does not call reset
    self.env.reset()

  @property
  def cfg(self):
    return self.env.cfg

  @property
  def unwrapped(self):
    return self.env

  @classmethod
  def class_name(cls) -> str:
    return cls.__name__

  @property
  def episode_length_buf(self) -> torch.Tensor:
    return self.env.episode_length_buf

  @episode_length_buf.setter
  def episode_length_buf(self, value: torch.Tensor) -> None:
    self.env.episode_length_buf.copy_(value)  # in place: graph-captured steps hold this tensor

  def seed(self, seed: int = -1) -> int:
    return self.env.seed(seed)

  def get_observations(self) -> dict:
    obs = getattr(self.env, "obs_buf", None)
    if obs is None:
      obs = self.env.observation_manager.compute()
    return dict(obs)

  def reset(self):
    obs, extras = self.env.reset()
    return dict(obs), extras

  def step(self, actions: torch.Tensor):
    if self.clip_actions is not None:
      actions = torch.clamp(actions, -self.clip_actions, self.clip_actions)
    obs, rew, terminated, truncated, extras = self.env.step(actions)
    dones = (terminated | truncated).to(dtype=torch.long)
    if not self.cfg.is_finite_horizon:
      extras["time_outs"] = truncated
    return dict(obs), rew, dones, extras

  def close(self) -> None:
    self.env.close()
