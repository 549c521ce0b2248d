"""Manager layer: term configs, SceneEntityCfg and the seven managers.

API mirror of `src/mjlab/managers/*` (manager_term_config.py:14-162,
scene_entity_config.py:31-188, action/observation/reward/termination/command/event/
curriculum managers) so task configs and MDP terms written against mjlab run here.
Terms compute with torch on the GPU; the simulation state they read aliases the HIP
engine's HBM buffers.
"""

from __future__ import annotations

import inspect
import math
import re
from dataclasses import dataclass, field
from typing import Any, Callable, Literal, Sequence

import torch

# --------------------------------------------------------------------------- configs


@dataclass
class ManagerTermBaseCfg:
  func: Any = None
  params: dict[str, Any] = field(default_factory=dict)


@dataclass(kw_only=True)
class ActionTermCfg:
  class_type: type | None = None
  asset_name: str = "robot"
  clip: dict[str, tuple] | None = None


@dataclass(kw_only=True)
class CommandTermCfg:
  class_type: type | None = None
  resampling_time_range: tuple[float, float] = (1.0, 1.0)
  debug_vis: bool = False


@dataclass(kw_only=True)
class CurriculumTermCfg(ManagerTermBaseCfg):
  pass


EventMode = Literal["startup", "reset", "interval"]


@dataclass(kw_only=True)
class EventTermCfg(ManagerTermBaseCfg):
  mode: str = "reset"
  interval_range_s: tuple[float, float] | None = None
  is_global_time: bool = False
  min_step_count_between_reset: int = 0
  domain_randomization: bool = False


@dataclass(kw_only=True)
class ObservationTermCfg(ManagerTermBaseCfg):
  noise: Any = None
  clip: tuple[float, float] | None = None
  scale: Any = None
  delay_min_lag: int = 0
  delay_max_lag: int = 0
  history_length: int = 0
  flatten_history_dim: bool = True


@dataclass
class ObservationGroupCfg:
  terms: dict[str, ObservationTermCfg]
  concatenate_terms: bool = True
  concatenate_dim: int = -1
  enable_corruption: bool = False
  history_length: int | None = None
  flatten_history_dim: bool = True


@dataclass(kw_only=True)
class RewardTermCfg(ManagerTermBaseCfg):
  weight: float = 0.0


@dataclass(kw_only=True)
class TerminationTermCfg(ManagerTermBaseCfg):
  time_out: bool = False


# --------------------------------------------------------------------------- noise
@dataclass(kw_only=True)
class UniformNoiseCfg:
  """Additive U(n_min, n_max) noise (`utils/noise/noise_cfg.py:52-77`)."""
  n_min: float = -1.0
  n_max: float = 1.0
  operation: str = "add"

  def apply(self, data: torch.Tensor) -> torch.Tensor:
    noise = torch.rand_like(data) * (self.n_max - self.n_min) + self.n_min
    if self.operation == "add":
      return data + noise
    if self.operation == "scale":
      return data * noise
    return noise


@dataclass(kw_only=True)
class GaussianNoiseCfg:
  mean: float = 0.0
  std: float = 1.0
  operation: str = "add"

  def apply(self, data: torch.Tensor) -> torch.Tensor:
    noise = self.mean + self.std * torch.randn_like(data)
    if self.operation == "add":
      return data + noise
    if self.operation == "scale":
      return data * noise
    return noise


# --------------------------------------------------------------------------- entity cfg
def resolve_matching_names(keys, names, preserve_order=False):
  """Regex full-match of `keys` over `names`; natural order unless preserve_order
  (`utils/lab_api/string.py:178-260`)."""
  if isinstance(keys, str):
    keys = [keys]
  idx, out, key_of = [], [], []
  for ti, n in enumerate(names):
    hit = None
    for ki, k in enumerate(keys):
      if re.fullmatch(k, n):
        if hit is not None:
          raise ValueError(f"Multiple matches for '{n}': '{keys[hit]}' and '{k}'!")
        hit = ki
    if hit is not None:
      idx.append(ti)
      out.append(n)
      key_of.append(hit)
  unmatched = [k for ki, k in enumerate(keys) if ki not in key_of]
  if unmatched:
    raise ValueError(f"Not all regular expressions are matched: {unmatched} in {list(names)}")
  if preserve_order:
    order = sorted(range(len(idx)), key=lambda i: (key_of[i], i))
    idx = [idx[i] for i in order]
    out = [out[i] for i in order]
  return idx, out


def resolve_matching_names_values(data: dict, list_of_strings, preserve_order=False):
  idx, names, vals = [], [], []
  for ti, n in enumerate(list_of_strings):
    for k, v in data.items():
      if re.fullmatch(k, n):
        idx.append(ti)
        names.append(n)
        vals.append(v)
        break
  return idx, names, vals


@dataclass
class SceneEntityCfg:
  """Names -> ids resolved against an entity (`managers/scene_entity_config.py:31-188`)."""
  name: str
  joint_names: str | tuple[str, ...] | None = None
  joint_ids: list[int] | slice = field(default_factory=lambda: slice(None))
  body_names: str | tuple[str, ...] | None = None
  body_ids: list[int] | slice = field(default_factory=lambda: slice(None))
  geom_names: str | tuple[str, ...] | None = None
  geom_ids: list[int] | slice = field(default_factory=lambda: slice(None))
  site_names: str | tuple[str, ...] | None = None
  site_ids: list[int] | slice = field(default_factory=lambda: slice(None))
  actuator_names: str | tuple[str, ...] | None = None
  actuator_ids: list[int] | slice = field(default_factory=lambda: slice(None))
  preserve_order: bool = False

  def resolve(self, scene) -> None:
    ent = scene[self.name]
    for kind, finder in (("joint", ent.find_joints), ("body", ent.find_bodies),
                         ("geom", ent.find_geoms), ("site", ent.find_sites),
                         ("actuator", ent.find_actuators)):
      names = getattr(self, f"{kind}_names")
      if names is None or (isinstance(names, tuple) and len(names) == 0):
        continue
      ids, _ = finder(names, preserve_order=self.preserve_order)
      total = len(getattr(ent, f"{kind}_names"))
      if ids == list(range(total)) and not self.preserve_order:
        setattr(self, f"{kind}_ids", slice(None))
      else:
        # device index tensor: indexing with it needs no host->device copy, so terms stay
        # capturable in a HIP graph (a Python list index would upload every call)
        setattr(self, f"{kind}_ids", torch.tensor(ids, dtype=torch.long, device=scene.device))


# --------------------------------------------------------------------------- base
class ManagerTermBase:
  def __init__(self, cfg, env):
    self.cfg = cfg
    self._env = env

  @property
  def num_envs(self):
    return self._env.num_envs

  @property
  def device(self):
    return self._env.device

  def reset(self, env_ids=None) -> None:
    pass


class ManagerBase:
  def __init__(self, cfg, env):
    self.cfg = cfg
    self._env = env
    self._prepare_terms()

  @property
  def num_envs(self) -> int:
    return self._env.num_envs

  @property
  def device(self):
    return self._env.device

  def _resolve_common_term_cfg(self, term_name: str, term_cfg) -> None:
    for value in term_cfg.params.values():
      if isinstance(value, SceneEntityCfg):
        value.resolve(self._env.scene)
    if inspect.isclass(term_cfg.func):
      term_cfg.func = term_cfg.func(cfg=term_cfg, env=self._env)

  def _prepare_terms(self):
    raise NotImplementedError


def _class_terms(cfgs):
  return [c for c in cfgs if hasattr(c.func, "reset") and callable(c.func.reset)]


# --------------------------------------------------------------------------- actions
class ActionTerm(ManagerTermBase):
  @property
  def action_dim(self) -> int:
    raise NotImplementedError

  @property
  def raw_action(self) -> torch.Tensor:
    raise NotImplementedError

  def process_actions(self, actions: torch.Tensor) -> None:
    raise NotImplementedError

  def apply_actions(self) -> None:
    raise NotImplementedError


class ActionManager(ManagerBase):
  """`managers/action_manager.py:45-154`: splits the flat action over terms and keeps
  action / prev_action / prev_prev_action histories."""

  def _prepare_terms(self):
    self._terms: dict[str, ActionTerm] = {}
    for name, tcfg in self.cfg.items():
      if tcfg is None:
        continue
      self._terms[name] = tcfg.class_type(tcfg, self._env)
    self._action = torch.zeros(self.num_envs, self.total_action_dim, device=self.device)
    self._prev_action = torch.zeros_like(self._action)
    self._prev_prev_action = torch.zeros_like(self._action)

  @property
  def total_action_dim(self) -> int:
    return sum(t.action_dim for t in self._terms.values())

  @property
  def action_term_dim(self) -> list[int]:
    return [t.action_dim for t in self._terms.values()]

  @property
  def active_terms(self) -> list[str]:
    return list(self._terms.keys())

  @property
  def action(self) -> torch.Tensor:
    return self._action

  @property
  def prev_action(self) -> torch.Tensor:
    return self._prev_action

  @property
  def prev_prev_action(self) -> torch.Tensor:
    return self._prev_prev_action

  def get_term(self, name: str) -> ActionTerm:
    return self._terms[name]

  def reset(self, env_ids=None) -> dict:
    if env_ids is None:
      env_ids = slice(None)
    self._prev_prev_action[env_ids] = 0.0
    self._prev_action[env_ids] = 0.0
    self._action[env_ids] = 0.0
    for t in self._terms.values():
      t.reset(env_ids=env_ids)
    return {}

  def reset_masked(self, mask: torch.Tensor) -> dict:
    m = mask.unsqueeze(1)
    for buf in (self._prev_prev_action, self._prev_action, self._action):
      buf.masked_fill_(m, 0.0)
    for t in self._terms.values():
      if hasattr(t, "reset_masked"):
        t.reset_masked(mask)
    return {}

  def process_action(self, action: torch.Tensor) -> None:
    if action.shape[1] != self.total_action_dim:
      raise ValueError(f"Invalid action shape, expected: {self.total_action_dim}, "
                       f"received: {action.shape[1]}.")
    self._prev_prev_action.copy_(self._prev_action)
    self._prev_action.copy_(self._action)
    self._action.copy_(action.to(self.device))
    idx = 0
    for t in self._terms.values():
      t.process_actions(action[:, idx: idx + t.action_dim])
      idx += t.action_dim

  def apply_action(self) -> None:
    for t in self._terms.values():
      t.apply_actions()


# --------------------------------------------------------------------------- observations
class ObservationManager(ManagerBase):
  """`managers/observation_manager.py:154-208`: per term func -> clone -> noise (if the
  group enables corruption) -> clip -> scale; groups concatenated on the last dim."""

  def _prepare_terms(self):
    self._group_obs_term_names: dict[str, list[str]] = {}
    self._group_obs_term_cfgs: dict[str, list[ObservationTermCfg]] = {}
    self._group_obs_term_dim: dict[str, list[tuple]] = {}
    self._group_obs_concatenate: dict[str, bool] = {}
    self._group_obs_dim: dict = {}
    self._obs_buffer = None
    for gname, gcfg in self.cfg.items():
      if gcfg is None:
        continue
      names, cfgs = [], []
      for tname, tcfg in gcfg.terms.items():
        if tcfg is None:
          continue
        if tcfg.history_length or tcfg.delay_max_lag:
          raise NotImplementedError("observation history/delay buffers are out of scope")
        if not gcfg.enable_corruption:
          tcfg.noise = None
        if tcfg.scale is not None and not isinstance(tcfg.scale, torch.Tensor):
          tcfg.scale = torch.tensor(tcfg.scale, dtype=torch.float32, device=self.device)
        self._resolve_common_term_cfg(tname, tcfg)
        names.append(tname)
        cfgs.append(tcfg)
      self._group_obs_term_names[gname] = names
      self._group_obs_term_cfgs[gname] = cfgs
      self._group_obs_concatenate[gname] = gcfg.concatenate_terms
    for gname, cfgs in self._group_obs_term_cfgs.items():
      dims = [tuple(c.func(self._env, **c.params).shape[1:]) for c in cfgs]
      self._group_obs_term_dim[gname] = dims
      if self._group_obs_concatenate[gname]:
        self._group_obs_dim[gname] = (sum(int(math.prod(d)) for d in dims),)
      else:
        self._group_obs_dim[gname] = dims

  @property
  def active_terms(self):
    return self._group_obs_term_names

  @property
  def group_obs_dim(self):
    return self._group_obs_dim

  @property
  def group_obs_term_dim(self):
    return self._group_obs_term_dim

  @property
  def group_obs_concatenate(self):
    return self._group_obs_concatenate

  def get_term_cfg(self, group_name: str, term_name: str):
    return self._group_obs_term_cfgs[group_name][self._group_obs_term_names[group_name].index(term_name)]

  def reset(self, env_ids=None) -> dict:
    self._obs_buffer = None
    for cfgs in self._group_obs_term_cfgs.values():
      for c in _class_terms(cfgs):
        c.func.reset(env_ids=env_ids)
    return {}

  def compute(self, update_history: bool = False):
    if not update_history and self._obs_buffer is not None:
      return self._obs_buffer
    self._obs_buffer = {g: self.compute_group(g) for g in self._group_obs_term_names}
    return self._obs_buffer

  def compute_group(self, group_name: str, update_history: bool = False):
    out = {}
    for name, c in zip(self._group_obs_term_names[group_name], self._group_obs_term_cfgs[group_name]):
      obs = c.func(self._env, **c.params).clone()
      if c.noise is not None:
        obs = c.noise.apply(obs)
      if c.clip:
        obs = obs.clip_(min=c.clip[0], max=c.clip[1])
      if c.scale is not None:
        obs = obs.mul_(c.scale)
      out[name] = obs
    if self._group_obs_concatenate[group_name]:
      return torch.cat([o.reshape(o.shape[0], -1) for o in out.values()], dim=-1)
    return out


# --------------------------------------------------------------------------- rewards
class RewardManager(ManagerBase):
  """`managers/reward_manager.py:77-91`: sum_i w_i f_i dt with nan_to_num, episode sums."""

  def _prepare_terms(self):
    self._term_names: list[str] = []
    self._term_cfgs: list[RewardTermCfg] = []
    for name, c in self.cfg.items():
      if c is None:
        continue
      self._resolve_common_term_cfg(name, c)
      self._term_names.append(name)
      self._term_cfgs.append(c)
    n = self.num_envs
    self._episode_sums = {k: torch.zeros(n, device=self.device) for k in self._term_names}
    self._reward_buf = torch.zeros(n, device=self.device)
    self._step_reward = torch.zeros(n, len(self._term_names), device=self.device)

  @property
  def active_terms(self):
    return self._term_names

  def get_term_cfg(self, name):
    return self._term_cfgs[self._term_names.index(name)]

  def reset(self, env_ids=None) -> dict:
    if env_ids is None:
      env_ids = slice(None)
    extras = {}
    for k, v in self._episode_sums.items():
      extras["Episode_Reward/" + k] = torch.mean(v[env_ids]) / self._env.max_episode_length_s
      v[env_ids] = 0.0
    for c in _class_terms(self._term_cfgs):
      c.func.reset(env_ids=env_ids)
    return extras

  def reset_masked(self, mask: torch.Tensor) -> dict:
    extras = {}
    cnt = torch.clamp(mask.sum(), min=1).float()
    for k, v in self._episode_sums.items():
      extras["Episode_Reward/" + k] = (v * mask).sum() / cnt / self._env.max_episode_length_s
      v.masked_fill_(mask, 0.0)
    for c in _class_terms(self._term_cfgs):
      if hasattr(c.func, "reset_masked"):
        c.func.reset_masked(mask)
    return extras

  def compute(self, dt: float) -> torch.Tensor:
    self._reward_buf.zero_()
    for i, (name, c) in enumerate(zip(self._term_names, self._term_cfgs)):
      if c.weight == 0.0:
        self._step_reward[:, i] = 0.0
        continue
      value = c.func(self._env, **c.params) * c.weight * dt
      value = torch.nan_to_num(value, nan=0.0, posinf=0.0, neginf=0.0)
      self._reward_buf += value
      self._episode_sums[name] += value
      self._step_reward[:, i] = value / dt
    return self._reward_buf


# --------------------------------------------------------------------------- terminations
class TerminationManager(ManagerBase):
  """`managers/termination_manager.py:87-97`."""

  def _prepare_terms(self):
    self._term_names, self._term_cfgs = [], []
    for name, c in self.cfg.items():
      if c is None:
        continue
      self._resolve_common_term_cfg(name, c)
      self._term_names.append(name)
      self._term_cfgs.append(c)
    n = self.num_envs
    self._term_dones = {k: torch.zeros(n, dtype=torch.bool, device=self.device)
                        for k in self._term_names}
    self._truncated_buf = torch.zeros(n, dtype=torch.bool, device=self.device)
    self._terminated_buf = torch.zeros_like(self._truncated_buf)

  @property
  def active_terms(self):
    return self._term_names

  @property
  def dones(self):
    return self._truncated_buf | self._terminated_buf

  @property
  def time_outs(self):
    return self._truncated_buf

  @property
  def terminated(self):
    return self._terminated_buf

  def get_term(self, name):
    return self._term_dones[name]

  def reset(self, env_ids=None) -> dict:
    if env_ids is None:
      env_ids = slice(None)
    extras = {}
    for k, v in self._term_dones.items():
      extras["Episode_Termination/" + k] = torch.count_nonzero(v[env_ids])
    for c in _class_terms(self._term_cfgs):
      c.func.reset(env_ids=env_ids)
    return extras

  def reset_masked(self, mask: torch.Tensor) -> dict:
    return {"Episode_Termination/" + k: (v & mask).sum() for k, v in self._term_dones.items()}

  def compute(self) -> torch.Tensor:
    self._truncated_buf.zero_()
    self._terminated_buf.zero_()
    for name, c in zip(self._term_names, self._term_cfgs):
      value = c.func(self._env, **c.params)
      if c.time_out:
        self._truncated_buf |= value
      else:
        self._terminated_buf |= value
      self._term_dones[name][:] = value
    return self._truncated_buf | self._terminated_buf


# --------------------------------------------------------------------------- commands
class CommandTerm(ManagerTermBase):
  """`managers/command_manager.py:19-100`: resampling timer + metrics."""

  def __init__(self, cfg, env):
    super().__init__(cfg, env)
    self.metrics: dict[str, torch.Tensor] = {}
    self.time_left = torch.zeros(self.num_envs, device=self.device)
    self.command_counter = torch.zeros(self.num_envs, device=self.device, dtype=torch.long)

  @property
  def command(self):
    raise NotImplementedError

  def reset(self, env_ids=None) -> dict:
    if env_ids is None:
      env_ids = torch.arange(self.num_envs, device=self.device)
    extras = {}
    for k, v in self.metrics.items():
      extras[k] = torch.mean(v[env_ids])
      v[env_ids] = 0.0
    self.command_counter[env_ids] = 0
    self._resample(env_ids)
    return extras

  def compute(self, dt: float) -> None:
    self._update_metrics()
    self.time_left -= dt
    if getattr(self._env, "sync_free", False):
      # a resampling period of >= 1e8 s (the tracking command's 1e9) never elapses: skip
      # the masked resample instead of recording a no-op into the step graph
      if self.cfg.resampling_time_range[0] < 1e8:
        self._resample_masked(self.time_left <= 0.0)
    else:
      ids = (self.time_left <= 0.0).nonzero().flatten()
      if len(ids) > 0:
        self._resample(ids)
    self._update_command()

  def reset_masked(self, mask: torch.Tensor) -> dict:
    cnt = torch.clamp(mask.sum(), min=1).float()
    extras = {}
    for k, v in self.metrics.items():
      extras[k] = (v * mask).sum() / cnt
      v.masked_fill_(mask, 0.0)
    self.command_counter.masked_fill_(mask, 0)
    self._resample_masked(mask)
    return extras

  def _resample_masked(self, mask: torch.Tensor) -> None:
    lo, hi = self.cfg.resampling_time_range
    fresh = torch.rand(self.num_envs, device=self.device) * (hi - lo) + lo
    self.time_left.copy_(torch.where(mask, fresh, self.time_left))
    self._resample_command_masked(mask)
    self.command_counter += mask.long()

  def _resample(self, env_ids: torch.Tensor) -> None:
    if len(env_ids) != 0:
      lo, hi = self.cfg.resampling_time_range
      self.time_left[env_ids] = torch.rand(len(env_ids), device=self.device) * (hi - lo) + lo
      self._resample_command(env_ids)
      self.command_counter[env_ids] += 1

  def _update_metrics(self): ...

  def _resample_command(self, env_ids): ...

  def _update_command(self): ...


class CommandManager(ManagerBase):
  def _prepare_terms(self):
    self._terms: dict[str, CommandTerm] = {}
    for name, c in self.cfg.items():
      if c is None:
        continue
      self._terms[name] = c.class_type(c, self._env)

  @property
  def active_terms(self):
    return list(self._terms.keys())

  def reset(self, env_ids=None) -> dict:
    extras = {}
    for name, t in self._terms.items():
      for k, v in t.reset(env_ids=env_ids).items():
        extras[f"Metrics/{name}/{k}"] = v
    return extras

  def reset_masked(self, mask: torch.Tensor) -> dict:
    extras = {}
    for name, t in self._terms.items():
      for k, v in t.reset_masked(mask).items():
        extras[f"Metrics/{name}/{k}"] = v
    return extras

  def compute(self, dt: float) -> None:
    for t in self._terms.values():
      t.compute(dt)

  def get_command(self, name: str) -> torch.Tensor:
    return self._terms[name].command

  def get_term(self, name: str) -> CommandTerm:
    return self._terms[name]

  def get_term_cfg(self, name: str):
    return self.cfg[name]


class NullCommandManager:
  active_terms: list = []

  def reset(self, env_ids=None):
    return {}

  def reset_masked(self, mask):
    return {}

  def compute(self, dt):
    pass

  def get_command(self, name):
    return None


# --------------------------------------------------------------------------- events
class EventManager(ManagerBase):
  """`managers/event_manager.py:100-220`: startup / reset / interval modes."""

  def _prepare_terms(self):
    self._mode_term_names: dict[str, list[str]] = {}
    self._mode_term_cfgs: dict[str, list[EventTermCfg]] = {}
    self._interval_time_left: list[torch.Tensor] = []
    self._reset_last_step: list[torch.Tensor] = []
    self._reset_once: list[torch.Tensor] = []
    self._dr_fields: list[str] = []
    for name, c in self.cfg.items():
      if c is None:
        continue
      self._resolve_common_term_cfg(name, c)
      self._mode_term_names.setdefault(c.mode, []).append(name)
      self._mode_term_cfgs.setdefault(c.mode, []).append(c)
      if c.mode == "interval":
        if c.interval_range_s is None:
          raise ValueError(f"Event term '{name}' has mode 'interval' but no interval_range_s")
        lo, hi = c.interval_range_s
        n = 1 if c.is_global_time else self.num_envs
        dev = "cpu" if c.is_global_time else self.device
        self._interval_time_left.append(torch.rand(n, device=dev) * (hi - lo) + lo)
      elif c.mode == "reset":
        self._reset_last_step.append(torch.zeros(self.num_envs, dtype=torch.int32, device=self.device))
        self._reset_once.append(torch.zeros(self.num_envs, dtype=torch.bool, device=self.device))
      if c.domain_randomization and c.params["field"] not in self._dr_fields:
        self._dr_fields.append(c.params["field"])

  @property
  def available_modes(self) -> list[str]:
    return list(self._mode_term_names.keys())

  @property
  def active_terms(self):
    return self._mode_term_names

  @property
  def domain_randomization_fields(self) -> tuple[str, ...]:
    return tuple(self._dr_fields)

  def reset(self, env_ids=None) -> dict:
    for cfgs in self._mode_term_cfgs.values():
      for c in _class_terms(cfgs):
        c.func.reset(env_ids=env_ids)
    if "interval" in self._mode_term_cfgs and env_ids is not None:
      for i, c in enumerate(self._mode_term_cfgs["interval"]):
        if not c.is_global_time:
          lo, hi = c.interval_range_s
          ids = env_ids if isinstance(env_ids, torch.Tensor) else torch.arange(self.num_envs, device=self.device)
          self._interval_time_left[i][ids] = torch.rand(len(ids), device=self.device) * (hi - lo) + lo
    return {}

  def reset_masked(self, mask: torch.Tensor) -> dict:
    for i, c in enumerate(self._mode_term_cfgs.get("interval", [])):
      if not c.is_global_time:
        lo, hi = c.interval_range_s
        fresh = torch.rand(self.num_envs, device=self.device) * (hi - lo) + lo
        self._interval_time_left[i].copy_(torch.where(mask, fresh, self._interval_time_left[i]))
    return {}

  def apply_masked(self, mode: str, mask: torch.Tensor | None = None, dt: float | None = None) -> None:
    """Sync-free variant for 'reset' (given a mask) and 'interval' (computes its own mask):
    every term must provide a `.masked` implementation (graph-capturable)."""
    for i, c in enumerate(self._mode_term_cfgs.get(mode, [])):
      fn = getattr(c.func, "masked", None)
      if fn is None:
        raise NotImplementedError(f"event term {c.func} has no masked variant")
      if mode == "interval":
        if c.is_global_time:
          raise NotImplementedError("global-time interval events are not graph-capturable")
        tl = self._interval_time_left[i]
        tl -= dt
        m = tl < 1e-6
        lo, hi = c.interval_range_s
        fresh = torch.rand(self.num_envs, device=self.device) * (hi - lo) + lo
        tl.copy_(torch.where(m, fresh, tl))
        fn(self._env, m, **c.params)
      else:
        if c.min_step_count_between_reset != 0:
          raise NotImplementedError("min_step_count_between_reset requires the eager path")
        fn(self._env, mask, **c.params)

  def apply(self, mode: str, env_ids=None, dt: float | None = None,
            global_env_step_count: int | None = None) -> None:
    if mode == "interval" and dt is None:
      raise ValueError(f"Event mode '{mode}' requires the time-step of the environment.")
    if mode == "reset" and global_env_step_count is None:
      raise ValueError("Event mode 'reset' requires the total number of environment steps.")
    for i, c in enumerate(self._mode_term_cfgs.get(mode, [])):
      if mode == "interval":
        tl = self._interval_time_left[i]
        tl -= dt
        lo, hi = c.interval_range_s
        if c.is_global_time:
          if tl.item() < 1e-6:
            tl[:] = torch.rand(1) * (hi - lo) + lo
            c.func(self._env, None, **c.params)
        else:
          ids = (tl < 1e-6).nonzero().flatten()
          if len(ids) > 0:
            tl[ids] = torch.rand(len(ids), device=self.device) * (hi - lo) + lo
            c.func(self._env, ids, **c.params)
      elif mode == "reset":
        if env_ids is None:
          env_ids = slice(None)
        ms = c.min_step_count_between_reset
        if ms == 0:
          self._reset_last_step[i][env_ids] = global_env_step_count
          self._reset_once[i][env_ids] = True
          c.func(self._env, env_ids, **c.params)
        else:
          last = self._reset_last_step[i][env_ids]
          once = self._reset_once[i][env_ids]
          valid = (global_env_step_count - last) >= ms
          valid |= (last == 0) & ~once
          ids = env_ids[valid] if isinstance(env_ids, torch.Tensor) else valid.nonzero().flatten()
          if len(ids) > 0:
            self._reset_once[i][ids] = True
            self._reset_last_step[i][ids] = global_env_step_count
            c.func(self._env, ids, **c.params)
      else:
        c.func(self._env, env_ids, **c.params)


# --------------------------------------------------------------------------- curriculum
class CurriculumManager(ManagerBase):
  def _prepare_terms(self):
    self._term_names, self._term_cfgs = [], []
    self._curriculum_state: dict[str, Any] = {}
    for name, c in self.cfg.items():
      if c is None:
        continue
      self._resolve_common_term_cfg(name, c)
      self._term_names.append(name)
      self._term_cfgs.append(c)

  @property
  def active_terms(self):
    return self._term_names

  def reset(self, env_ids=None) -> dict:
    extras = {}
    for name, state in self._curriculum_state.items():
      if isinstance(state, dict):
        for k, v in state.items():
          extras[f"Curriculum/{name}/{k}"] = v
      elif state is not None:
        extras[f"Curriculum/{name}"] = state
    for c in _class_terms(self._term_cfgs):
      c.func.reset(env_ids=env_ids)
    return extras

  def reset_masked(self, mask) -> dict:
    return self.reset(None)

  def compute(self, env_ids=None, skip_masked: bool = False) -> None:
    """skip_masked: leave out the terms with a mask form (per-env terms such as the terrain
    levels), which the sync-free step runs on its reset mask (compute_masked)."""
    if env_ids is None:
      env_ids = slice(None)
    for name, c in zip(self._term_names, self._term_cfgs):
      if skip_masked and hasattr(c.func, "masked"):
        continue
      self._curriculum_state[name] = c.func(self._env, env_ids, **c.params)

  def compute_masked(self, mask) -> None:
    """The mask forms of the per-env terms, for the envs resetting this step (the
    reference runs them in _reset_idx, before the reset events read the env origins)."""
    for name, c in zip(self._term_names, self._term_cfgs):
      if hasattr(c.func, "masked"):
        self._curriculum_state[name] = c.func.masked(self._env, mask, **c.params)


class NullCurriculumManager:
  active_terms: list = []

  def compute(self, env_ids=None, skip_masked: bool = False) -> None:
    pass

  def compute_masked(self, mask) -> None:
    pass

  def reset(self, env_ids=None):
    return {}

  def reset_masked(self, mask):
    return {}
