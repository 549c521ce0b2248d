"""MDP term library used by the velocity / tracking / jump tasks.

Generic terms restate `src/mjlab/envs/mdp/{observations,rewards,terminations,events}.py`
and the joint-position action (`envs/mdp/actions/joint_actions.py:18-129`); velocity-task
terms restate `src/mjlab/tasks/velocity/mdp/{rewards,observations,velocity_command,
curriculums}.py`.  Same names, parameters and math.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

from .managers import (ActionTerm, ActionTermCfg, CommandTerm, CommandTermCfg, SceneEntityCfg,
                       resolve_matching_names_values)
from .math_utils import quat_apply, quat_apply_inverse, quat_from_euler_xyz, quat_mul, \
  sample_uniform, wrap_to_pi

_ROBOT = SceneEntityCfg("robot")


# =========================================================================== actions
@dataclass(kw_only=True)
class JointPositionActionCfg(ActionTermCfg):
  actuator_names: tuple[str, ...] = (".*",)
  scale: float | dict[str, float] = 1.0
  offset: float | dict[str, float] = 0.0
  use_default_offset: bool = True

  def __post_init__(self):
    self.class_type = JointPositionAction


class JointPositionAction(ActionTerm):
  """target = a * scale + offset - encoder_bias -> joint_pos_target (joint_actions.py)."""

  def __init__(self, cfg: JointPositionActionCfg, env):
    super().__init__(cfg, env)
    self._asset = env.scene[cfg.asset_name]
    ids, names = self._asset.find_joints_by_actuator_names(cfg.actuator_names)
    self._joint_ids = torch.tensor(ids, device=self.device, dtype=torch.long)
    self._joint_names = names
    n = len(ids)
    self._raw = torch.zeros(self.num_envs, n, device=self.device)
    self._processed = torch.zeros_like(self._raw)
    if isinstance(cfg.scale, (int, float)):
      self._scale = float(cfg.scale)
    else:
      self._scale = torch.ones(self.num_envs, n, device=self.device)
      idx, _, val = resolve_matching_names_values(cfg.scale, names)
      self._scale[:, idx] = torch.tensor(val, device=self.device)
    if isinstance(cfg.offset, (int, float)):
      self._offset = float(cfg.offset)
    else:
      self._offset = torch.zeros_like(self._raw)
      idx, _, val = resolve_matching_names_values(cfg.offset, names)
      self._offset[:, idx] = torch.tensor(val, device=self.device)
    if cfg.use_default_offset:
      self._offset = self._asset.data.default_joint_pos[:, self._joint_ids].clone()

  @property
  def action_dim(self):
    return len(self._joint_names)

  @property
  def raw_action(self):
    return self._raw

  @property
  def scale(self):
    return self._scale

  @property
  def offset(self):
    return self._offset

  def process_actions(self, actions):
    self._raw[:] = actions
    self._processed = self._raw * self._scale + self._offset

  def apply_actions(self):
    bias = self._asset.data.encoder_bias[:, self._joint_ids]
    self._asset.set_joint_position_target(self._processed - bias, joint_ids=self._joint_ids)

  def reset(self, env_ids=None):
    self._raw[slice(None) if env_ids is None else env_ids] = 0.0


# =========================================================================== observations
def base_lin_vel(env, asset_cfg=_ROBOT):
  return env.scene[asset_cfg.name].data.root_link_lin_vel_b


def base_ang_vel(env, asset_cfg=_ROBOT):
  return env.scene[asset_cfg.name].data.root_link_ang_vel_b


def projected_gravity(env, asset_cfg=_ROBOT):
  return env.scene[asset_cfg.name].data.projected_gravity_b


def joint_pos_rel(env, biased: bool = False, asset_cfg=_ROBOT):
  a = env.scene[asset_cfg.name]
  jp = a.data.joint_pos_biased if biased else a.data.joint_pos
  return jp[:, asset_cfg.joint_ids] - a.data.default_joint_pos[:, asset_cfg.joint_ids]


def joint_vel_rel(env, asset_cfg=_ROBOT):
  a = env.scene[asset_cfg.name]
  return a.data.joint_vel[:, asset_cfg.joint_ids] - a.data.default_joint_vel[:, asset_cfg.joint_ids]


def last_action(env, action_name: str | None = None):
  if action_name is None:
    return env.action_manager.action
  return env.action_manager.get_term(action_name).raw_action


def generated_commands(env, command_name: str):
  return env.command_manager.get_command(command_name)


def builtin_sensor(env, sensor_name: str):
  return env.scene[sensor_name].data


def foot_height(env, asset_cfg=_ROBOT):
  return env.scene[asset_cfg.name].data.site_pos_w[:, asset_cfg.site_ids, 2]


def foot_air_time(env, sensor_name: str):
  return env.scene[sensor_name].data.current_air_time


def foot_contact(env, sensor_name: str):
  return (env.scene[sensor_name].data.found > 0).float()


def foot_contact_forces(env, sensor_name: str):
  f = env.scene[sensor_name].data.force.flatten(start_dim=1)
  return torch.sign(f) * torch.log1p(torch.abs(f))


# =========================================================================== terminations
def time_out(env):
  return env.episode_length_buf >= env.max_episode_length


def bad_orientation(env, limit_angle: float, asset_cfg=_ROBOT):
  g = env.scene[asset_cfg.name].data.projected_gravity_b
  return torch.acos(-g[:, 2]).abs() > limit_angle


def root_height_below_minimum(env, minimum_height: float, asset_cfg=_ROBOT):
  return env.scene[asset_cfg.name].data.root_link_pos_w[:, 2] < minimum_height


def nan_detection(env):
  """`envs/mdp/terminations.py:45-47`: NaN or Inf anywhere in qpos, qvel, qacc or
  qacc_warmstart of the env (NanGuard.detect_nans)."""
  from .sim.sim import NanGuard
  return NanGuard.detect_nans(env.sim.data)


def illegal_contact(env, sensor_name: str):
  return torch.any(env.scene[sensor_name].data.found > 0, dim=-1)


# =========================================================================== rewards
def _command_active(env, command_name, threshold):
  c = env.command_manager.get_command(command_name)
  total = torch.norm(c[:, :2], dim=1) + torch.abs(c[:, 2])
  return (total > threshold).float()


def track_linear_velocity(env, std: float, command_name: str, asset_cfg=_ROBOT):
  a = env.scene[asset_cfg.name]
  c = env.command_manager.get_command(command_name)
  v = a.data.root_link_lin_vel_b
  err = torch.sum(torch.square(c[:, :2] - v[:, :2]), dim=1) + torch.square(v[:, 2])
  return torch.exp(-err / std ** 2)


def track_angular_velocity(env, std: float, command_name: str, asset_cfg=_ROBOT):
  a = env.scene[asset_cfg.name]
  c = env.command_manager.get_command(command_name)
  w = a.data.root_link_ang_vel_b
  err = torch.square(c[:, 2] - w[:, 2]) + torch.sum(torch.square(w[:, :2]), dim=1)
  return torch.exp(-err / std ** 2)


def flat_orientation(env, std: float, asset_cfg=_ROBOT):
  a = env.scene[asset_cfg.name]
  if not isinstance(asset_cfg.body_ids, slice) and len(asset_cfg.body_ids) > 0:
    q = a.data.body_link_quat_w[:, asset_cfg.body_ids, :].squeeze(1)
    g = quat_apply_inverse(q, a.data.gravity_vec_w)
  else:
    g = a.data.projected_gravity_b
  return torch.exp(-torch.sum(torch.square(g[:, :2]), dim=1) / std ** 2)


def self_collision_cost(env, sensor_name: str):
  return env.scene[sensor_name].data.found.squeeze(-1)


def body_angular_velocity_penalty(env, asset_cfg=_ROBOT):
  w = env.scene[asset_cfg.name].data.body_link_ang_vel_w[:, asset_cfg.body_ids, :].squeeze(1)
  return torch.sum(torch.square(w[:, :2]), dim=1)


def angular_momentum_penalty(env, sensor_name: str):
  h = env.scene[sensor_name].data
  sq = torch.sum(torch.square(h), dim=-1)
  env.extras["log"]["Metrics/angular_momentum_mean"] = torch.mean(torch.sqrt(sq))
  return sq


def joint_pos_limits(env, asset_cfg=_ROBOT):
  a = env.scene[asset_cfg.name]
  lim = a.data.soft_joint_pos_limits
  q = a.data.joint_pos[:, asset_cfg.joint_ids]
  out = -(q - lim[:, asset_cfg.joint_ids, 0]).clip(max=0.0)
  out += (q - lim[:, asset_cfg.joint_ids, 1]).clip(min=0.0)
  return torch.sum(out, dim=1)


def is_alive(env):
  """`envs/mdp/rewards.py:22-24`."""
  return (~env.termination_manager.terminated).float()


def is_terminated(env):
  return env.termination_manager.terminated.float()


def joint_torques_l2(env, asset_cfg=_ROBOT):
  """`envs/mdp/rewards.py:32-37` (all actuators, whatever asset_cfg selects)."""
  return torch.sum(torch.square(env.scene[asset_cfg.name].data.actuator_force), dim=1)


def action_acc_l2(env):
  """`envs/mdp/rewards.py:63-70`."""
  am = env.action_manager
  return torch.sum(torch.square(am.action - 2 * am.prev_action + am.prev_prev_action), dim=1)


def action_rate_l2(env):
  return torch.sum(torch.square(env.action_manager.action - env.action_manager.prev_action), dim=1)


def feet_air_time(env, sensor_name: str, threshold_min: float = 0.05, threshold_max: float = 0.5,
                  command_name: str | None = None, command_threshold: float = 0.5):
  t = env.scene[sensor_name].data.current_air_time
  reward = torch.sum(((t > threshold_min) & (t < threshold_max)).float(), dim=1)
  in_air = (t > 0).float()
  env.extras["log"]["Metrics/air_time_mean"] = torch.sum(t * in_air) / torch.clamp(in_air.sum(), min=1)
  if command_name is not None:
    reward = reward * _command_active(env, command_name, command_threshold)
  return reward


def feet_clearance(env, target_height: float, command_name: str | None = None,
                   command_threshold: float = 0.01, asset_cfg=_ROBOT):
  a = env.scene[asset_cfg.name]
  z = a.data.site_pos_w[:, asset_cfg.site_ids, 2]
  v = torch.norm(a.data.site_lin_vel_w[:, asset_cfg.site_ids, :2], dim=-1)
  cost = torch.sum(torch.abs(z - target_height) * v, dim=1)
  if command_name is not None:
    cost = cost * _command_active(env, command_name, command_threshold)
  return cost


class feet_swing_height:
  """Stateful: peak height per foot while airborne, cost at landing."""

  def __init__(self, cfg, env):
    self.peak_heights = torch.zeros(env.num_envs, len(cfg.params["asset_cfg"].site_names),
                                    device=env.device)
    self.step_dt = env.step_dt

  def reset(self, env_ids=None):
    pass

  def __call__(self, env, sensor_name, target_height, command_name, command_threshold, asset_cfg):
    a = env.scene[asset_cfg.name]
    s = env.scene[sensor_name]
    h = a.data.site_pos_w[:, asset_cfg.site_ids, 2]
    in_air = s.data.found == 0
    self.peak_heights.copy_(torch.where(in_air, torch.maximum(self.peak_heights, h), self.peak_heights))
    first = s.compute_first_contact(dt=self.step_dt)
    active = _command_active(env, command_name, command_threshold)
    err = self.peak_heights / target_height - 1.0
    cost = torch.sum(torch.square(err) * first.float(), dim=1) * active
    nland = torch.sum(first.float())
    env.extras["log"]["Metrics/peak_height_mean"] = (
      torch.sum(self.peak_heights * first.float()) / torch.clamp(nland, min=1))
    self.peak_heights.masked_fill_(first, 0.0)
    return cost


def feet_slip(env, sensor_name: str, command_name: str, command_threshold: float = 0.01,
              asset_cfg=_ROBOT):
  a = env.scene[asset_cfg.name]
  s = env.scene[sensor_name]
  active = _command_active(env, command_name, command_threshold)
  inc = (s.data.found > 0).float()
  v = torch.norm(a.data.site_lin_vel_w[:, asset_cfg.site_ids, :2], dim=-1)
  cost = torch.sum(torch.square(v) * inc, dim=1) * active
  env.extras["log"]["Metrics/slip_velocity_mean"] = torch.sum(v * inc) / torch.clamp(inc.sum(), min=1)
  return cost


def soft_landing(env, sensor_name: str, command_name: str | None = None,
                 command_threshold: float = 0.05):
  s = env.scene[sensor_name]
  fm = torch.norm(s.data.force, dim=-1)
  first = s.compute_first_contact(dt=env.step_dt)
  impact = fm * first.float()
  cost = torch.sum(impact, dim=1)
  env.extras["log"]["Metrics/landing_force_mean"] = torch.sum(impact) / torch.clamp(first.float().sum(), min=1)
  if command_name is not None:
    cost = cost * _command_active(env, command_name, command_threshold)
  return cost


class variable_posture:
  """exp(-mean((q-q0)^2/std^2)) with std chosen by command speed band."""

  def __init__(self, cfg, env):
    p = cfg.params
    a = env.scene[p["asset_cfg"].name]
    self.default_joint_pos = a.data.default_joint_pos
    _, names = a.find_joints(p["asset_cfg"].joint_names)
    mk = lambda d: torch.tensor(resolve_matching_names_values(d, names)[2], device=env.device,
                                dtype=torch.float32)
    self.std_standing = mk(p["std_standing"])
    self.std_walking = mk(p["std_walking"])
    self.std_running = mk(p["std_running"])

  def reset(self, env_ids=None):
    pass

  def __call__(self, env, std_standing, std_walking, std_running, asset_cfg, command_name,
               walking_threshold=0.5, running_threshold=1.5):
    a = env.scene[asset_cfg.name]
    c = env.command_manager.get_command(command_name)
    sp = torch.norm(c[:, :2], dim=1) + torch.abs(c[:, 2])
    st = (sp < walking_threshold).float().unsqueeze(1)
    wk = ((sp >= walking_threshold) & (sp < running_threshold)).float().unsqueeze(1)
    rn = (sp >= running_threshold).float().unsqueeze(1)
    std = self.std_standing * st + self.std_walking * wk + self.std_running * rn
    err = torch.square(a.data.joint_pos[:, asset_cfg.joint_ids] -
                       self.default_joint_pos[:, asset_cfg.joint_ids])
    return torch.exp(-torch.mean(err / std ** 2, dim=1))


# =========================================================================== events
def reset_root_state_uniform(env, env_ids, pose_range: dict, velocity_range: dict | None = None,
                             asset_cfg=_ROBOT):
  if env_ids is None:
    env_ids = torch.arange(env.num_envs, device=env.device)
  a = env.scene[asset_cfg.name]
  keys = ["x", "y", "z", "roll", "pitch", "yaw"]
  r = torch.tensor([pose_range.get(k, (0.0, 0.0)) for k in keys], device=env.device)
  ps = sample_uniform(r[:, 0], r[:, 1], (len(env_ids), 6), env.device)
  rs = a.data.default_root_state[env_ids].clone()
  pos = rs[:, 0:3] + ps[:, 0:3] + env.scene.env_origins[env_ids]
  quat = quat_mul(rs[:, 3:7], quat_from_euler_xyz(ps[:, 3], ps[:, 4], ps[:, 5]))
  vr = torch.tensor([(velocity_range or {}).get(k, (0.0, 0.0)) for k in keys], device=env.device)
  vel = rs[:, 7:13] + sample_uniform(vr[:, 0], vr[:, 1], (len(env_ids), 6), env.device)
  a.write_root_link_pose_to_sim(torch.cat([pos, quat], dim=-1), env_ids=env_ids)
  a.write_root_link_velocity_to_sim(vel, env_ids=env_ids)


def reset_joints_by_offset(env, env_ids, position_range, velocity_range, asset_cfg=_ROBOT):
  if env_ids is None:
    env_ids = torch.arange(env.num_envs, device=env.device)
  a = env.scene[asset_cfg.name]
  jp = a.data.default_joint_pos[env_ids][:, asset_cfg.joint_ids].clone()
  jp += sample_uniform(*position_range, jp.shape, env.device)
  lim = a.data.soft_joint_pos_limits[env_ids][:, asset_cfg.joint_ids]
  jp = jp.clamp_(lim[..., 0], lim[..., 1])
  jv = a.data.default_joint_vel[env_ids][:, asset_cfg.joint_ids].clone()
  jv += sample_uniform(*velocity_range, jv.shape, env.device)
  jid = asset_cfg.joint_ids
  if isinstance(jid, list):
    jid = torch.tensor(jid, device=env.device)
  a.write_joint_state_to_sim(jp.view(len(env_ids), -1), jv.view(len(env_ids), -1),
                             env_ids=env_ids, joint_ids=jid)


def push_by_setting_velocity(env, env_ids, velocity_range: dict, asset_cfg=_ROBOT):
  a = env.scene[asset_cfg.name]
  vel = a.data.root_link_vel_w[env_ids]
  keys = ["x", "y", "z", "roll", "pitch", "yaw"]
  r = torch.tensor([velocity_range.get(k, (0.0, 0.0)) for k in keys], device=env.device)
  vel += sample_uniform(r[:, 0], r[:, 1], vel.shape, env.device)
  a.write_root_link_velocity_to_sim(vel, env_ids=env_ids)


# ---- sync-free (mask) variants used by the graph-captured env step.  They draw randoms
# for every env and commit them only where `mask` is set (same distributions as the
# index-based versions above; RNG streams differ, as they do from the reference anyway).
_CACHE: dict = {}


def _range_tensor(spec, device):
  key = (tuple(sorted(spec.items())) if isinstance(spec, dict) else tuple(spec), str(device))
  if key not in _CACHE:
    keys = ["x", "y", "z", "roll", "pitch", "yaw"]
    vals = [spec.get(k, (0.0, 0.0)) for k in keys] if isinstance(spec, dict) else [spec]
    _CACHE[key] = torch.tensor(vals, device=device, dtype=torch.float32)
  return _CACHE[key]


def _joint_ids_tensor(ids, device):
  if isinstance(ids, (slice, torch.Tensor)):
    return ids
  key = ("jid", tuple(ids), str(device))
  if key not in _CACHE:
    _CACHE[key] = torch.tensor(ids, device=device, dtype=torch.long)
  return _CACHE[key]


def _reset_root_state_uniform_masked(env, mask, pose_range, velocity_range=None, asset_cfg=_ROBOT):
  a = env.scene[asset_cfg.name]
  n = env.num_envs
  r = _range_tensor(pose_range, env.device)
  ps = torch.rand(n, 6, device=env.device) * (r[:, 1] - r[:, 0]) + r[:, 0]
  rs = a.data.default_root_state
  pos = rs[:, 0:3] + ps[:, 0:3] + env.scene.env_origins
  quat = quat_mul(rs[:, 3:7], quat_from_euler_xyz(ps[:, 3], ps[:, 4], ps[:, 5]))
  vr = _range_tensor(velocity_range or {}, env.device)
  vel = rs[:, 7:13] + torch.rand(n, 6, device=env.device) * (vr[:, 1] - vr[:, 0]) + vr[:, 0]
  a.data.write_root_pose_masked(torch.cat([pos, quat], dim=-1), mask)
  a.data.write_root_velocity_masked(vel, mask)


def _reset_joints_by_offset_masked(env, mask, position_range, velocity_range, asset_cfg=_ROBOT):
  a = env.scene[asset_cfg.name]
  jid = _joint_ids_tensor(asset_cfg.joint_ids, env.device)
  jp = a.data.default_joint_pos[:, jid]
  jp = jp + torch.rand_like(jp) * (position_range[1] - position_range[0]) + position_range[0]
  lim = a.data.soft_joint_pos_limits[:, jid]
  jp = torch.minimum(torch.maximum(jp, lim[..., 0]), lim[..., 1])
  jv = a.data.default_joint_vel[:, jid]
  jv = jv + torch.rand_like(jv) * (velocity_range[1] - velocity_range[0]) + velocity_range[0]
  a.data.write_joint_state_masked(jp, jv, mask, None if isinstance(jid, slice) else jid)


def _push_by_setting_velocity_masked(env, mask, velocity_range, asset_cfg=_ROBOT):
  a = env.scene[asset_cfg.name]
  vel = a.data.root_link_vel_w
  r = _range_tensor(velocity_range, env.device)
  vel = vel + torch.rand_like(vel) * (r[:, 1] - r[:, 0]) + r[:, 0]
  a.data.write_root_velocity_masked(vel, mask)


reset_root_state_uniform.masked = _reset_root_state_uniform_masked
reset_joints_by_offset.masked = _reset_joints_by_offset_masked
push_by_setting_velocity.masked = _push_by_setting_velocity_masked


# `envs/mdp/events.py:264-289`: entity type, address use and default axes per field.
FIELD_SPECS = {
  "dof_armature": ("dof", None, None), "dof_frictionloss": ("dof", None, None),
  "dof_damping": ("dof", None, None),
  "jnt_range": ("joint", None, None), "jnt_stiffness": ("joint", None, None),
  "body_mass": ("body", None, None), "body_ipos": ("body", [0, 1, 2], None),
  "body_iquat": ("body", [0, 1, 2, 3], None), "body_inertia": ("body", None, None),
  "body_pos": ("body", [0, 1, 2], None), "body_quat": ("body", [0, 1, 2, 3], None),
  "geom_friction": ("geom", [0], [0, 1, 2]), "geom_pos": ("geom", [0, 1, 2], None),
  "geom_quat": ("geom", [0, 1, 2, 3], None), "geom_rgba": ("geom", [0, 1, 2, 3], None),
  "site_pos": ("site", [0, 1, 2], None), "site_quat": ("site", [0, 1, 2, 3], None),
  "qpos0": ("qpos", None, None),
}


def _sample_distribution(distribution, lo, hi, shape, device):
  if distribution == "uniform":
    return sample_uniform(lo, hi, shape, device)
  if distribution == "log_uniform":
    return torch.exp(sample_uniform(math.log(lo), math.log(hi), shape, device))
  if distribution == "gaussian":
    return torch.randn(shape, device=device) * hi + lo
  raise ValueError(f"Unknown distribution: {distribution}")


def randomize_field(env, env_ids, field: str, ranges, distribution: str = "uniform",
                    operation: str = "abs", asset_cfg=None, axes=None):
  """Unified model-field randomization (`envs/mdp/events.py:292-354`).  `ranges` is
  (lo, hi) for every target axis or {axis: (lo, hi)}; "add"/"scale" start from the
  stored default (no accumulation across resets), "abs" keeps non-target axes.  The
  field must have been expanded (EventManager does that for domain_randomization terms)."""
  if field not in FIELD_SPECS:
    raise ValueError(f"Unknown field '{field}'. Supported fields: {list(FIELD_SPECS.keys())}")
  etype, default_axes, valid_axes = FIELD_SPECS[field]
  asset_cfg = asset_cfg or _ROBOT
  a = env.scene[asset_cfg.name]
  if env_ids is None:
    env_ids = torch.arange(env.num_envs, device=env.device)
  env_ids = env_ids.to(env.device, dtype=torch.long)
  t = getattr(env.sim.model, field)
  ix = a.indexing
  ids = {"dof": lambda: ix.joint_v_adr[asset_cfg.joint_ids],
         "qpos": lambda: ix.joint_q_adr[asset_cfg.joint_ids],
         "joint": lambda: ix.joint_ids[asset_cfg.joint_ids],
         "body": lambda: ix.body_ids[asset_cfg.body_ids],
         "geom": lambda: ix.geom_ids[asset_cfg.geom_ids],
         "site": lambda: ix.site_ids[asset_cfg.site_ids]}[etype]()
  field_ndim = t.dim() - 1
  if axes is not None:
    target = list(axes)
  elif isinstance(ranges, dict):
    target = list(ranges.keys())
  elif default_axes is not None:
    target = list(default_axes)
  else:
    target = list(range(t.shape[-1])) if field_ndim > 1 else [0]
  if valid_axes is not None and set(target) - set(valid_axes):
    raise ValueError(f"Invalid axes {set(target) - set(valid_axes)} for field. Valid axes: {valid_axes}")
  if isinstance(ranges, dict):
    missing = set(target) - set(ranges.keys())
    if missing:
      raise ValueError(f"Missing ranges for axes {missing} in field '{field}'. Required axes: {target}")
    axis_ranges = {ax: ranges[ax] for ax in target}
  elif isinstance(ranges, (tuple, list)):
    axis_ranges = {ax: tuple(ranges) for ax in target}
  else:
    raise TypeError(f"ranges must be tuple or dict, got {type(ranges)}")
  eg, ig = torch.meshgrid(env_ids, ids, indexing="ij")
  cur = t[eg, ig]
  if operation in ("scale", "add"):
    base = env.sim.get_default_field(field)[ids].unsqueeze(0).expand_as(cur)
  else:
    base = cur
  if operation == "scale":
    rnd = torch.ones_like(base)
  elif operation == "add":
    rnd = torch.zeros_like(base)
  elif operation == "abs":
    rnd = base.clone()
  else:
    raise ValueError(f"Unknown operation: {operation}")
  for ax in target:
    lo, hi = axis_ranges[ax]
    if cur.dim() > 2:
      rnd[..., ax] = _sample_distribution(distribution, lo, hi, cur.shape[:-1], env.device)
    else:
      rnd = _sample_distribution(distribution, lo, hi, cur.shape, env.device)
  if operation == "add":
    t[eg, ig] = base + rnd
  elif operation == "scale":
    t[eg, ig] = base * rnd
  else:
    t[eg, ig] = rnd


def randomize_terrain(env, env_ids):
  """`envs/mdp/events.py:26-37`: a random sub-terrain (level row and type column) for each
  resetting env (play / evaluation mode)."""
  terrain = env.scene.terrain
  if terrain is None:
    return
  if env_ids is None:
    env_ids = torch.arange(env.num_envs, device=env.device)
  terrain.randomize_env_origins(env_ids)


def _randomize_terrain_masked(env, mask):
  terrain = env.scene.terrain
  if terrain is not None:
    terrain.randomize_env_origins_masked(mask)


randomize_terrain.masked = _randomize_terrain_masked


def randomize_encoder_bias(env, env_ids, bias_range, asset_cfg=_ROBOT):
  """`envs/mdp/events.py:709-745`: per-env joint encoder offsets (read by
  joint_pos_rel(biased=True) and subtracted by the joint-position action)."""
  a = env.scene[asset_cfg.name]
  if env_ids is None:
    env_ids = torch.arange(env.num_envs, device=env.device)
  jid = asset_cfg.joint_ids
  nj = a.num_joints if isinstance(jid, slice) else len(jid)
  b = sample_uniform(bias_range[0], bias_range[1], (len(env_ids), nj), env.device)
  if isinstance(jid, slice):
    a.data.encoder_bias[env_ids] = b
  else:
    a.data.encoder_bias[env_ids[:, None], torch.as_tensor(jid, device=env.device)] = b


# =========================================================================== commands
@dataclass(kw_only=True)
class UniformVelocityCommandCfg(CommandTermCfg):
  asset_name: str = "robot"
  heading_command: bool = False
  heading_control_stiffness: float = 1.0
  rel_standing_envs: float = 0.0
  rel_heading_envs: float = 1.0
  init_velocity_prob: float = 0.0

  @dataclass
  class Ranges:
    lin_vel_x: tuple[float, float] = (-1.0, 1.0)
    lin_vel_y: tuple[float, float] = (-1.0, 1.0)
    ang_vel_z: tuple[float, float] = (-1.0, 1.0)
    heading: tuple[float, float] | None = None

  ranges: "UniformVelocityCommandCfg.Ranges" = field(default_factory=lambda: UniformVelocityCommandCfg.Ranges())

  def __post_init__(self):
    self.class_type = UniformVelocityCommand


class UniformVelocityCommand(CommandTerm):
  """`tasks/velocity/mdp/velocity_command.py:25-101`."""

  def __init__(self, cfg: UniformVelocityCommandCfg, env):
    super().__init__(cfg, env)
    self.robot = env.scene[cfg.asset_name]
    n = self.num_envs
    self.vel_command_b = torch.zeros(n, 3, device=self.device)
    self.heading_target = torch.zeros(n, device=self.device)
    self.heading_error = torch.zeros(n, device=self.device)
    self.is_heading_env = torch.zeros(n, dtype=torch.bool, device=self.device)
    self.is_standing_env = torch.zeros_like(self.is_heading_env)
    self.metrics["error_vel_xy"] = torch.zeros(n, device=self.device)
    self.metrics["error_vel_yaw"] = torch.zeros(n, device=self.device)

  @property
  def command(self):
    return self.vel_command_b

  def _update_metrics(self):
    steps = self.cfg.resampling_time_range[1] / self._env.step_dt
    v = self.robot.data.root_link_lin_vel_b
    w = self.robot.data.root_link_ang_vel_b
    self.metrics["error_vel_xy"] += torch.norm(self.vel_command_b[:, :2] - v[:, :2], dim=-1) / steps
    self.metrics["error_vel_yaw"] += torch.abs(self.vel_command_b[:, 2] - w[:, 2]) / steps

  def _resample_command(self, env_ids):
    r = torch.empty(len(env_ids), device=self.device)
    rg = self.cfg.ranges
    self.vel_command_b[env_ids, 0] = r.uniform_(*rg.lin_vel_x)
    self.vel_command_b[env_ids, 1] = r.uniform_(*rg.lin_vel_y)
    self.vel_command_b[env_ids, 2] = r.uniform_(*rg.ang_vel_z)
    if self.cfg.heading_command:
      self.heading_target[env_ids] = r.uniform_(*rg.heading)
      self.is_heading_env[env_ids] = r.uniform_(0.0, 1.0) <= self.cfg.rel_heading_envs
    self.is_standing_env[env_ids] = r.uniform_(0.0, 1.0) <= self.cfg.rel_standing_envs

  def _resample_command_masked(self, mask):
    n = self.num_envs
    rg = self.cfg.ranges
    u = torch.rand(n, 6, device=self.device)
    new = torch.stack([u[:, 0] * (rg.lin_vel_x[1] - rg.lin_vel_x[0]) + rg.lin_vel_x[0],
                       u[:, 1] * (rg.lin_vel_y[1] - rg.lin_vel_y[0]) + rg.lin_vel_y[0],
                       u[:, 2] * (rg.ang_vel_z[1] - rg.ang_vel_z[0]) + rg.ang_vel_z[0]], dim=1)
    self.vel_command_b.copy_(torch.where(mask.unsqueeze(1), new, self.vel_command_b))
    if self.cfg.heading_command:
      ht = u[:, 3] * (rg.heading[1] - rg.heading[0]) + rg.heading[0]
      self.heading_target.copy_(torch.where(mask, ht, self.heading_target))
      self.is_heading_env.copy_(torch.where(mask, u[:, 4] <= self.cfg.rel_heading_envs,
                                            self.is_heading_env))
    self.is_standing_env.copy_(torch.where(mask, u[:, 5] <= self.cfg.rel_standing_envs,
                                           self.is_standing_env))

  def _update_command(self):
    if self.cfg.heading_command:
      self.heading_error.copy_(wrap_to_pi(self.heading_target - self.robot.data.heading_w))
      lo, hi = self.cfg.ranges.ang_vel_z
      hc = torch.clip(self.cfg.heading_control_stiffness * self.heading_error, min=lo, max=hi)
      self.vel_command_b[:, 2] = torch.where(self.is_heading_env, hc, self.vel_command_b[:, 2])
    self.vel_command_b.masked_fill_(self.is_standing_env.unsqueeze(1), 0.0)


# =========================================================================== curriculum
def _terrain_moves(env, ids, command_name, asset_name="robot"):
  """`tasks/velocity/mdp/curriculums.py:30-64`: walked farther than half a patch -> up;
  less than half the commanded distance over an episode -> down."""
  terrain = env.scene.terrain
  root = env.scene[asset_name].data.root_link_pos_w[ids, :2]
  dist = torch.norm(root - env.scene.env_origins[ids, :2], dim=1)
  up = dist > terrain.size[0] / 2
  cmd = env.command_manager.get_command(command_name)[ids, :2]
  down = (dist < torch.norm(cmd, dim=1) * env.max_episode_length_s * 0.5) & ~up
  return up, down


def terrain_levels_vel(env, env_ids, command_name: str, asset_cfg=None):
  """Terrain-level curriculum (`curriculums.py:30-64`) for the resetting envs env_ids;
  returns the mean terrain level."""
  terrain = env.scene.terrain
  up, down = _terrain_moves(env, env_ids, command_name, asset_cfg.name if asset_cfg else "robot")
  terrain.update_env_origins(env_ids, up, down)
  return torch.mean(terrain.terrain_levels.float())


def _terrain_levels_vel_masked(env, mask, command_name: str, asset_cfg=None):
  """The same over a reset mask (sync-free / graph-captured step): one HIP kernel on the
  GPU (`Terrain.update_env_origins_native`), the torch form elsewhere."""
  terrain = env.scene.terrain
  name = asset_cfg.name if asset_cfg else "robot"
  cmd = env.command_manager.get_command(command_name)
  # the kernel reads the command rows with a stride of 3 (lin_x, lin_y, ang_z)
  if (terrain.env_origins.is_cuda and cmd.is_contiguous() and cmd.dtype == torch.float32
      and cmd.dim() == 2 and cmd.shape[1] == 3):
    root = int(env.scene[name].indexing.root_body_id)
    terrain.update_env_origins_native(mask.contiguous(), env.sim.data.xpos, root, cmd,
                                      env.max_episode_length_s)
    return terrain.mean_level
  up, down = _terrain_moves(env, slice(None), command_name, name)
  terrain.update_env_origins_masked(mask, up, down)
  return terrain.mean_level


terrain_levels_vel.masked = _terrain_levels_vel_masked


def commands_vel(env, env_ids, command_name: str, velocity_stages: list):
  cfg = env.command_manager.get_term(command_name).cfg
  for st in velocity_stages:
    if env.common_step_counter > st["step"]:
      for k in ("lin_vel_x", "lin_vel_y", "ang_vel_z"):
        if st.get(k) is not None:
          setattr(cfg.ranges, k, st[k])
  r = cfg.ranges
  return {"lin_vel_x_min": r.lin_vel_x[0], "lin_vel_x_max": r.lin_vel_x[1],
          "lin_vel_y_min": r.lin_vel_y[0], "lin_vel_y_max": r.lin_vel_y[1],
          "ang_vel_z_min": r.ang_vel_z[0], "ang_vel_z_max": r.ang_vel_z[1]}
