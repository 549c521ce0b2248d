"""Fused HIP managers for the velocity tasks (include/mjx355_task.h, csrc/velocity_task.hip).

`FusedVelocityStep.build(env)` inspects a ManagerBasedRlEnv. If every action /
observation / reward / termination / command / event term is one the fused kernels
implement (the velocity-task term set of tasks/velocity/velocity_env_cfg.py:33-354 and
config/{g1,go1}/env_cfgs.py), it returns a step object whose `step(action)` runs the whole
env step as ~20 launches:
  task_action; decimation x (mjx_step + task_substep); task_post; mjx_reset(mask);
  task_reset; mjx_forward_masked(mask); task_observe.
Otherwise it returns None and the env keeps the torch manager path.

The kernels read and write the managers' own tensors (action histories, command state,
episode sums, termination flags, contact-sensor air times, swing-height peaks), so every
Python accessor of the reference API keeps working. Episode logs go to device scalars
that are exposed in `extras["log"]` under the reference's key names.
"""

from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import jump, mdp
from ._lib import MjxError, check, lib

MAXJ, MAXF, MAXT, MAXC = 64, 8, 24, 32
_f2 = ctypes.c_float * 2
_f62 = (ctypes.c_float * 2) * 6
_FP = ctypes.POINTER(ctypes.c_float)
_U8 = ctypes.POINTER(ctypes.c_uint8)
_I64 = ctypes.POINTER(ctypes.c_int64)
_U64 = ctypes.POINTER(ctypes.c_uint64)


class TaskDesc(ctypes.Structure):
  """ctypes mirror of mjxTaskDesc (include/mjx355_task.h)."""
  _fields_ = [
    ("nworld", ctypes.c_int), ("nq", ctypes.c_int), ("nv", ctypes.c_int), ("nu", ctypes.c_int),
    ("nsensordata", ctypes.c_int), ("nbody", ctypes.c_int), ("nsite", ctypes.c_int),
    ("qpos", _FP), ("qvel", _FP), ("ctrl", _FP), ("time", _FP),
    ("xpos", _FP), ("xquat", _FP), ("cvel", _FP), ("subtree_com", _FP), ("site_xpos", _FP),
    ("sensordata", _FP),
    ("root_body", ctypes.c_int), ("free_q_adr", ctypes.c_int), ("free_v_adr", ctypes.c_int),
    ("njoint", ctypes.c_int),
    ("joint_q_adr", ctypes.c_int * MAXJ), ("joint_v_adr", ctypes.c_int * MAXJ),
    ("ctrl_of_action", ctypes.c_int * MAXJ), ("target_of_action", ctypes.c_int * MAXJ),
    ("action_scale", ctypes.c_float * MAXJ), ("action_offset", ctypes.c_float * MAXJ),
    ("default_joint_pos", ctypes.c_float * MAXJ),
    ("soft_lo", ctypes.c_float * MAXJ), ("soft_hi", ctypes.c_float * MAXJ),
    ("std_standing", ctypes.c_float * MAXJ), ("std_walking", ctypes.c_float * MAXJ),
    ("std_running", ctypes.c_float * MAXJ),
    ("default_root_state", ctypes.c_float * 13), ("env_origins", _FP),
    ("nfeet", ctypes.c_int), ("foot_site", ctypes.c_int * MAXF),
    ("foot_site_body", ctypes.c_int * MAXF), ("feet_found_adr", ctypes.c_int * MAXF),
    ("feet_force_adr", ctypes.c_int * MAXF),
    ("imu_lin_vel_adr", ctypes.c_int), ("imu_ang_vel_adr", ctypes.c_int),
    ("angmom_adr", ctypes.c_int), ("selfcol_found_adr", ctypes.c_int),
    ("nillegal", ctypes.c_int), ("illegal_found_adr", ctypes.c_int * MAXC),
    ("orient_body", ctypes.c_int),
    ("step_dt", ctypes.c_float), ("episode_length_s", ctypes.c_float),
    ("max_episode_length", ctypes.c_int),
    ("nreward", ctypes.c_int), ("reward_kind", ctypes.c_int * MAXT),
    ("reward_weight", ctypes.c_float * MAXT), ("reward_p0", ctypes.c_float * MAXT),
    ("reward_p1", ctypes.c_float * MAXT), ("reward_p2", ctypes.c_float * MAXT),
    ("ntermination", ctypes.c_int), ("termination_kind", ctypes.c_int * MAXT),
    ("termination_is_timeout", ctypes.c_int * MAXT), ("termination_p0", ctypes.c_float * MAXT),
    ("lin_vel_x", _f2), ("lin_vel_y", _f2), ("ang_vel_z", _f2), ("heading", _f2),
    ("resampling_time", _f2), ("rel_standing_envs", ctypes.c_float),
    ("rel_heading_envs", ctypes.c_float), ("heading_stiffness", ctypes.c_float),
    ("heading_command", ctypes.c_int),
    ("reset_pose_range", _f62), ("reset_vel_range", _f62),
    ("reset_joint_pos_range", _f2), ("reset_joint_vel_range", _f2),
    ("has_push", ctypes.c_int), ("push_interval", _f2), ("push_vel_range", _f62),
    ("npolicy", ctypes.c_int), ("ncritic", ctypes.c_int), ("critic_extras", ctypes.c_int),
    ("noise_lin_vel", ctypes.c_float), ("noise_ang_vel", ctypes.c_float),
    ("noise_gravity", ctypes.c_float), ("noise_joint_pos", ctypes.c_float),
    ("noise_joint_vel", ctypes.c_float), ("corrupt_policy", ctypes.c_int),
    ("seed", ctypes.c_uint64),
    ("action", _FP), ("prev_action", _FP), ("prev_prev_action", _FP), ("joint_pos_target", _FP),
    ("episode_length", _I64),
    ("command", _FP), ("heading_target", _FP), ("heading_error", _FP), ("cmd_time_left", _FP),
    ("is_heading_env", _U8), ("is_standing_env", _U8), ("command_counter", _I64),
    ("metric_err_xy", _FP), ("metric_err_yaw", _FP), ("push_time_left", _FP),
    ("episode_sums", _FP), ("step_reward", _FP), ("reward_buf", _FP),
    ("reset_buf", _U8), ("terminated", _U8), ("time_outs", _U8), ("term_dones", _U8),
    ("cur_air", _FP), ("last_air", _FP), ("cur_contact", _FP), ("last_contact", _FP),
    ("last_time", _FP), ("peak_heights", _FP), ("obs_policy", _FP), ("obs_critic", _FP),
    ("log_reward", _FP), ("log_termination", _FP), ("log_command", _FP), ("log_metric", _FP),
    ("step_counter", _U64),
    ("command_kind", ctypes.c_int), ("jump_target_height", ctypes.c_float),
    ("actuator_force", _FP), ("act_ctrl", ctypes.c_int * MAXJ), ("explosive_joints", ctypes.c_uint64),
    ("jump_peak", _FP), ("jump_initial", _FP), ("jump_initialized", _U8),
    ("landing_timer", _FP), ("was_in_air", _U8),
  ]


_REWARD_KIND = {
  mdp.track_linear_velocity: 0, mdp.track_angular_velocity: 1, mdp.flat_orientation: 2,
  mdp.body_angular_velocity_penalty: 4, mdp.angular_momentum_penalty: 5,
  mdp.joint_pos_limits: 6, mdp.action_rate_l2: 7, mdp.feet_air_time: 8,
  mdp.feet_clearance: 9, mdp.feet_slip: 11, mdp.soft_landing: 12, mdp.self_collision_cost: 13,
}
_METRIC_KEYS = ("Metrics/angular_momentum_mean", "Metrics/air_time_mean", "Metrics/peak_height_mean",
                "Metrics/slip_velocity_mean", "Metrics/landing_force_mean",
                "Metrics/peak_jump_height", "Metrics/jump_height", "Metrics/landing_success_rate")
NMETRIC = len(_METRIC_KEYS)
_METRIC_OF_KIND = {5: 0, 8: 1, 10: 2, 11: 3, 12: 4, 18: 1}
_EXCESSIVE_FORCE = (jump.excessive_landing_force,)
_POLICY = [("base_lin_vel", mdp.builtin_sensor), ("base_ang_vel", mdp.builtin_sensor),
           ("projected_gravity", mdp.projected_gravity), ("joint_pos", mdp.joint_pos_rel),
           ("joint_vel", mdp.joint_vel_rel), ("actions", mdp.last_action),
           ("command", mdp.generated_commands)]
_CRITIC_EXTRA = [("foot_height", mdp.foot_height), ("foot_air_time", mdp.foot_air_time),
                 ("foot_contact", mdp.foot_contact), ("foot_contact_forces", mdp.foot_contact_forces)]


class Unsupported(Exception):
  pass


def _need(cond, what):
  if not cond:
    raise Unsupported(what)


def _ptr(t: torch.Tensor, typ=_FP):
  _need(t.is_contiguous(), "non-contiguous tensor")
  return ctypes.cast(ctypes.c_void_p(t.data_ptr()), typ)


def _noise(cfg):
  n = cfg.noise
  if n is None:
    return 0.0
  _need(type(n).__name__ == "UniformNoiseCfg" and getattr(n, "operation", "add") == "add",
        "non-additive noise")
  _need(abs(n.n_min + n.n_max) < 1e-12, "asymmetric noise")
  return float(n.n_max)


def _range6(spec):
  keys = ["x", "y", "z", "roll", "pitch", "yaw"]
  return [tuple(map(float, (spec or {}).get(k, (0.0, 0.0)))) for k in keys]


class FusedVelocityStep:
  """One env step of a velocity task as fused HIP launches (see module docstring)."""

  @classmethod
  def build(cls, env):
    try:
      return cls(env)
    except Unsupported as e:
      env._fused_unsupported = str(e)
      return None

  def __init__(self, env):
    self.env = env
    L = lib()
    L.mjx_task_desc_size.restype = ctypes.c_size_t
    _need(L.mjx_task_desc_size() == ctypes.sizeof(TaskDesc), "mjxTaskDesc layout mismatch")
    L.mjx_task_create.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
    for n in ("mjx_task_action",):
      getattr(L, n).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    for n in ("mjx_task_substep", "mjx_task_post", "mjx_task_reset", "mjx_task_observe"):
      getattr(L, n).argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.mjx_task_destroy.argtypes = [ctypes.c_void_p]
    L.mjx_task_last_error.restype = ctypes.c_char_p
    self._L = L
    self._keep = []
    self._task = None
    self._desc = self._make_desc(env)
    self.upload()
    self._engine_air = self._track_air_time()

  # ------------------------------------------------------------------ descriptor
  def _make_desc(self, env):
    d = TaskDesc()
    robot, sens = self._base(d, env)
    scene, nj = env.scene, d.njoint
    # rewards
    rm = env.reward_manager
    _need(len(rm._term_names) <= MAXT, "too many reward terms")
    d.nreward = len(rm._term_names)
    feet_sensor = None
    site_names = None
    orient_body = -1
    self._metric_active = [False] * NMETRIC
    for k, (name, c) in enumerate(zip(rm._term_names, rm._term_cfgs)):
      f, p = c.func, c.params
      d.reward_weight[k] = float(c.weight)
      if isinstance(f, mdp.variable_posture):
        kind = 3
        d.reward_p0[k], d.reward_p1[k] = float(p.get("walking_threshold", 0.5)), float(p.get("running_threshold", 1.5))
        for j in range(nj):
          d.std_standing[j] = float(f.std_standing[j])
          d.std_walking[j] = float(f.std_walking[j])
          d.std_running[j] = float(f.std_running[j])
        _need(f.std_standing.numel() == nj, "posture over all joints")
      elif isinstance(f, mdp.feet_swing_height):
        kind = 10
        d.reward_p0[k], d.reward_p1[k] = float(p["target_height"]), float(p["command_threshold"])
        feet_sensor = self._same(feet_sensor, p["sensor_name"])
        site_names = self._same(site_names, tuple(p["asset_cfg"].site_names))
        self._peak = f.peak_heights
      else:
        _need(f in _REWARD_KIND, f"reward term {name}")
        kind = _REWARD_KIND[f]
        if kind in (0, 1):
          d.reward_p0[k] = float(p["std"])
          _need(p["command_name"] == "twist", "command name")
        elif kind in (2, 4):
          orient_body = self._orient(d, k, kind, p, robot, orient_body)
        elif kind == 5:
          d.angmom_adr = sens[p["sensor_name"]][0]
        elif kind == 8:
          d.reward_p0[k], d.reward_p1[k] = float(p["threshold_min"]), float(p["threshold_max"])
          d.reward_p2[k] = float(p["command_threshold"])
          feet_sensor = self._same(feet_sensor, p["sensor_name"])
        elif kind == 9:
          d.reward_p0[k], d.reward_p1[k] = float(p["target_height"]), float(p["command_threshold"])
          site_names = self._same(site_names, tuple(p["asset_cfg"].site_names))
        elif kind == 11:
          d.reward_p0[k] = float(p["command_threshold"])
          feet_sensor = self._same(feet_sensor, p["sensor_name"])
          site_names = self._same(site_names, tuple(p["asset_cfg"].site_names))
        elif kind == 12:
          d.reward_p0[k] = float(p.get("command_threshold", 0.05))
          d.reward_p1[k] = float(p.get("command_name") is None)  # ungated
          feet_sensor = self._same(feet_sensor, p["sensor_name"])
        elif kind == 13:
          s = scene[p["sensor_name"]]
          d.selfcol_found_adr = self._slot_adrs(s, "found")[0]
      d.reward_kind[k] = kind
      if c.weight != 0.0 and kind in _METRIC_OF_KIND:
        self._metric_active[_METRIC_OF_KIND[kind]] = True
    d.orient_body = orient_body
    self._feet(d, robot, feet_sensor, site_names)
    self._terminations(d, env)
    self._reward_buffers(d, env)
    # command
    cm = env.command_manager
    _need(list(getattr(cm, "_terms", {}).keys()) == ["twist"], "single 'twist' command")
    ct = cm._terms["twist"]
    _need(isinstance(ct, mdp.UniformVelocityCommand), "UniformVelocityCommand")
    cc = ct.cfg
    _need(float(getattr(cc, "init_velocity_prob", 0.0)) == 0.0, "init_velocity_prob")
    self._cmd_term = ct
    self._set_command_ranges(d, cc)
    d.rel_standing_envs, d.rel_heading_envs = float(cc.rel_standing_envs), float(cc.rel_heading_envs)
    d.heading_stiffness, d.heading_command = float(cc.heading_control_stiffness), int(bool(cc.heading_command))
    d.resampling_time[0], d.resampling_time[1] = map(float, cc.resampling_time_range)
    d.command, d.heading_target = _ptr(ct.vel_command_b), _ptr(ct.heading_target)
    d.heading_error, d.cmd_time_left = _ptr(ct.heading_error), _ptr(ct.time_left)
    d.is_heading_env, d.is_standing_env = _ptr(ct.is_heading_env, _U8), _ptr(ct.is_standing_env, _U8)
    d.command_counter = _ptr(ct.command_counter, _I64)
    d.metric_err_xy, d.metric_err_yaw = _ptr(ct.metrics["error_vel_xy"]), _ptr(ct.metrics["error_vel_yaw"])
    self._events(d, env)
    # observations
    om = env.observation_manager
    groups = om._group_obs_term_names
    _need(set(groups) == {"policy", "critic"}, "policy + critic groups")
    pol = list(zip(groups["policy"], om._group_obs_term_cfgs["policy"]))
    cri = list(zip(groups["critic"], om._group_obs_term_cfgs["critic"]))
    _need([(nme, c.func) for nme, c in pol] == _POLICY, "policy terms")
    base_c = [(nme, c.func) for nme, c in cri]
    _need(base_c[:7] == _POLICY and base_c[7:] in ([], _CRITIC_EXTRA), "critic terms")
    d.critic_extras = int(len(base_c) > 7)
    if d.critic_extras:
      _need(cri[8][1].params["sensor_name"] == feet_sensor and
            tuple(cri[7][1].params["asset_cfg"].site_names) == site_names, "critic feet terms")
    self._obs_noise(d, env, pol, cri, sens)
    for i in (5, 6):
      _need(pol[i][1].noise is None, "noise on actions/command")
    d.npolicy = 9 + 3 * nj + 3
    d.ncritic = d.npolicy + (6 * d.nfeet if d.critic_extras else 0)
    self._io(d, env)
    return d

  def _base(self, d, env):
    """Simulation pointers, the joint-position action, joints, default root state, origins."""
    sim, scene, m = env.sim, env.scene, env.sim.mj_model
    dev = torch.device(env.device)
    sd = sim.data
    n = env.num_envs
    d.nworld, d.nq, d.nv, d.nu = n, m.nq, m.nv, m.nu
    d.nsensordata, d.nbody, d.nsite = m.nsensordata, m.nbody, m.nsite
    for f in ("qpos", "qvel", "ctrl", "time", "xpos", "xquat", "cvel", "subtree_com",
              "site_xpos", "sensordata"):
      setattr(d, f, _ptr(getattr(sd, f)))
    # actions
    am = env.action_manager
    _need(len(am._terms) == 1, "one action term")
    (aterm,) = am._terms.values()
    _need(isinstance(aterm, mdp.JointPositionAction), "JointPositionAction only")
    robot = aterm._asset
    self._robot = robot
    rdata = robot.data
    _need(float(rdata.encoder_bias.abs().max()) == 0.0 if rdata.encoder_bias.numel() else True,
          "encoder bias")
    idx = robot.indexing
    nj = len(idx.joint_q_adr)
    _need(nj <= MAXJ and aterm.action_dim == nj, "action dim == actuated joints")
    d.root_body = int(idx.root_body_id)
    d.free_q_adr, d.free_v_adr = int(idx.free_joint_q_adr[0]), int(idx.free_joint_v_adr[0])
    d.njoint = nj
    jq, jv = idx.joint_q_adr.tolist(), idx.joint_v_adr.tolist()
    for j in range(nj):
      d.joint_q_adr[j], d.joint_v_adr[j] = jq[j], jv[j]
    jids = aterm._joint_ids.tolist()
    act_local = robot._act_joint_local_t.tolist()
    ctrl_ids = idx.ctrl_ids.tolist()
    scale = aterm._scale if isinstance(aterm._scale, float) else None
    for k, jk in enumerate(jids):
      a = act_local.index(jk)
      d.ctrl_of_action[k] = ctrl_ids[a]
      d.target_of_action[k] = jk
      d.action_scale[k] = scale if scale is not None else float(aterm._scale[0, k])
      off = aterm._offset
      d.action_offset[k] = off if isinstance(off, float) else float(off[0, k])
    _need(rdata.joint_pos_target.shape[1] == nj, "joint target width")
    _need(torch.all(rdata.default_joint_pos == rdata.default_joint_pos[:1]).item(),
          "per-env default joint pos")
    dj = rdata.default_joint_pos[0].tolist()
    lim = rdata.soft_joint_pos_limits[0].tolist()
    for j in range(nj):
      d.default_joint_pos[j] = dj[j]
      d.soft_lo[j], d.soft_hi[j] = lim[j]
    _need(torch.all(rdata.default_joint_vel == 0).item(), "nonzero default joint vel")
    rs = rdata.default_root_state[0].tolist()
    for i in range(13):
      d.default_root_state[i] = rs[i]
    origins = scene.env_origins.contiguous()
    self._keep.append(origins)
    d.env_origins = _ptr(origins)
    # sensors
    sens = {name: (int(m.sensor_adr[i]), int(m.sensor_dim[i])) for i, name in enumerate(m.names["sensor"])}
    d.imu_lin_vel_adr = d.imu_ang_vel_adr = d.angmom_adr = d.selfcol_found_adr = -1
    return robot, sens

  def _orient(self, d, k, kind, p, robot, orient_body):
    ids = p.get("asset_cfg").body_ids if p.get("asset_cfg") is not None else slice(None)
    body = self._body_of(robot, ids)
    if kind == 2:
      d.reward_p0[k] = float(p["std"])
    if body is not None:
      return self._same(orient_body if orient_body >= 0 else None, body)
    _need(kind == 2, "body_ang_vel needs a body")
    return orient_body

  def _feet(self, d, robot, feet_sensor, site_names):
    """Feet: contact-sensor slots (found / force, air-time buffers) and foot sites."""
    scene, n, dev = self.env.scene, self.env.num_envs, torch.device(self.env.device)
    idx = robot.indexing
    _need(feet_sensor is not None and site_names is not None, "feet terms")
    fs = scene[feet_sensor]
    found, force = self._slot_adrs(fs, "found"), self._slot_adrs(fs, "force")
    _need(len(found) == len(site_names) <= MAXF and fs._air is not None, "feet sensor layout")
    d.nfeet = len(found)
    site_ids, _ = robot.find_sites(list(site_names), preserve_order=True)
    sid_global = idx.site_ids.tolist()
    sbody = idx.site_body_ids.tolist()
    for i in range(d.nfeet):
      d.foot_site[i] = sid_global[site_ids[i]]
      d.foot_site_body[i] = sbody[site_ids[i]]
      d.feet_found_adr[i], d.feet_force_adr[i] = found[i], force[i]
    air = fs._air
    for key, attr in (("current_air_time", "cur_air"), ("last_air_time", "last_air"),
                      ("current_contact_time", "cur_contact"), ("last_contact_time", "last_contact"),
                      ("last_time", "last_time")):
      setattr(d, attr, _ptr(air[key]))
    self._feet_sensor = fs
    if not hasattr(self, "_peak"):
      self._peak = torch.zeros(n, d.nfeet, device=dev)
    d.peak_heights = _ptr(self._peak)

  def _terminations(self, d, env):
    scene, n, dev = env.scene, env.num_envs, torch.device(env.device)
    tm = env.termination_manager
    d.ntermination = len(tm._term_names)
    for k, (name, c) in enumerate(zip(tm._term_names, tm._term_cfgs)):
      if c.func is mdp.time_out:
        d.termination_kind[k] = 0
      elif c.func is mdp.bad_orientation:
        d.termination_kind[k] = 1
        d.termination_p0[k] = float(c.params["limit_angle"])
      elif c.func is mdp.root_height_below_minimum:
        d.termination_kind[k] = 3
        _need(c.params.get("asset_cfg") is None or c.params["asset_cfg"].name == "robot", "root height asset")
        d.termination_p0[k] = float(c.params["minimum_height"])
      elif c.func in _EXCESSIVE_FORCE:
        d.termination_kind[k] = 4
        _need(scene[c.params["sensor_name"]] is self._feet_sensor, "impact sensor is the feet sensor")
        d.termination_p0[k] = float(c.params.get("force_threshold", 2500.0))
      elif c.func is mdp.illegal_contact:
        d.termination_kind[k] = 2
        adrs = self._slot_adrs(scene[c.params["sensor_name"]], "found")
        _need(len(adrs) <= MAXC, "illegal contact slots")
        d.nillegal = len(adrs)
        for i, a in enumerate(adrs):
          d.illegal_found_adr[i] = a
      else:
        raise Unsupported(f"termination {name}")
      d.termination_is_timeout[k] = int(bool(c.time_out))
    self._term_dones = torch.zeros(max(d.ntermination, 1), n, dtype=torch.bool, device=dev)
    for k, name in enumerate(tm._term_names):
      tm._term_dones[name] = self._term_dones[k]
    d.term_dones = _ptr(self._term_dones, _U8)
    d.terminated = _ptr(tm._terminated_buf, _U8)
    d.time_outs = _ptr(tm._truncated_buf, _U8)
    self.reset_buf = torch.zeros(n, dtype=torch.bool, device=dev)
    d.reset_buf = _ptr(self.reset_buf, _U8)
    self._term_names = list(tm._term_names)

  def _reward_buffers(self, d, env):
    """Episode sums as rows of one [nreward, n] tensor; step reward / reward buffers; timing."""
    rm, n, dev = env.reward_manager, env.num_envs, torch.device(env.device)
    self._episode_sums = torch.zeros(max(d.nreward, 1), n, device=dev)
    for k, name in enumerate(rm._term_names):
      self._episode_sums[k].copy_(rm._episode_sums[name])
      rm._episode_sums[name] = self._episode_sums[k]
    d.episode_sums = _ptr(self._episode_sums)
    d.step_reward, d.reward_buf = _ptr(rm._step_reward), _ptr(rm._reward_buf)
    # timing
    d.step_dt, d.episode_length_s = float(env.step_dt), float(env.max_episode_length_s)
    # play configs use a 1e9 s episode: clamp into the descriptor's int32 (never reached)
    d.max_episode_length = min(int(env.max_episode_length), 2 ** 31 - 1)
    _need(env.episode_length_buf.dtype == torch.int64, "episode length dtype")
    d.episode_length = _ptr(env.episode_length_buf, _I64)
    self._reward_names = list(rm._term_names)

  def _events(self, d, env):
    """Reset events (root state + joint offsets) and the optional push interval event."""
    n, dev = env.num_envs, torch.device(env.device)
    em = env.event_manager
    reset_terms = em._mode_term_cfgs.get("reset", [])
    funcs = [c.func for c in reset_terms]
    _need(funcs == [mdp.reset_root_state_uniform, mdp.reset_joints_by_offset], "reset events")
    rb, rj = reset_terms
    for i, (lo, hi) in enumerate(_range6(rb.params["pose_range"])):
      d.reset_pose_range[i][0], d.reset_pose_range[i][1] = lo, hi
    for i, (lo, hi) in enumerate(_range6(rb.params.get("velocity_range"))):
      d.reset_vel_range[i][0], d.reset_vel_range[i][1] = lo, hi
    _need(rj.params.get("asset_cfg") is None or isinstance(rj.params["asset_cfg"].joint_ids, slice),
          "reset joints over all joints")
    d.reset_joint_pos_range[0], d.reset_joint_pos_range[1] = map(float, rj.params["position_range"])
    d.reset_joint_vel_range[0], d.reset_joint_vel_range[1] = map(float, rj.params["velocity_range"])
    inter = em._mode_term_cfgs.get("interval", [])
    _need(len(inter) <= 1, "one interval event")
    if inter:
      c = inter[0]
      _need(c.func is mdp.push_by_setting_velocity and not c.is_global_time, "push event")
      d.has_push = 1
      d.push_interval[0], d.push_interval[1] = map(float, c.interval_range_s)
      for i, (lo, hi) in enumerate(_range6(c.params["velocity_range"])):
        d.push_vel_range[i][0], d.push_vel_range[i][1] = lo, hi
      d.push_time_left = _ptr(em._interval_time_left[0])
    else:
      self._dummy_push = torch.zeros(n, device=dev)
      d.push_time_left = _ptr(self._dummy_push)
    _need(set(em._mode_term_cfgs) <= {"reset", "interval", "startup"}, "event modes")

  def _obs_noise(self, d, env, pol, cri, sens):
    """Shared proprioceptive head (lin vel, ang vel, gravity, joint pos / vel): sensors and
    policy noise; no clip / scale anywhere, no critic corruption."""
    om = env.observation_manager
    for _, c in pol + cri:
      _need(not c.clip and c.scale is None, "obs clip/scale")
    _need(pol[0][1].params["sensor_name"] == cri[0][1].params["sensor_name"], "sensor")
    d.imu_lin_vel_adr = sens[pol[0][1].params["sensor_name"]][0]
    d.imu_ang_vel_adr = sens[pol[1][1].params["sensor_name"]][0]
    for nme, c in cri:
      _need(c.noise is None or not om.cfg["critic"].enable_corruption, "critic noise")
    d.corrupt_policy = int(bool(om.cfg["policy"].enable_corruption))
    d.noise_lin_vel, d.noise_ang_vel, d.noise_gravity = (_noise(pol[i][1]) for i in range(3))
    d.noise_joint_pos, d.noise_joint_vel = _noise(pol[3][1]), _noise(pol[4][1])

  def _io(self, d, env):
    """Observation buffers, action pointers, seed, log scalars."""
    om, am, n, dev = env.observation_manager, env.action_manager, env.num_envs, torch.device(env.device)
    rdata = self._robot.data
    _need(om.group_obs_dim["policy"] == (d.npolicy,) and om.group_obs_dim["critic"] == (d.ncritic,),
          "observation dims")
    self.obs = {"policy": torch.zeros(n, d.npolicy, device=dev),
                "critic": torch.zeros(n, d.ncritic, device=dev)}
    d.obs_policy, d.obs_critic = _ptr(self.obs["policy"]), _ptr(self.obs["critic"])
    d.action, d.prev_action = _ptr(am._action), _ptr(am._prev_action)
    d.prev_prev_action, d.joint_pos_target = _ptr(am._prev_prev_action), _ptr(rdata.joint_pos_target)
    d.seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    # logs
    self.log_reward = torch.zeros(max(d.nreward, 1), device=dev)
    self.log_term = torch.zeros(max(d.ntermination, 1), device=dev)
    self.log_cmd = torch.zeros(2, device=dev)
    self.log_metric = torch.zeros(NMETRIC, device=dev)
    self.step_counter = torch.zeros(1, dtype=torch.int64, device=dev)
    d.log_reward, d.log_termination = _ptr(self.log_reward), _ptr(self.log_term)
    d.log_command, d.log_metric = _ptr(self.log_cmd), _ptr(self.log_metric)
    d.step_counter = _ptr(self.step_counter, _U64)
    self._keep.extend([self._term_dones, self.reset_buf, self._episode_sums])
    return d

  @staticmethod
  def _same(prev, new):
    _need(prev is None or prev == new, "terms disagree on feet/body")
    return new

  @staticmethod
  def _body_of(robot, ids):
    if isinstance(ids, slice) or ids is None or len(ids) == 0:
      return None
    ids = ids.tolist() if isinstance(ids, torch.Tensor) else list(ids)
    _need(len(ids) == 1, "single body")
    return int(robot.indexing.body_ids[ids[0]])

  @staticmethod
  def _slot_adrs(sensor, field):
    _need(getattr(sensor, "_num_slots", 1) == 1, "one contact slot per primary")
    return [adr for _, f, adr, _ in sensor._slots if f == field]

  @staticmethod
  def _set_command_ranges(d, cc):
    r = cc.ranges
    d.lin_vel_x[0], d.lin_vel_x[1] = map(float, r.lin_vel_x)
    d.lin_vel_y[0], d.lin_vel_y[1] = map(float, r.lin_vel_y)
    d.ang_vel_z[0], d.ang_vel_z[1] = map(float, r.ang_vel_z)
    hd = r.heading if r.heading is not None else (0.0, 0.0)
    d.heading[0], d.heading[1] = map(float, hd)

  def _track_air_time(self) -> bool:
    """Hand the feet air-time buffers to the engine (mjx_sim_track_air_time): phase C of
    every substep then updates them, replacing the per-substep task kernel.  False with an
    older engine build (A/B runs), which keeps k_substep."""
    sim, d = self.env.sim, self._desc
    tl = lib()
    if not hasattr(tl, "mjx_sim_track_air_time") or d.nfeet == 0:
      return False
    adr = (ctypes.c_int32 * d.nfeet)(*[d.feet_found_adr[i] for i in range(d.nfeet)])
    air = self._feet_sensor._air
    ptrs = [ctypes.c_void_p(air[k].data_ptr()) for k in
            ("current_air_time", "last_air_time", "current_contact_time", "last_contact_time", "last_time")]
    for k in ("current_air_time", "last_air_time", "current_contact_time", "last_contact_time", "last_time"):
      _need(air[k].is_contiguous() and air[k].dtype == torch.float32, "air-time buffers")
    stream = ctypes.c_void_p(torch.cuda.current_stream(sim._torch_device).cuda_stream)
    check(tl.mjx_sim_track_air_time(sim._sim, d.nfeet, adr, *ptrs, stream))
    self._feet_sensor.engine_owned = True
    return True

  def release(self) -> None:
    """Hand the air-time buffers back to the torch ContactSensor.update path: the engine
    stops updating them (n = 0).  Called when the env drops or replaces this fused step
    (enable_graph); without it a later torch-manager step would advance air time twice per
    substep."""
    if not getattr(self, "_engine_air", False):
      return
    sim = self.env.sim
    if getattr(sim, "_sim", None) is not None and sim._sim.value:
      stream = ctypes.c_void_p(torch.cuda.current_stream(sim._torch_device).cuda_stream)
      check(lib().mjx_sim_track_air_time(sim._sim, 0, None, None, None, None, None, None, stream))
    self._feet_sensor.engine_owned = False
    self._engine_air = False

  # ------------------------------------------------------------------ device handle
  def upload(self):
    """(Re)create the device copy of the descriptor (after a curriculum changed command
    ranges or reward weights)."""
    self._set_command_ranges(self._desc, self._cmd_term.cfg)
    for k, c in enumerate(self.env.reward_manager._term_cfgs):
      self._desc.reward_weight[k] = float(c.weight)
    if self._task is not None:
      self._L.mjx_task_destroy(self._task)
    h = ctypes.c_void_p()
    rc = self._L.mjx_task_create(ctypes.byref(self._desc), ctypes.byref(h))
    if rc != 0:
      raise MjxError(self._L.mjx_task_last_error().decode())
    self._task = h

  def __del__(self):
    try:
      self.release()
    except Exception:
      pass
    try:
      if self._task is not None:
        self._L.mjx_task_destroy(self._task)
    except Exception:
      pass

  def _ok(self, rc):
    if rc != 0:
      raise MjxError(self._L.mjx_task_last_error().decode())

  # ------------------------------------------------------------------ the env step
  # False while the env records a graph whose replays run apply_action() before them (the
  # action kernel then reads the caller's tensor: no copy into a static input buffer)
  action_in_step = True

  def apply_action(self, action: torch.Tensor):
    stream = ctypes.c_void_p(torch.cuda.current_stream(self.env.sim._torch_device).cuda_stream)
    self._ok(self._L.mjx_task_action(self._task, ctypes.c_void_p(action.data_ptr()), stream))

  def step(self, action: torch.Tensor):
    env, L, sim = self.env, self._L, self.env.sim
    stream = ctypes.c_void_p(torch.cuda.current_stream(sim._torch_device).cuda_stream)
    if self.action_in_step:
      self._ok(L.mjx_task_action(self._task, ctypes.c_void_p(action.data_ptr()), stream))
    if self._engine_air:
      # the engine updates the feet air times every substep (mjx_sim_track_air_time) and
      # nothing reads mjData between substeps: one mjx_step of `decimation` substeps, whose
      # full mjData outputs (frames, contacts, forces) are written after the last only
      sim.step(nsubstep=env.cfg.decimation)
    else:
      for _ in range(env.cfg.decimation):
        sim.step()
        self._ok(L.mjx_task_substep(self._task, stream))
    self._ok(L.mjx_task_post(self._task, stream))
    # per-env curriculum terms (terrain levels) of the resetting envs, before the reset
    # events read the env origins (the reference's _reset_idx order)
    cur = env.curriculum_manager
    cur.compute_masked(self.reset_buf)
    for name, state in getattr(cur, "_curriculum_state", {}).items():
      if isinstance(state, torch.Tensor):
        env.extras.setdefault("log", {})[f"Curriculum/{name}"] = state
    mask = ctypes.c_void_p(self.reset_buf.data_ptr())
    check(lib().mjx_reset(sim._sim, mask, stream))
    self._ok(L.mjx_task_reset(self._task, stream))
    check(lib().mjx_forward_masked(sim._sim, mask, stream))
    self._ok(L.mjx_task_observe(self._task, stream))
    tm = env.termination_manager
    return self.obs, env.reward_manager._reward_buf, tm._terminated_buf, tm._truncated_buf

  def log(self) -> dict:
    """Episode logs as device scalars under the reference's keys."""
    out = {}
    for k, name in enumerate(self._reward_names):
      out["Episode_Reward/" + name] = self.log_reward[k]
    for k, name in enumerate(self._term_names):
      out["Episode_Termination/" + name] = self.log_term[k]
    out["Metrics/twist/error_vel_xy"] = self.log_cmd[0]
    out["Metrics/twist/error_vel_yaw"] = self.log_cmd[1]
    for i, key in enumerate(_METRIC_KEYS):
      if self._metric_active[i]:
        out[key] = self.log_metric[i]
    return out


# ============================================================================ jump task
CMD_JUMP = 1
_JUMP_REWARD_KIND = {
  jump.explosive_takeoff: 15, jump.synchronized_extension: 16, jump.vertical_impulse: 17,
  jump.air_time_bonus: 18, jump.symmetric_landing: 20, mdp.action_acc_l2: 21,
  mdp.joint_torques_l2: 22, mdp.is_alive: 23, mdp.flat_orientation: 2,
  mdp.angular_momentum_penalty: 5, mdp.soft_landing: 12, mdp.action_rate_l2: 7,
  mdp.joint_pos_limits: 6,
}
_JUMP_POLICY = [("base_lin_vel", mdp.builtin_sensor), ("base_ang_vel", mdp.builtin_sensor),
                ("projected_gravity", mdp.projected_gravity), ("joint_pos", mdp.joint_pos_rel),
                ("joint_vel", mdp.joint_vel_rel), ("actions", mdp.last_action),
                ("height_above_ground", jump.height_above_ground),
                ("vertical_velocity", jump.vertical_velocity), ("contact_state", jump.foot_contact),
                ("time_in_air", jump.foot_air_time), ("command", mdp.generated_commands)]
_JUMP_CRITIC_EXTRA = [("foot_height", jump.foot_height), ("foot_contact_forces", jump.foot_contact_forces)]


class FusedJumpStep(FusedVelocityStep):
  """The jump task (tasks/jump/jump_env_cfg.py:36-354) on the same
  fused kernels: command_kind MJX_CMD_JUMP selects JumpCommand, the jump reward / termination
  kinds and the jump observation layout.  The stateful rewards (jump_height_reward,
  landing_balance) run on their own objects' tensors, so a torch-side reader sees the same
  peaks / timers."""

  def _make_desc(self, env):
    d = TaskDesc()
    robot, sens = self._base(d, env)
    scene, nj, dev = env.scene, d.njoint, torch.device(env.device)
    d.command_kind = CMD_JUMP
    idx = robot.indexing
    ctrl_ids = idx.ctrl_ids.tolist()
    _need(len(ctrl_ids) == nj and d.nu == nj, "one actuator per joint")
    for j in range(nj):  # Entity.actuator_force = data.actuator_force[:, ctrl_ids] (scene.py)
      d.act_ctrl[j] = ctrl_ids[j]
    d.actuator_force = _ptr(env.sim.data.actuator_force)
    # observations first: the feet sites come from the critic's foot_height term
    om = env.observation_manager
    groups = om._group_obs_term_names
    _need(set(groups) == {"policy", "critic"}, "policy + critic groups")
    pol = list(zip(groups["policy"], om._group_obs_term_cfgs["policy"]))
    cri = list(zip(groups["critic"], om._group_obs_term_cfgs["critic"]))
    _need([(nme, c.func) for nme, c in pol] == _JUMP_POLICY, "jump policy terms")
    _need([(nme, c.func) for nme, c in cri] == _JUMP_POLICY + _JUMP_CRITIC_EXTRA, "jump critic terms")
    feet_sensor = pol[8][1].params["sensor_name"]
    for i in (9,):
      _need(pol[i][1].params["sensor_name"] == feet_sensor, "jump obs sensor")
    _need(cri[12][1].params["sensor_name"] == feet_sensor, "jump critic force sensor")
    site_names = tuple(cri[11][1].params["asset_cfg"].site_names)
    # rewards
    rm = env.reward_manager
    _need(len(rm._term_names) <= MAXT, "too many reward terms")
    d.nreward = len(rm._term_names)
    orient_body = -1
    self._metric_active = [False] * NMETRIC
    self._jump_height = self._landing = None
    for k, (name, c) in enumerate(zip(rm._term_names, rm._term_cfgs)):
      f, p = c.func, c.params
      d.reward_weight[k] = float(c.weight)
      if "sensor_name" in p and p["sensor_name"] != "robot/root_angmom":
        _need(p["sensor_name"] == feet_sensor, f"{name}: feet sensor")
      if isinstance(f, jump.jump_height_reward):
        kind = 14
        d.reward_p0[k], d.reward_p1[k] = float(p["target_height"]), float(p["std"])
        self._jump_height = f
        self._metric_active[5] = self._metric_active[6] = c.weight != 0.0
      elif isinstance(f, jump.landing_balance):
        kind = 19
        d.reward_p0[k] = float(p.get("stability_time", 0.5))
        _need(abs(f.step_dt - env.step_dt) < 1e-12, "landing timer dt")
        self._landing = f
        self._metric_active[7] = c.weight != 0.0
      else:
        _need(f in _JUMP_REWARD_KIND, f"jump reward term {name}")
        kind = _JUMP_REWARD_KIND[f]
        if kind == 2:
          orient_body = self._orient(d, k, kind, p, robot, orient_body)
        elif kind == 5:
          d.angmom_adr = sens[p["sensor_name"]][0]
        elif kind == 12:
          d.reward_p0[k] = float(p.get("command_threshold", 0.05))
          _need(p.get("command_name") is None, "jump soft_landing is ungated")
          d.reward_p1[k] = 1.0
        elif kind == 15:
          d.reward_p0[k] = float(p.get("power_threshold", 500.0))
          ac = p.get("asset_cfg")
          ids = ac.joint_ids if ac is not None else slice(None)
          ids = list(range(nj)) if isinstance(ids, slice) else [int(i) for i in ids]
          d.explosive_joints = sum(1 << i for i in ids)
        elif kind == 18:
          d.reward_p0[k] = float(p.get("min_air_time", 0.2))
      d.reward_kind[k] = kind
      if c.weight != 0.0 and kind in _METRIC_OF_KIND:
        self._metric_active[_METRIC_OF_KIND[kind]] = True
    d.orient_body = orient_body
    self._feet(d, robot, feet_sensor, site_names)
    n = env.num_envs
    if self._jump_height is None:
      self._jump_height = jump.jump_height_reward(None, env)
    if self._landing is None:
      self._landing = jump.landing_balance(None, env)
    jh, lb = self._jump_height, self._landing
    d.jump_peak, d.jump_initial = _ptr(jh.peak_heights), _ptr(jh.initial_heights)
    d.jump_initialized = _ptr(jh.initialized, _U8)
    d.landing_timer, d.was_in_air = _ptr(lb.stability_timer), _ptr(lb.was_in_air, _U8)
    self._terminations(d, env)
    self._reward_buffers(d, env)
    # command: JumpCommand (commands.py:17-62)
    cm = env.command_manager
    _need(list(getattr(cm, "_terms", {}).keys()) == ["jump"], "single 'jump' command")
    ct = cm._terms["jump"]
    _need(isinstance(ct, jump.JumpCommand), "JumpCommand")
    self._cmd_term = ct
    d.resampling_time[0], d.resampling_time[1] = map(float, ct.cfg.resampling_time_range)
    d.jump_target_height = float(ct.cfg.target_height)
    d.command, d.cmd_time_left = _ptr(ct.height_command), _ptr(ct.time_left)
    d.command_counter = _ptr(ct.command_counter, _I64)
    d.metric_err_xy, d.metric_err_yaw = _ptr(ct.metrics["target_height"]), _ptr(ct.metrics["peak_height"])
    self._events(d, env)
    _need(not d.has_push, "no interval events in the jump task")
    self._obs_noise(d, env, pol, cri, sens)
    for i in range(5, 11):
      _need(pol[i][1].noise is None, "noise beyond the proprioceptive terms")
    d.npolicy = 9 + 3 * nj + 2 + 2 * d.nfeet + 1
    d.ncritic = d.npolicy + 4 * d.nfeet
    self._io(d, env)
    return d

  def upload(self):
    """Curricula move the target height (progressive_jump_height) and reward weights."""
    self._desc.jump_target_height = float(self._cmd_term.cfg.target_height)
    for k, c in enumerate(self.env.reward_manager._term_cfgs):
      self._desc.reward_weight[k] = float(c.weight)
    if self._task is not None:
      self._L.mjx_task_destroy(self._task)
    h = ctypes.c_void_p()
    rc = self._L.mjx_task_create(ctypes.byref(self._desc), ctypes.byref(h))
    if rc != 0:
      raise MjxError(self._L.mjx_task_last_error().decode())
    self._task = h

  def log(self) -> dict:
    out = {}
    for k, name in enumerate(self._reward_names):
      out["Episode_Reward/" + name] = self.log_reward[k]
    for k, name in enumerate(self._term_names):
      out["Episode_Termination/" + name] = self.log_term[k]
    out["Metrics/jump/target_height"] = self.log_cmd[0]
    out["Metrics/jump/peak_height"] = self.log_cmd[1]
    for i, key in enumerate(_METRIC_KEYS):
      if self._metric_active[i]:
        out[key] = self.log_metric[i]
    return out
