"""Fused HIP managers for the motion-tracking task (include/mjx355_task.h mjx_track_*,
csrc/tracking_task.hip).

`FusedTrackingStep.build(env)` inspects a ManagerBasedRlEnv. If every action /
observation / reward / termination / command / event term is one the fused kernels
implement (the term set of tasks/tracking/tracking_env_cfg.py:42-317 and
config/g1/env_cfgs.py:15-100, mirrored by mjlab_amd/tracking.py), it returns a step object
whose `step(action)` runs the env step as ~20 launches:
  track_action; decimation x mjx_step; track_post; mjx_reset(mask); track_reset;
  mjx_forward_masked(mask); track_observe.
Otherwise it returns None and the env keeps the torch manager path.

The kernels read and write the managers' own tensors (action histories, MotionCommand
time steps / relative body targets / failure bins / metrics, episode sums, termination
flags, push timers), so every accessor of the reference API keeps working.
"""

from __future__ import annotations

import ctypes

import torch

from . import mdp
from . import tracking as trk
from ._lib import MjxError, check, lib
from .fused import MAXJ, MAXT, Unsupported, _f2, _f62, _FP, _I64, _need, _noise, _ptr, _range6, _U8, _U64

MAXB, NMETRIC = 32, 13
_I32 = ctypes.c_int
METRIC_NAMES = ("error_anchor_pos", "error_anchor_rot", "error_anchor_lin_vel",
                "error_anchor_ang_vel", "error_body_pos", "error_body_rot", "error_body_lin_vel",
                "error_body_ang_vel", "error_joint_pos", "error_joint_vel", "sampling_entropy",
                "sampling_top1_prob", "sampling_top1_bin")


class TrackDesc(ctypes.Structure):
  """ctypes mirror of mjxTrackDesc (include/mjx355_task.h)."""
  _fields_ = [
    ("nworld", _I32), ("nq", _I32), ("nv", _I32), ("nu", _I32), ("nsensordata", _I32),
    ("nbody", _I32),
    ("qpos", _FP), ("qvel", _FP), ("ctrl", _FP),
    ("xpos", _FP), ("xquat", _FP), ("cvel", _FP), ("subtree_com", _FP), ("sensordata", _FP),
    ("root_body", _I32), ("free_q_adr", _I32), ("free_v_adr", _I32), ("njoint", _I32),
    ("joint_q_adr", _I32 * MAXJ), ("joint_v_adr", _I32 * MAXJ),
    ("ctrl_of_action", _I32 * MAXJ), ("target_of_action", _I32 * MAXJ),
    ("action_scale", ctypes.c_float * MAXJ), ("action_offset", ctypes.c_float * MAXJ),
    ("default_joint_pos", ctypes.c_float * MAXJ),
    ("soft_lo", ctypes.c_float * MAXJ), ("soft_hi", ctypes.c_float * MAXJ),
    ("encoder_bias", _FP), ("env_origins", _FP),
    ("nframe", _I32), ("nmb", _I32),
    ("m_joint_pos", _FP), ("m_joint_vel", _FP),
    ("m_body_pos", _FP), ("m_body_quat", _FP), ("m_body_lin", _FP), ("m_body_ang", _FP),
    ("robot_body", _I32 * MAXB), ("anchor_motion", _I32), ("anchor_body", _I32),
    ("step_dt", ctypes.c_float), ("episode_length_s", ctypes.c_float),
    ("max_episode_length", _I32),
    ("nreward", _I32), ("reward_kind", _I32 * MAXT), ("reward_weight", ctypes.c_float * MAXT),
    ("reward_std", ctypes.c_float * MAXT), ("reward_bodies", ctypes.c_uint32 * MAXT),
    ("ntermination", _I32), ("termination_kind", _I32 * MAXT),
    ("termination_is_timeout", _I32 * MAXT), ("termination_threshold", ctypes.c_float * MAXT),
    ("termination_bodies", ctypes.c_uint32 * MAXT),
    ("selfcol_found_adr", _I32), ("imu_lin_vel_adr", _I32), ("imu_ang_vel_adr", _I32),
    ("pose_range", _f62), ("vel_range", _f62), ("joint_position_range", _f2),
    ("sampling_mode", _I32), ("bin_count", _I32), ("kernel_size", _I32),
    ("kernel", ctypes.c_float * 8), ("uniform_ratio", ctypes.c_float),
    ("adaptive_alpha", ctypes.c_float),
    ("has_push", _I32), ("push_interval", _f2), ("push_vel_range", _f62),
    ("npolicy", _I32), ("ncritic", _I32), ("corrupt_policy", _I32),
    ("policy_anchor_pos", _I32), ("policy_lin_vel", _I32),
    ("noise_anchor_pos", ctypes.c_float), ("noise_anchor_ori", ctypes.c_float),
    ("noise_lin_vel", ctypes.c_float), ("noise_ang_vel", ctypes.c_float),
    ("noise_joint_pos", ctypes.c_float), ("noise_joint_vel", ctypes.c_float),
    ("seed", ctypes.c_uint64),
    ("action", _FP), ("prev_action", _FP), ("prev_prev_action", _FP), ("joint_pos_target", _FP),
    ("episode_length", _I64), ("time_steps", _I64),
    ("body_pos_rel", _FP), ("body_quat_rel", _FP),
    ("bin_failed_count", _FP), ("current_bin_failed", _FP), ("sampling", _FP),
    ("metrics", _FP), ("time_left", _FP), ("command_counter", _I64), ("push_time_left", _FP),
    ("episode_sums", _FP), ("step_reward", _FP), ("reward_buf", _FP),
    ("reset_buf", _U8), ("terminated", _U8), ("time_outs", _U8), ("term_dones", _U8),
    ("resample_mask", _U8),
    ("obs_policy", _FP), ("obs_critic", _FP),
    ("log_reward", _FP), ("log_termination", _FP), ("log_metric", _FP),
    ("step_counter", _U64),
  ]


_BODY_REWARDS = {trk.motion_relative_body_position_error_exp: 2,
                 trk.motion_relative_body_orientation_error_exp: 3,
                 trk.motion_global_body_linear_velocity_error_exp: 4,
                 trk.motion_global_body_angular_velocity_error_exp: 5}
_REWARDS = {trk.motion_global_anchor_position_error_exp: 0,
            trk.motion_global_anchor_orientation_error_exp: 1, **_BODY_REWARDS,
            mdp.action_rate_l2: 6, mdp.joint_pos_limits: 7, mdp.self_collision_cost: 8}
_TERMS = {mdp.time_out: 0, trk.bad_anchor_pos_z_only: 1, trk.bad_anchor_ori: 2,
          trk.bad_motion_body_pos_z_only: 3, trk.bad_anchor_pos: 4, trk.bad_motion_body_pos: 5}
_CRITIC = [("command", mdp.generated_commands), ("motion_anchor_pos_b", trk.motion_anchor_pos_b),
           ("motion_anchor_ori_b", trk.motion_anchor_ori_b), ("body_pos", trk.robot_body_pos_b),
           ("body_ori", trk.robot_body_ori_b), ("base_lin_vel", mdp.builtin_sensor),
           ("base_ang_vel", mdp.builtin_sensor), ("joint_pos", mdp.joint_pos_rel),
           ("joint_vel", mdp.joint_vel_rel), ("actions", mdp.last_action)]


class FusedTrackingStep:
  """One env step of the tracking task as fused HIP launches (see module docstring)."""

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
    _need(hasattr(L, "mjx_track_desc_size"), "library without the tracking kernels")
    L.mjx_track_desc_size.restype = ctypes.c_size_t
    _need(L.mjx_track_desc_size() == ctypes.sizeof(TrackDesc), "mjxTrackDesc layout mismatch")
    L.mjx_track_create.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
    L.mjx_track_action.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    for n in ("mjx_track_post", "mjx_track_reset", "mjx_track_observe"):
      getattr(L, n).argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.mjx_track_destroy.argtypes = [ctypes.c_void_p]
    L.mjx_track_last_error.restype = ctypes.c_char_p
    self._L = L
    self._keep = []
    self._task = None
    self._desc = self._make_desc(env)
    self.upload()

  # ------------------------------------------------------------------ descriptor
  def _make_desc(self, env):
    d = TrackDesc()
    sim, scene, m = env.sim, env.scene, env.sim.mj_model
    dev = torch.device(env.device)
    sd = sim.data
    n = env.num_envs
    d.nworld, d.nq, d.nv, d.nu = n, m.nq, m.nv, m.nu
    d.nsensordata, d.nbody = m.nsensordata, m.nbody
    for f in ("qpos", "qvel", "ctrl", "xpos", "xquat", "cvel", "subtree_com", "sensordata"):
      setattr(d, f, _ptr(getattr(sd, f)))
    # command
    cm = env.command_manager
    _need(list(getattr(cm, "_terms", {}).keys()) == ["motion"], "single 'motion' command")
    c = cm._terms["motion"]
    _need(isinstance(c, trk.MotionCommand), "MotionCommand")
    cc = c.cfg
    # actions
    am = env.action_manager
    _need(len(am._terms) == 1, "one action term")
    (aterm,) = am._terms.values()
    _need(isinstance(aterm, mdp.JointPositionAction), "JointPositionAction only")
    robot = aterm._asset
    _need(robot is c.robot, "command and action on one entity")
    rdata = robot.data
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
    off = aterm._offset
    _need(isinstance(off, float) or bool(torch.all(off == off[:1]).item()), "per-env action offset")
    for k, jk in enumerate(jids):
      d.ctrl_of_action[k] = ctrl_ids[act_local.index(jk)]
      d.target_of_action[k] = jk
      d.action_scale[k] = aterm._scale if isinstance(aterm._scale, float) else float(aterm._scale[0, k])
      d.action_offset[k] = off if isinstance(off, float) else float(off[0, k])
    _need(torch.all(rdata.default_joint_pos == rdata.default_joint_pos[:1]).item(), "per-env default joint pos")
    _need(torch.all(rdata.soft_joint_pos_limits == rdata.soft_joint_pos_limits[:1]).item(), "per-env soft limits")
    _need(torch.all(rdata.default_joint_vel == 0).item(), "nonzero default joint vel")
    dj = rdata.default_joint_pos[0].tolist()
    lim = rdata.soft_joint_pos_limits[0].tolist()
    for j in range(nj):
      d.default_joint_pos[j] = dj[j]
      d.soft_lo[j], d.soft_hi[j] = lim[j]
    d.encoder_bias = _ptr(rdata.encoder_bias)
    origins = scene.env_origins.contiguous()
    self._keep.append(origins)
    d.env_origins = _ptr(origins)
    # motion
    mo = c.motion
    body_ids = idx.body_ids.tolist()
    nmb = len(cc.body_names)
    _need(1 <= nmb <= MAXB, "command body count")
    d.nframe, d.nmb = int(mo.time_step_total), nmb
    arrays = [t.contiguous() for t in (mo.joint_pos, mo.joint_vel, mo.body_pos_w, mo.body_quat_w,
                                       mo.body_lin_vel_w, mo.body_ang_vel_w)]
    _need(arrays[0].shape[1] == nj, "motion joint count")
    self._keep.extend(arrays)
    (d.m_joint_pos, d.m_joint_vel, d.m_body_pos, d.m_body_quat, d.m_body_lin,
     d.m_body_ang) = (_ptr(t) for t in arrays)
    for k, bi in enumerate(c.body_indexes.tolist()):
      d.robot_body[k] = body_ids[bi]
    d.anchor_motion = int(c.motion_anchor_body_index)
    d.anchor_body = body_ids[c.robot_anchor_body_index]
    mode = {"start": 0, "uniform": 1, "adaptive": 2}.get(cc.sampling_mode)
    _need(mode is not None, "sampling mode")
    d.sampling_mode = mode
    d.bin_count = int(c.bin_count)
    ker = c.kernel.tolist()
    _need(1 <= len(ker) <= 8, "adaptive kernel size")
    d.kernel_size = len(ker)
    for i, v in enumerate(ker):
      d.kernel[i] = v
    d.uniform_ratio, d.adaptive_alpha = float(cc.adaptive_uniform_ratio), float(cc.adaptive_alpha)
    for i, (lo, hi) in enumerate(_range6(cc.pose_range)):
      d.pose_range[i][0], d.pose_range[i][1] = lo, hi
    for i, (lo, hi) in enumerate(_range6(cc.velocity_range)):
      d.vel_range[i][0], d.vel_range[i][1] = lo, hi
    d.joint_position_range[0], d.joint_position_range[1] = map(float, cc.joint_position_range)
    _need(float(cc.resampling_time_range[0]) >= 1e8, "timed motion resampling")
    d.time_steps = _ptr(c.time_steps, _I64)
    d.body_pos_rel, d.body_quat_rel = _ptr(c.body_pos_relative_w), _ptr(c.body_quat_relative_w)
    d.bin_failed_count, d.current_bin_failed = _ptr(c.bin_failed_count), _ptr(c._current_bin_failed)
    self._sampling = torch.zeros(d.bin_count + 4, device=dev)
    d.sampling = _ptr(self._sampling)
    # metrics: one [13, n] tensor, the command's metric dict viewing its rows
    _need(tuple(c.metrics.keys()) == METRIC_NAMES, "command metrics")
    self._metrics = torch.zeros(NMETRIC, n, device=dev)
    for k, name in enumerate(METRIC_NAMES):
      self._metrics[k].copy_(c.metrics[name])
      c.metrics[name] = self._metrics[k]
    d.metrics = _ptr(self._metrics)
    d.time_left, d.command_counter = _ptr(c.time_left), _ptr(c.command_counter, _I64)
    self._cmd = c
    # sensors
    sens = {name: int(m.sensor_adr[i]) for i, name in enumerate(m.names["sensor"])}
    d.selfcol_found_adr = d.imu_lin_vel_adr = d.imu_ang_vel_adr = -1
    body_pos = {name: k for k, name in enumerate(cc.body_names)}

    def bodies_mask(names):
      if names is None:
        return (1 << nmb) - 1
      return sum(1 << body_pos[x] for x in names if x in body_pos)

    # rewards
    rm = env.reward_manager
    _need(len(rm._term_names) <= MAXT, "too many reward terms")
    d.nreward = len(rm._term_names)
    for k, (name, cfg) in enumerate(zip(rm._term_names, rm._term_cfgs)):
      f, p = cfg.func, cfg.params
      _need(f in _REWARDS, f"reward term {name}")
      kind = _REWARDS[f]
      d.reward_kind[k] = kind
      d.reward_weight[k] = float(cfg.weight)
      if kind <= 5:
        _need(p.get("command_name") == "motion", "reward command name")
        d.reward_std[k] = float(p["std"])
      if kind in _BODY_REWARDS.values():
        d.reward_bodies[k] = bodies_mask(p.get("body_names"))
        _need(d.reward_bodies[k] != 0, "empty reward body set")
      if kind == 7:
        a = p.get("asset_cfg")
        _need(a is None or isinstance(a.joint_ids, slice), "joint_pos_limits over all joints")
      if kind == 8:
        adrs = self._found_adrs(scene[p["sensor_name"]])
        _need(len(adrs) == 1, "self-collision sensor with one slot")
        d.selfcol_found_adr = adrs[0]
    # terminations
    tm = env.termination_manager
    _need(len(tm._term_names) <= MAXT, "too many termination terms")
    d.ntermination = len(tm._term_names)
    for k, (name, cfg) in enumerate(zip(tm._term_names, tm._term_cfgs)):
      _need(cfg.func in _TERMS, f"termination {name}")
      kind = _TERMS[cfg.func]
      d.termination_kind[k] = kind
      d.termination_is_timeout[k] = int(bool(cfg.time_out))
      if kind > 0:
        _need(cfg.params.get("command_name") == "motion", "termination command name")
        d.termination_threshold[k] = float(cfg.params["threshold"])
      if kind in (3, 5):
        d.termination_bodies[k] = bodies_mask(cfg.params.get("body_names"))
    self._term_dones = torch.zeros(max(d.ntermination, 1), n, dtype=torch.bool, device=dev)
    for k, name in enumerate(tm._term_names):
      tm._term_dones[name] = self._term_dones[k]
    d.term_dones = _ptr(self._term_dones, _U8)
    d.terminated = _ptr(tm._terminated_buf, _U8)
    d.time_outs = _ptr(tm._truncated_buf, _U8)
    self.reset_buf = torch.zeros(n, dtype=torch.bool, device=dev)
    self._resample_mask = torch.zeros(n, dtype=torch.bool, device=dev)
    d.reset_buf, d.resample_mask = _ptr(self.reset_buf, _U8), _ptr(self._resample_mask, _U8)
    self._episode_sums = torch.zeros(max(d.nreward, 1), n, device=dev)
    for k, name in enumerate(rm._term_names):
      self._episode_sums[k].copy_(rm._episode_sums[name])
      rm._episode_sums[name] = self._episode_sums[k]
    d.episode_sums = _ptr(self._episode_sums)
    d.step_reward, d.reward_buf = _ptr(rm._step_reward), _ptr(rm._reward_buf)
    d.step_dt, d.episode_length_s = float(env.step_dt), float(env.max_episode_length_s)
    # play configs use a 1e9 s episode: clamp into the descriptor's int32 (never reached)
    d.max_episode_length = min(int(env.max_episode_length), 2 ** 31 - 1)
    _need(env.episode_length_buf.dtype == torch.int64, "episode length dtype")
    d.episode_length = _ptr(env.episode_length_buf, _I64)
    # events: startup (done), interval push; no reset-mode terms (the command's RSI resets)
    em = env.event_manager
    _need(set(em._mode_term_cfgs) <= {"interval", "startup"}, "event modes")
    inter = em._mode_term_cfgs.get("interval", [])
    _need(len(inter) <= 1, "one interval event")
    if inter:
      ci = inter[0]
      _need(ci.func is mdp.push_by_setting_velocity and not ci.is_global_time, "push event")
      d.has_push = 1
      d.push_interval[0], d.push_interval[1] = map(float, ci.interval_range_s)
      for i, (lo, hi) in enumerate(_range6(ci.params["velocity_range"])):
        d.push_vel_range[i][0], d.push_vel_range[i][1] = lo, hi
      d.push_time_left = _ptr(em._interval_time_left[0])
    else:
      self._dummy_push = torch.zeros(n, device=dev)
      d.push_time_left = _ptr(self._dummy_push)
    # observations
    om = env.observation_manager
    groups = om._group_obs_term_names
    _need(set(groups) == {"policy", "critic"}, "policy + critic groups")
    cri = list(zip(groups["critic"], om._group_obs_term_cfgs["critic"]))
    pol = list(zip(groups["policy"], om._group_obs_term_cfgs["policy"]))
    _need([(nme, cfg.func) for nme, cfg in cri] == _CRITIC, "critic terms")
    pol_expect = [x for x in _CRITIC if x[0] not in ("body_pos", "body_ori")]
    pol_names = [nme for nme, _ in pol]
    d.policy_anchor_pos = int("motion_anchor_pos_b" in pol_names)
    d.policy_lin_vel = int("base_lin_vel" in pol_names)
    pol_expect = [x for x in pol_expect if x[0] in pol_names]
    _need([(nme, cfg.func) for nme, cfg in pol] == pol_expect, "policy terms")
    for nme, cfg in pol + cri:
      _need(not cfg.clip and cfg.scale is None, "obs clip/scale")
      if cfg.func is mdp.generated_commands or cfg.func in (trk.motion_anchor_pos_b, trk.motion_anchor_ori_b,
                                                            trk.robot_body_pos_b, trk.robot_body_ori_b):
        _need(cfg.params.get("command_name") == "motion", "observation command name")
      if cfg.func in (mdp.joint_pos_rel, mdp.joint_vel_rel):
        a = cfg.params.get("asset_cfg")
        _need(a is None or isinstance(a.joint_ids, slice), "joint observations over all joints")
      if cfg.func is mdp.last_action:
        _need(cfg.params.get("action_name") is None, "last_action of the manager")
    polf = dict(pol)
    _need(bool(polf["joint_pos"].params.get("biased", False)), "biased policy joint_pos")
    _need(not bool(dict(cri)["joint_pos"].params.get("biased", False)), "unbiased critic joint_pos")
    for nme, cfg in cri:
      _need(cfg.noise is None or not om.cfg["critic"].enable_corruption, "critic noise")
    d.imu_lin_vel_adr = sens[dict(cri)["base_lin_vel"].params["sensor_name"]]
    d.imu_ang_vel_adr = sens[dict(cri)["base_ang_vel"].params["sensor_name"]]
    for key in ("base_lin_vel", "base_ang_vel"):
      if key in polf:
        _need(polf[key].params["sensor_name"] == dict(cri)[key].params["sensor_name"], "sensor")
    d.corrupt_policy = int(bool(om.cfg["policy"].enable_corruption))
    d.noise_anchor_pos = _noise(polf["motion_anchor_pos_b"]) if "motion_anchor_pos_b" in polf else 0.0
    d.noise_anchor_ori = _noise(polf["motion_anchor_ori_b"])
    d.noise_lin_vel = _noise(polf["base_lin_vel"]) if "base_lin_vel" in polf else 0.0
    d.noise_ang_vel, d.noise_joint_pos = _noise(polf["base_ang_vel"]), _noise(polf["joint_pos"])
    d.noise_joint_vel = _noise(polf["joint_vel"])
    for key in ("command", "actions"):
      _need(polf[key].noise is None, "noise on command/actions")
    d.ncritic = 5 * nj + 9 * nmb + 15
    d.npolicy = 5 * nj + 9 + 3 * d.policy_anchor_pos + 3 * d.policy_lin_vel
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
    self.log_metric = torch.zeros(NMETRIC, device=dev)
    self.step_counter = torch.zeros(1, dtype=torch.int64, device=dev)
    d.log_reward, d.log_termination = _ptr(self.log_reward), _ptr(self.log_term)
    d.log_metric = _ptr(self.log_metric)
    d.step_counter = _ptr(self.step_counter, _U64)
    self._reward_names, self._term_names = list(rm._term_names), list(tm._term_names)
    self._keep.extend([self._term_dones, self.reset_buf, self._resample_mask, self._episode_sums,
                       self._metrics, self._sampling])
    return d

  @staticmethod
  def _found_adrs(sensor):
    _need(getattr(sensor, "_num_slots", 1) == 1, "one contact slot per primary")
    return [adr for _, f, adr, _ in sensor._slots if f == "found"]

  # ------------------------------------------------------------------ device handle
  def upload(self):
    """(Re)create the device copy of the descriptor (after a curriculum changed reward
    weights)."""
    for k, c in enumerate(self.env.reward_manager._term_cfgs):
      self._desc.reward_weight[k] = float(c.weight)
    if self._task is not None:
      self._L.mjx_track_destroy(self._task)
    h = ctypes.c_void_p()
    rc = self._L.mjx_track_create(ctypes.byref(self._desc), ctypes.byref(h))
    if rc != 0:
      raise MjxError(self._L.mjx_track_last_error().decode())
    self._task = h

  def __del__(self):
    try:
      if self._task is not None:
        self._L.mjx_track_destroy(self._task)
    except Exception:
      pass

  def _ok(self, rc):
    if rc != 0:
      raise MjxError(self._L.mjx_track_last_error().decode())

  # ------------------------------------------------------------------ the env step
  action_in_step = True  # as FusedVelocityStep.action_in_step

  def apply_action(self, action: torch.Tensor):
    stream = ctypes.c_void_p(torch.cuda.current_stream(self.env.sim._torch_device).cuda_stream)
    self._ok(self._L.mjx_track_action(self._task, ctypes.c_void_p(action.data_ptr()), stream))

  def step(self, action: torch.Tensor):
    env, L, sim = self.env, self._L, self.env.sim
    stream = ctypes.c_void_p(torch.cuda.current_stream(sim._torch_device).cuda_stream)
    if self.action_in_step:
      self._ok(L.mjx_track_action(self._task, ctypes.c_void_p(action.data_ptr()), stream))
    sim.step(nsubstep=env.cfg.decimation)  # mjData outputs written after the last substep
    self._ok(L.mjx_track_post(self._task, stream))
    mask = ctypes.c_void_p(self.reset_buf.data_ptr())
    check(lib().mjx_reset(sim._sim, mask, stream))
    self._ok(L.mjx_track_reset(self._task, stream))
    check(lib().mjx_forward_masked(sim._sim, mask, stream))
    self._ok(L.mjx_track_observe(self._task, stream))
    tm = env.termination_manager
    return self.obs, env.reward_manager._reward_buf, tm._terminated_buf, tm._truncated_buf

  def log(self) -> dict:
    """Episode logs as device scalars under the reference's keys."""
    out = {}
    for k, name in enumerate(self._reward_names):
      out["Episode_Reward/" + name] = self.log_reward[k]
    for k, name in enumerate(self._term_names):
      out["Episode_Termination/" + name] = self.log_term[k]
    for k, name in enumerate(METRIC_NAMES):
      out["Metrics/motion/" + name] = self.log_metric[k]
    return out
