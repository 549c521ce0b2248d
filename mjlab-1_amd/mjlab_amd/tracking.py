"""Motion-tracking task (BeyondMimic) on the MI355X engine: MotionCommand, tracking MDP
terms and the `Mjlab-Tracking-Flat-Unitree-G1` config.

Restates `src/mjlab/tasks/tracking/mdp/{commands,rewards,terminations,observations}.py`
and `tasks/tracking/{tracking_env_cfg.py,config/g1/env_cfgs.py}`: same names, parameters
and math.  Every term also has a sync-free form (masks instead of index lists, no host
reads) so the tracking env step is captured in one HIP graph like the velocity task.

Motions use the reference's `MotionLoader` npz schema (`commands.py:32-68`; written by
`scripts/csv_to_npz.py:206-301`): fps, joint_pos/joint_vel [T, nj], body_pos_w /
body_lin_vel_w / body_ang_vel_w [T, nb, 3], body_quat_w [T, nb, 4].  Real motions come
from W&B in the reference, which is unreachable offline, so `synthesize_motion` builds
one the way csv_to_npz does: it writes root + joint states into the engine, runs
`Simulation.forward` (HIP), and records the robot's body link states (SURVEY.md 8d,
config 4: sinusoids of amplitude 0.2 rad with seeded phases about the knees-bent
keyframe, T=500 at 50 fps).
"""

from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import mdp
from .managers import (CommandTerm, CommandTermCfg, EventTermCfg, ObservationGroupCfg,
                       ObservationTermCfg, RewardTermCfg, SceneEntityCfg, TerminationTermCfg,
                       UniformNoiseCfg)
from .math_utils import (matrix_from_quat, quat_apply, quat_apply_inverse,
                         quat_error_magnitude, quat_from_euler_xyz, quat_inv, quat_mul,
                         sample_uniform, subtract_frame_transforms, yaw_quat)

MOTION_DIR = os.path.join(os.path.dirname(__file__), "assets", "motions")
SYNTHETIC_G1_MOTION = os.path.join(MOTION_DIR, "g1_synthetic_sine.npz")


# =========================================================================== motions
class MotionLoader:
  """`commands.py:32-68`: motion arrays on device; body arrays indexed by the
  command's body list."""

  def __init__(self, motion_file: str, body_indexes: torch.Tensor, device: str = "cpu"):
    with np.load(motion_file, allow_pickle=False) as data:
      t = lambda k: torch.tensor(data[k], dtype=torch.float32, device=device)
      self.joint_pos = t("joint_pos")
      self.joint_vel = t("joint_vel")
      self._body_pos_w = t("body_pos_w")
      self._body_quat_w = t("body_quat_w")
      self._body_lin_vel_w = t("body_lin_vel_w")
      self._body_ang_vel_w = t("body_ang_vel_w")
    self._body_indexes = body_indexes
    self.time_step_total = self.joint_pos.shape[0]
    # gathered once: the reference re-indexes the [T, nb] arrays on every property read
    self.body_pos_w = self._body_pos_w[:, body_indexes].contiguous()
    self.body_quat_w = self._body_quat_w[:, body_indexes].contiguous()
    self.body_lin_vel_w = self._body_lin_vel_w[:, body_indexes].contiguous()
    self.body_ang_vel_w = self._body_ang_vel_w[:, body_indexes].contiguous()


def synthesize_motion(scene_name: str = "g1_tracking", device: str = "cuda:0", T: int = 500,
                      fps: float = 50.0, amplitude: float = 0.2, seed: int = 0) -> dict:
  """Synthetic reference motion recorded through the engine's forward kinematics, as
  `csv_to_npz.run_sim` records a retargeted clip (`scripts/csv_to_npz.py:187-301`).

  Root: forward drift 0.25 m/s, vertical bob 1 cm at 0.5 Hz, yaw 0.2 rad at 0.1 Hz about
  the keyframe root pose.  Joints: keyframe + amplitude * sin(2 pi f_j t + phi_j), f_j ~
  U(0.3, 1.0) Hz, phi_j ~ U(0, 2 pi) (numpy seed), clipped to 0.9 x the joint range.
  Velocities are the analytic derivatives; body link velocities come from cvel."""
  from .scene import Scene
  from .scenes import load_scene
  from .sim import Simulation, SimulationCfg

  m = load_scene(scene_name)
  sim = Simulation(T, SimulationCfg(), m, device)
  scene = Scene.for_model(m, T, device)
  scene.initialize(m, sim.model, sim.data)
  robot = scene["robot"]
  rd = robot.data
  rng = np.random.default_rng(seed)
  nj = robot.num_joints
  f = torch.tensor(rng.uniform(0.3, 1.0, nj), dtype=torch.float32, device=device)
  ph = torch.tensor(rng.uniform(0.0, 2 * math.pi, nj), dtype=torch.float32, device=device)
  t = torch.arange(T, device=device, dtype=torch.float32) / fps
  w = 2 * math.pi * f[None, :] * t[:, None] + ph[None, :]
  q0 = rd.default_joint_pos[0]
  jp = q0[None, :] + amplitude * torch.sin(w)
  jv = amplitude * 2 * math.pi * f[None, :] * torch.cos(w)
  lim = rd.soft_joint_pos_limits[0]
  clipped = (jp < lim[:, 0]) | (jp > lim[:, 1])
  jp = torch.minimum(torch.maximum(jp, lim[:, 0]), lim[:, 1])
  jv = torch.where(clipped, torch.zeros_like(jv), jv)
  root = rd.default_root_state[0]
  pos = root[0:3].repeat(T, 1)
  pos[:, 0] += 0.25 * t
  pos[:, 2] += 0.01 * torch.sin(math.pi * t)
  yaw = 0.2 * torch.sin(0.2 * math.pi * t)
  z = torch.zeros_like(yaw)
  quat = quat_mul(quat_from_euler_xyz(z, z, yaw), root[3:7].expand(T, 4))
  lin = torch.stack([torch.full_like(t, 0.25), z, 0.01 * math.pi * torch.cos(math.pi * t)], -1)
  ang = torch.stack([z, z, 0.2 * 0.2 * math.pi * torch.cos(0.2 * math.pi * t)], -1)
  robot.write_root_state_to_sim(torch.cat([pos, quat, lin, ang], -1))
  robot.write_joint_state_to_sim(jp, jv)
  sim.forward()
  torch.cuda.synchronize(device)
  out = {
    "fps": np.array([fps], dtype=np.float64),
    "joint_pos": rd.joint_pos.cpu().numpy(), "joint_vel": rd.joint_vel.cpu().numpy(),
    "body_pos_w": rd.body_link_pos_w.cpu().numpy(), "body_quat_w": rd.body_link_quat_w.cpu().numpy(),
    "body_lin_vel_w": rd.body_link_lin_vel_w.cpu().numpy(),
    "body_ang_vel_w": rd.body_link_ang_vel_w.cpu().numpy(),
  }
  del sim
  return out


def write_motion_npz(path: str, motion: dict) -> None:
  """Atomic publish: each process writes its own temp file in the target directory, then
  renames it over `path` (ranks racing on a fresh checkout each publish a whole file)."""
  import tempfile
  d = os.path.dirname(path) or "."
  os.makedirs(d, exist_ok=True)
  fd, tmp = tempfile.mkstemp(dir=d, prefix=".motion-", suffix=".npz")
  try:
    with os.fdopen(fd, "wb") as f:
      np.savez(f, **motion)
    os.replace(tmp, path)
  except BaseException:
    if os.path.exists(tmp):
      os.remove(tmp)
    raise


def ensure_synthetic_motion(path: str = SYNTHETIC_G1_MOTION, device: str = "cuda:0") -> str:
  if not os.path.exists(path):
    write_motion_npz(path, synthesize_motion(device=device))
  return path


# =========================================================================== command
@dataclass(kw_only=True)
class MotionCommandCfg(CommandTermCfg):
  """`commands.py:480-502`."""
  motion_file: str
  anchor_body_name: str
  body_names: tuple[str, ...]
  asset_name: str
  class_type: type | None = None
  pose_range: dict[str, tuple[float, float]] = field(default_factory=dict)
  velocity_range: dict[str, tuple[float, float]] = field(default_factory=dict)
  joint_position_range: tuple[float, float] = (-0.52, 0.52)
  adaptive_kernel_size: int = 1
  adaptive_lambda: float = 0.8
  adaptive_uniform_ratio: float = 0.1
  adaptive_alpha: float = 0.001
  sampling_mode: str = "adaptive"

  def __post_init__(self):
    if self.class_type is None:
      self.class_type = MotionCommand


_KEYS6 = ("x", "y", "z", "roll", "pitch", "yaw")


class MotionCommand(CommandTerm):
  """`commands.py:71-413`: reference motion time index per env, reference-state
  initialisation on resample, adaptive (failure-binned) start sampling, and the
  yaw-aligned relative body targets."""

  def __init__(self, cfg: MotionCommandCfg, env):
    super().__init__(cfg, env)
    self.robot = env.scene[cfg.asset_name]
    self.robot_anchor_body_index = self.robot.body_names.index(cfg.anchor_body_name)
    self.motion_anchor_body_index = cfg.body_names.index(cfg.anchor_body_name)
    self.body_indexes = torch.tensor(
      self.robot.find_bodies(cfg.body_names, preserve_order=True)[0], dtype=torch.long,
      device=self.device)
    if cfg.motion_file == SYNTHETIC_G1_MOTION:
      ensure_synthetic_motion(cfg.motion_file, self.device)
    self.motion = MotionLoader(cfg.motion_file, self.body_indexes, device=self.device)
    n, nb = self.num_envs, len(cfg.body_names)
    self.time_steps = torch.zeros(n, dtype=torch.long, device=self.device)
    self.body_pos_relative_w = torch.zeros(n, nb, 3, device=self.device)
    self.body_quat_relative_w = torch.zeros(n, nb, 4, device=self.device)
    self.body_quat_relative_w[:, :, 0] = 1.0
    self.bin_count = int(self.motion.time_step_total // (1 / env.step_dt)) + 1
    self.bin_failed_count = torch.zeros(self.bin_count, device=self.device)
    self._current_bin_failed = torch.zeros(self.bin_count, device=self.device)
    k = torch.tensor([cfg.adaptive_lambda ** i for i in range(cfg.adaptive_kernel_size)],
                     device=self.device)
    self.kernel = k / k.sum()
    for name in ("error_anchor_pos", "error_anchor_rot", "error_anchor_lin_vel",
                 "error_anchor_ang_vel", "error_body_pos", "error_body_rot", "error_body_lin_vel",
                 "error_body_ang_vel", "error_joint_pos",
                 "error_joint_vel", "sampling_entropy", "sampling_top1_prob",
                 "sampling_top1_bin"):
      self.metrics[name] = torch.zeros(n, device=self.device)
    self._pose_rng = self._ranges(cfg.pose_range)
    self._vel_rng = self._ranges(cfg.velocity_range)
    self._origins = env.scene.env_origins

  def _ranges(self, spec):
    return torch.tensor([spec.get(k, (0.0, 0.0)) for k in _KEYS6], device=self.device)

  # ------------------------------------------------------------------ motion reads
  @property
  def command(self) -> torch.Tensor:
    return torch.cat([self.joint_pos, self.joint_vel], dim=1)

  @property
  def joint_pos(self):
    return self.motion.joint_pos[self.time_steps]

  @property
  def joint_vel(self):
    return self.motion.joint_vel[self.time_steps]

  @property
  def body_pos_w(self):
    return self.motion.body_pos_w[self.time_steps] + self._origins[:, None, :]

  @property
  def body_quat_w(self):
    return self.motion.body_quat_w[self.time_steps]

  @property
  def body_lin_vel_w(self):
    return self.motion.body_lin_vel_w[self.time_steps]

  @property
  def body_ang_vel_w(self):
    return self.motion.body_ang_vel_w[self.time_steps]

  @property
  def anchor_pos_w(self):
    return self.motion.body_pos_w[self.time_steps, self.motion_anchor_body_index] + self._origins

  @property
  def anchor_quat_w(self):
    return self.motion.body_quat_w[self.time_steps, self.motion_anchor_body_index]

  @property
  def anchor_lin_vel_w(self):
    return self.motion.body_lin_vel_w[self.time_steps, self.motion_anchor_body_index]

  @property
  def anchor_ang_vel_w(self):
    return self.motion.body_ang_vel_w[self.time_steps, self.motion_anchor_body_index]

  # ------------------------------------------------------------------ robot reads
  @property
  def robot_joint_pos(self):
    return self.robot.data.joint_pos

  @property
  def robot_joint_vel(self):
    return self.robot.data.joint_vel

  @property
  def robot_body_pos_w(self):
    return self.robot.data.body_link_pos_w[:, self.body_indexes]

  @property
  def robot_body_quat_w(self):
    return self.robot.data.body_link_quat_w[:, self.body_indexes]

  @property
  def robot_body_lin_vel_w(self):
    return self.robot.data.body_link_lin_vel_w[:, self.body_indexes]

  @property
  def robot_body_ang_vel_w(self):
    return self.robot.data.body_link_ang_vel_w[:, self.body_indexes]

  @property
  def robot_anchor_pos_w(self):
    return self.robot.data.body_link_pos_w[:, self.robot_anchor_body_index]

  @property
  def robot_anchor_quat_w(self):
    return self.robot.data.body_link_quat_w[:, self.robot_anchor_body_index]

  @property
  def robot_anchor_lin_vel_w(self):
    return self.robot.data.body_link_lin_vel_w[:, self.robot_anchor_body_index]

  @property
  def robot_anchor_ang_vel_w(self):
    return self.robot.data.body_link_ang_vel_w[:, self.robot_anchor_body_index]

  # ------------------------------------------------------------------ metrics
  def _update_metrics(self):
    """`commands.py:223-257` (in place, so graph-captured steps see fresh values)."""
    M = self.metrics
    M["error_anchor_pos"].copy_(torch.norm(self.anchor_pos_w - self.robot_anchor_pos_w, dim=-1))
    M["error_anchor_rot"].copy_(quat_error_magnitude(self.anchor_quat_w, self.robot_anchor_quat_w))
    M["error_anchor_lin_vel"].copy_(
      torch.norm(self.anchor_lin_vel_w - self.robot_anchor_lin_vel_w, dim=-1))
    M["error_anchor_ang_vel"].copy_(
      torch.norm(self.anchor_ang_vel_w - self.robot_anchor_ang_vel_w, dim=-1))
    M["error_body_pos"].copy_(
      torch.norm(self.body_pos_relative_w - self.robot_body_pos_w, dim=-1).mean(dim=-1))
    M["error_body_rot"].copy_(
      quat_error_magnitude(self.body_quat_relative_w, self.robot_body_quat_w).mean(dim=-1))
    M["error_body_lin_vel"].copy_(torch.norm(
      self.body_lin_vel_w - self.robot_body_lin_vel_w, dim=-1).mean(dim=-1))
    M["error_body_ang_vel"].copy_(torch.norm(
      self.body_ang_vel_w - self.robot_body_ang_vel_w, dim=-1).mean(dim=-1))
    M["error_joint_pos"].copy_(torch.norm(self.joint_pos - self.robot_joint_pos, dim=-1))
    M["error_joint_vel"].copy_(torch.norm(self.joint_vel - self.robot_joint_vel, dim=-1))

  # ------------------------------------------------------------------ sampling
  def _sampling_probabilities(self):
    p = self.bin_failed_count + self.cfg.adaptive_uniform_ratio / float(self.bin_count)
    p = torch.nn.functional.pad(p.view(1, 1, -1), (0, self.cfg.adaptive_kernel_size - 1),
                                mode="replicate")
    p = torch.nn.functional.conv1d(p, self.kernel.view(1, 1, -1)).view(-1)
    return p / p.sum()

  def _sampling_metrics(self, p):
    H = -(p * (p + 1e-12).log()).sum()
    pmax, imax = p.max(dim=0)
    self.metrics["sampling_entropy"].fill_(0.0).add_(H / math.log(self.bin_count))
    self.metrics["sampling_top1_prob"].fill_(0.0).add_(pmax)
    self.metrics["sampling_top1_bin"].fill_(0.0).add_(imax.float() / self.bin_count)

  def _current_bins(self):
    return torch.clamp((self.time_steps * self.bin_count) // max(self.motion.time_step_total, 1),
                       0, self.bin_count - 1)

  def _adaptive_sampling(self, env_ids):
    """`commands.py:258-300`."""
    failed = self._env.termination_manager.terminated[env_ids]
    if torch.any(failed):
      fail_bins = self._current_bins()[env_ids][failed]
      self._current_bin_failed[:] = torch.bincount(fail_bins, minlength=self.bin_count)
    p = self._sampling_probabilities()
    bins = torch.multinomial(p, len(env_ids), replacement=True)
    self.time_steps[env_ids] = ((bins + sample_uniform(0.0, 1.0, (len(env_ids),), self.device))
                                / self.bin_count * (self.motion.time_step_total - 1)).long()
    self._sampling_metrics(p)

  def _adaptive_sampling_masked(self, mask):
    failed = (self._env.termination_manager.terminated & mask).float()
    counts = torch.zeros(self.bin_count, device=self.device).scatter_add_(
      0, self._current_bins(), failed)
    self._current_bin_failed.copy_(torch.where(failed.sum() > 0, counts, self._current_bin_failed))
    p = self._sampling_probabilities()
    bins = torch.multinomial(p, self.num_envs, replacement=True)
    fresh = ((bins + torch.rand(self.num_envs, device=self.device)) / self.bin_count
             * (self.motion.time_step_total - 1)).long()
    self.time_steps.copy_(torch.where(mask, fresh, self.time_steps))
    self._sampling_metrics(p)

  def _uniform_sampling(self, env_ids):
    self.time_steps[env_ids] = torch.randint(0, self.motion.time_step_total, (len(env_ids),),
                                             device=self.device)
    self.metrics["sampling_entropy"].fill_(1.0)
    self.metrics["sampling_top1_prob"].fill_(1.0 / self.bin_count)
    self.metrics["sampling_top1_bin"].fill_(0.5)

  # ------------------------------------------------------------------ reference-state init
  def _reference_state(self, n):
    """Root/joint state of the current motion frame plus the configured noise, for all
    envs (`commands.py:318-357`)."""
    root_pos = self.body_pos_w[:, 0].clone()
    root_ori = self.body_quat_w[:, 0].clone()
    root_lin = self.body_lin_vel_w[:, 0].clone()
    root_ang = self.body_ang_vel_w[:, 0].clone()
    r = sample_uniform(self._pose_rng[:, 0], self._pose_rng[:, 1], (n, 6), self.device)
    return root_pos, root_ori, root_lin, root_ang, r

  def _resample_command(self, env_ids):
    """`commands.py:309-375`."""
    mode = self.cfg.sampling_mode
    if mode == "start":
      self.time_steps[env_ids] = 0
    elif mode == "uniform":
      self._uniform_sampling(env_ids)
    else:
      self._adaptive_sampling(env_ids)
    root_pos, root_ori, root_lin, root_ang, r = self._reference_state(len(env_ids))
    root_pos[env_ids] += r[:, 0:3]
    root_ori[env_ids] = quat_mul(quat_from_euler_xyz(r[:, 3], r[:, 4], r[:, 5]), root_ori[env_ids])
    v = sample_uniform(self._vel_rng[:, 0], self._vel_rng[:, 1], (len(env_ids), 6), self.device)
    root_lin[env_ids] += v[:, :3]
    root_ang[env_ids] += v[:, 3:]
    jp = self.joint_pos.clone()
    jv = self.joint_vel.clone()
    lo, hi = self.cfg.joint_position_range
    jp += sample_uniform(lo, hi, jp.shape, self.device)
    lim = self.robot.data.soft_joint_pos_limits[env_ids]
    jp[env_ids] = torch.clip(jp[env_ids], lim[:, :, 0], lim[:, :, 1])
    self.robot.write_joint_state_to_sim(jp[env_ids], jv[env_ids], env_ids=env_ids)
    root_state = torch.cat([root_pos[env_ids], root_ori[env_ids], root_lin[env_ids],
                            root_ang[env_ids]], dim=-1)
    self.robot.write_root_state_to_sim(root_state, env_ids=env_ids)
    self.robot.data.clear_state(env_ids)

  def _resample_command_masked(self, mask):
    mode = self.cfg.sampling_mode
    if mode == "start":
      self.time_steps.masked_fill_(mask, 0)
    elif mode == "uniform":
      fresh = torch.randint(0, self.motion.time_step_total, (self.num_envs,), device=self.device)
      self.time_steps.copy_(torch.where(mask, fresh, self.time_steps))
      self.metrics["sampling_entropy"].fill_(1.0)
      self.metrics["sampling_top1_prob"].fill_(1.0 / self.bin_count)
      self.metrics["sampling_top1_bin"].fill_(0.5)
    else:
      self._adaptive_sampling_masked(mask)
    n = self.num_envs
    root_pos, root_ori, root_lin, root_ang, r = self._reference_state(n)
    root_pos = root_pos + r[:, 0:3]
    root_ori = quat_mul(quat_from_euler_xyz(r[:, 3], r[:, 4], r[:, 5]), root_ori)
    v = sample_uniform(self._vel_rng[:, 0], self._vel_rng[:, 1], (n, 6), self.device)
    root_lin = root_lin + v[:, :3]
    root_ang = root_ang + v[:, 3:]
    lo, hi = self.cfg.joint_position_range
    jp = self.joint_pos + sample_uniform(lo, hi, (n, self.robot.num_joints), self.device)
    lim = self.robot.data.soft_joint_pos_limits
    jp = torch.minimum(torch.maximum(jp, lim[..., 0]), lim[..., 1])
    d = self.robot.data
    d.write_joint_state_masked(jp, self.joint_vel, mask)
    d.write_root_pose_masked(torch.cat([root_pos, root_ori], -1), mask)
    d.write_root_velocity_masked(torch.cat([root_lin, root_ang], -1), mask)
    d.clear_state_masked(mask)

  # ------------------------------------------------------------------ per-step update
  def _relative_targets(self):
    """`commands.py:384-404`: yaw-aligned motion bodies placed at the robot anchor."""
    nb = len(self.cfg.body_names)
    apos = self.anchor_pos_w[:, None, :].expand(-1, nb, -1)
    aquat = self.anchor_quat_w[:, None, :].expand(-1, nb, -1)
    rpos = self.robot_anchor_pos_w[:, None, :].expand(-1, nb, -1)
    rquat = self.robot_anchor_quat_w[:, None, :].expand(-1, nb, -1)
    delta_pos = torch.cat([rpos[..., :2], apos[..., 2:3]], dim=-1)
    delta_ori = yaw_quat(quat_mul(rquat, quat_inv(aquat)))
    self.body_quat_relative_w.copy_(quat_mul(delta_ori, self.body_quat_w))
    self.body_pos_relative_w.copy_(delta_pos + quat_apply(delta_ori, self.body_pos_w - apos))

  def _adaptive_update(self):
    if self.cfg.sampling_mode == "adaptive":
      a = self.cfg.adaptive_alpha
      self.bin_failed_count.mul_(1 - a).add_(a * self._current_bin_failed)
      self._current_bin_failed.zero_()

  def _update_command(self):
    """`commands.py:377-413`."""
    self.time_steps += 1
    if getattr(self._env, "sync_free", False):
      self._resample_command_masked(self.time_steps >= self.motion.time_step_total)
    else:
      env_ids = torch.where(self.time_steps >= self.motion.time_step_total)[0]
      if env_ids.numel() > 0:
        self._resample_command(env_ids)
    self._relative_targets()
    self._adaptive_update()


# =========================================================================== MDP terms
def _cmd(env, name) -> MotionCommand:
  return env.command_manager.get_term(name)


def _body_sel(command, body_names):
  """`rewards.py:17-24`: indexes into the command's body list (all if None)."""
  if body_names is None:
    return slice(None)
  cache = command.__dict__.setdefault("_body_sel_cache", {})
  key = tuple(body_names)
  if key not in cache:  # device index tensor: no host->device copy inside a graph capture
    ids = [i for i, n in enumerate(command.cfg.body_names) if n in body_names]
    cache[key] = torch.tensor(ids, dtype=torch.long, device=command.body_pos_relative_w.device)
  return cache[key]


# observations (`tasks/tracking/mdp/observations.py:18-69`)
def motion_anchor_pos_b(env, command_name: str):
  c = _cmd(env, command_name)
  pos, _ = subtract_frame_transforms(c.robot_anchor_pos_w, c.robot_anchor_quat_w,
                                     c.anchor_pos_w, c.anchor_quat_w)
  return pos.view(env.num_envs, -1)


def motion_anchor_ori_b(env, command_name: str):
  c = _cmd(env, command_name)
  _, ori = subtract_frame_transforms(c.robot_anchor_pos_w, c.robot_anchor_quat_w,
                                     c.anchor_pos_w, c.anchor_quat_w)
  mat = matrix_from_quat(ori)
  return mat[..., :2].reshape(mat.shape[0], -1)


def _robot_bodies_in_anchor(c):
  nb = len(c.cfg.body_names)
  return subtract_frame_transforms(c.robot_anchor_pos_w[:, None, :].expand(-1, nb, -1),
                                   c.robot_anchor_quat_w[:, None, :].expand(-1, nb, -1),
                                   c.robot_body_pos_w, c.robot_body_quat_w)


def robot_body_pos_b(env, command_name: str):
  pos_b, _ = _robot_bodies_in_anchor(_cmd(env, command_name))
  return pos_b.reshape(env.num_envs, -1)


def robot_body_ori_b(env, command_name: str):
  _, ori_b = _robot_bodies_in_anchor(_cmd(env, command_name))
  mat = matrix_from_quat(ori_b)
  return mat[..., :2].reshape(mat.shape[0], -1)


# rewards (`tasks/tracking/mdp/rewards.py:26-120`)
def motion_global_anchor_position_error_exp(env, command_name: str, std: float):
  c = _cmd(env, command_name)
  err = torch.sum(torch.square(c.anchor_pos_w - c.robot_anchor_pos_w), dim=-1)
  return torch.exp(-err / std ** 2)


def motion_global_anchor_orientation_error_exp(env, command_name: str, std: float):
  c = _cmd(env, command_name)
  err = quat_error_magnitude(c.anchor_quat_w, c.robot_anchor_quat_w) ** 2
  return torch.exp(-err / std ** 2)


def motion_relative_body_position_error_exp(env, command_name: str, std: float,
                                            body_names: tuple[str, ...] | None = None):
  c = _cmd(env, command_name)
  i = _body_sel(c, body_names)
  err = torch.sum(torch.square(c.body_pos_relative_w[:, i] - c.robot_body_pos_w[:, i]), dim=-1)
  return torch.exp(-err.mean(-1) / std ** 2)


def motion_relative_body_orientation_error_exp(env, command_name: str, std: float,
                                               body_names: tuple[str, ...] | None = None):
  c = _cmd(env, command_name)
  i = _body_sel(c, body_names)
  err = quat_error_magnitude(c.body_quat_relative_w[:, i], c.robot_body_quat_w[:, i]) ** 2
  return torch.exp(-err.mean(-1) / std ** 2)


def motion_global_body_linear_velocity_error_exp(env, command_name: str, std: float,
                                                 body_names: tuple[str, ...] | None = None):
  c = _cmd(env, command_name)
  i = _body_sel(c, body_names)
  err = torch.sum(torch.square(c.body_lin_vel_w[:, i] - c.robot_body_lin_vel_w[:, i]), dim=-1)
  return torch.exp(-err.mean(-1) / std ** 2)


def motion_global_body_angular_velocity_error_exp(env, command_name: str, std: float,
                                                  body_names: tuple[str, ...] | None = None):
  c = _cmd(env, command_name)
  i = _body_sel(c, body_names)
  err = torch.sum(torch.square(c.body_ang_vel_w[:, i] - c.robot_body_ang_vel_w[:, i]), dim=-1)
  return torch.exp(-err.mean(-1) / std ** 2)


# terminations (`tasks/tracking/mdp/terminations.py:18-86`)
def bad_anchor_pos(env, command_name: str, threshold: float):
  c = _cmd(env, command_name)
  return torch.norm(c.anchor_pos_w - c.robot_anchor_pos_w, dim=1) > threshold


def bad_anchor_pos_z_only(env, command_name: str, threshold: float):
  c = _cmd(env, command_name)
  return torch.abs(c.anchor_pos_w[:, -1] - c.robot_anchor_pos_w[:, -1]) > threshold


def bad_anchor_ori(env, asset_cfg: SceneEntityCfg, command_name: str, threshold: float):
  a = env.scene[asset_cfg.name]
  c = _cmd(env, command_name)
  mg = quat_apply_inverse(c.anchor_quat_w, a.data.gravity_vec_w)
  rg = quat_apply_inverse(c.robot_anchor_quat_w, a.data.gravity_vec_w)
  return (mg[:, 2] - rg[:, 2]).abs() > threshold


def bad_motion_body_pos(env, command_name: str, threshold: float,
                        body_names: tuple[str, ...] | None = None):
  c = _cmd(env, command_name)
  i = _body_sel(c, body_names)
  err = torch.norm(c.body_pos_relative_w[:, i] - c.robot_body_pos_w[:, i], dim=-1)
  return torch.any(err > threshold, dim=-1)


def bad_motion_body_pos_z_only(env, command_name: str, threshold: float,
                               body_names: tuple[str, ...] | None = None):
  c = _cmd(env, command_name)
  i = _body_sel(c, body_names)
  err = torch.abs(c.body_pos_relative_w[:, i, -1] - c.robot_body_pos_w[:, i, -1])
  return torch.any(err > threshold, dim=-1)


# =========================================================================== task config
VELOCITY_RANGE = {"x": (-0.5, 0.5), "y": (-0.5, 0.5), "z": (-0.2, 0.2),
                  "roll": (-0.52, 0.52), "pitch": (-0.52, 0.52), "yaw": (-0.78, 0.78)}

G1_TRACKING_BODIES = (
  "pelvis", "left_hip_roll_link", "left_knee_link", "left_ankle_roll_link",
  "right_hip_roll_link", "right_knee_link", "right_ankle_roll_link", "torso_link",
  "left_shoulder_roll_link", "left_elbow_link", "left_wrist_yaw_link",
  "right_shoulder_roll_link", "right_elbow_link", "right_wrist_yaw_link")


def make_tracking_env_cfg():
  """`tasks/tracking/tracking_env_cfg.py:44-317`."""
  from .envs import ManagerBasedRlEnvCfg, SceneCfg
  from .sim import MujocoCfg, SimulationCfg
  from .terrains import TerrainImporterCfg
  U = UniformNoiseCfg
  policy = {
    "command": ObservationTermCfg(func=mdp.generated_commands, params={"command_name": "motion"}),
    "motion_anchor_pos_b": ObservationTermCfg(func=motion_anchor_pos_b, params={"command_name": "motion"},
                                              noise=U(n_min=-0.25, n_max=0.25)),
    "motion_anchor_ori_b": ObservationTermCfg(func=motion_anchor_ori_b, params={"command_name": "motion"},
                                              noise=U(n_min=-0.05, n_max=0.05)),
    "base_lin_vel": ObservationTermCfg(func=mdp.builtin_sensor, params={"sensor_name": "robot/imu_lin_vel"},
                                       noise=U(n_min=-0.5, n_max=0.5)),
    "base_ang_vel": ObservationTermCfg(func=mdp.builtin_sensor, params={"sensor_name": "robot/imu_ang_vel"},
                                       noise=U(n_min=-0.2, n_max=0.2)),
    "joint_pos": ObservationTermCfg(func=mdp.joint_pos_rel, noise=U(n_min=-0.01, n_max=0.01),
                                    params={"biased": True}),
    "joint_vel": ObservationTermCfg(func=mdp.joint_vel_rel, noise=U(n_min=-0.5, n_max=0.5)),
    "actions": ObservationTermCfg(func=mdp.last_action),
  }
  critic = {
    "command": ObservationTermCfg(func=mdp.generated_commands, params={"command_name": "motion"}),
    "motion_anchor_pos_b": ObservationTermCfg(func=motion_anchor_pos_b, params={"command_name": "motion"}),
    "motion_anchor_ori_b": ObservationTermCfg(func=motion_anchor_ori_b, params={"command_name": "motion"}),
    "body_pos": ObservationTermCfg(func=robot_body_pos_b, params={"command_name": "motion"}),
    "body_ori": ObservationTermCfg(func=robot_body_ori_b, params={"command_name": "motion"}),
    "base_lin_vel": ObservationTermCfg(func=mdp.builtin_sensor, params={"sensor_name": "robot/imu_lin_vel"}),
    "base_ang_vel": ObservationTermCfg(func=mdp.builtin_sensor, params={"sensor_name": "robot/imu_ang_vel"}),
    "joint_pos": ObservationTermCfg(func=mdp.joint_pos_rel),
    "joint_vel": ObservationTermCfg(func=mdp.joint_vel_rel),
    "actions": ObservationTermCfg(func=mdp.last_action),
  }
  observations = {
    "policy": ObservationGroupCfg(terms=policy, concatenate_terms=True, enable_corruption=True),
    "critic": ObservationGroupCfg(terms=critic, concatenate_terms=True, enable_corruption=False),
  }
  actions = {"joint_pos": mdp.JointPositionActionCfg(asset_name="robot", actuator_names=(".*",),
                                                    scale=0.5, use_default_offset=True)}
  commands = {"motion": MotionCommandCfg(
    asset_name="robot", resampling_time_range=(1.0e9, 1.0e9), debug_vis=True,
    pose_range={"x": (-0.05, 0.05), "y": (-0.05, 0.05), "z": (-0.01, 0.01),
                "roll": (-0.1, 0.1), "pitch": (-0.1, 0.1), "yaw": (-0.2, 0.2)},
    velocity_range=dict(VELOCITY_RANGE), joint_position_range=(-0.1, 0.1),
    motion_file="", anchor_body_name="", body_names=())}
  events = {
    "push_robot": EventTermCfg(func=mdp.push_by_setting_velocity, mode="interval",
                               interval_range_s=(1.0, 3.0),
                               params={"velocity_range": dict(VELOCITY_RANGE)}),
    "base_com": EventTermCfg(mode="startup", func=mdp.randomize_field, domain_randomization=True,
                             params={"asset_cfg": SceneEntityCfg("robot", body_names=()),
                                     "operation": "add", "field": "body_ipos",
                                     "ranges": {0: (-0.025, 0.025), 1: (-0.05, 0.05),
                                                2: (-0.05, 0.05)}}),
    "encoder_bias": EventTermCfg(mode="startup", func=mdp.randomize_encoder_bias,
                                 params={"asset_cfg": SceneEntityCfg("robot"),
                                         "bias_range": (-0.01, 0.01)}),
    "foot_friction": EventTermCfg(mode="startup", func=mdp.randomize_field, domain_randomization=True,
                                  params={"asset_cfg": SceneEntityCfg("robot", geom_names=()),
                                          "operation": "abs", "field": "geom_friction",
                                          "ranges": (0.3, 1.2)}),
  }
  m = {"command_name": "motion"}
  rewards = {
    "motion_global_root_pos": RewardTermCfg(func=motion_global_anchor_position_error_exp, weight=0.5,
                                            params={**m, "std": 0.3}),
    "motion_global_root_ori": RewardTermCfg(func=motion_global_anchor_orientation_error_exp, weight=0.5,
                                            params={**m, "std": 0.4}),
    "motion_body_pos": RewardTermCfg(func=motion_relative_body_position_error_exp, weight=1.0,
                                     params={**m, "std": 0.3}),
    "motion_body_ori": RewardTermCfg(func=motion_relative_body_orientation_error_exp, weight=1.0,
                                     params={**m, "std": 0.4}),
    "motion_body_lin_vel": RewardTermCfg(func=motion_global_body_linear_velocity_error_exp, weight=1.0,
                                         params={**m, "std": 1.0}),
    "motion_body_ang_vel": RewardTermCfg(func=motion_global_body_angular_velocity_error_exp, weight=1.0,
                                         params={**m, "std": 3.14}),
    "action_rate_l2": RewardTermCfg(func=mdp.action_rate_l2, weight=-1e-1),
    "joint_limit": RewardTermCfg(func=mdp.joint_pos_limits, weight=-10.0,
                                 params={"asset_cfg": SceneEntityCfg("robot", joint_names=(".*",))}),
    "self_collisions": RewardTermCfg(func=mdp.self_collision_cost, weight=-10.0,
                                     params={"sensor_name": "self_collision"}),
  }
  terminations = {
    "time_out": TerminationTermCfg(func=mdp.time_out, time_out=True),
    "anchor_pos": TerminationTermCfg(func=bad_anchor_pos_z_only, params={**m, "threshold": 0.25}),
    "anchor_ori": TerminationTermCfg(func=bad_anchor_ori, params={
      "asset_cfg": SceneEntityCfg("robot"), **m, "threshold": 0.8}),
    "ee_body_pos": TerminationTermCfg(func=bad_motion_body_pos_z_only, params={
      **m, "threshold": 0.25, "body_names": ()}),
  }
  return ManagerBasedRlEnvCfg(
    scene=SceneCfg(num_envs=1, terrain=TerrainImporterCfg(terrain_type="plane")),
    observations=observations,
    actions=actions, commands=commands, events=events, rewards=rewards,
    terminations=terminations,
    # the reference's njmax (250 rows per world) as the max capacity; random-action tracking
    # worlds reach 190 rows and 49 contacts, past the default 48 / 160 carve, so the fast
    # carve is 56 / 200 (a world past it is re-solved at 250 / 250).  Measured (round 5):
    # 56 / 200 2.72 M env-steps/s, 64 / 250 2.68 M, 48 / 160 2.46 M (73 re-solves per 100
    # env steps); DESIGN.md section 3
    sim=SimulationCfg(nconmax=35, njmax=250, engine_capacity=(56, 200),
                      mujoco=MujocoCfg(timestep=0.005, iterations=10, ls_iterations=20)),
    decimation=4, episode_length_s=10.0)


def unitree_g1_flat_tracking_env_cfg(has_state_estimation: bool = True, play: bool = False,
                                     motion_file: str = SYNTHETIC_G1_MOTION):
  """`tasks/tracking/config/g1/env_cfgs.py:15-100`."""
  from . import asset_zoo as az
  from .sensor import ContactMatch, ContactSensorCfg
  cfg = make_tracking_env_cfg()
  cfg.scene.entities = {"robot": az.get_g1_robot_cfg()}
  cfg.scene.sensors = (ContactSensorCfg(
    name="self_collision", primary=ContactMatch(mode="subtree", pattern="pelvis", entity="robot"),
    secondary=ContactMatch(mode="subtree", pattern="pelvis", entity="robot"),
    fields=("found",), reduce="none", num_slots=1),)
  cfg.actions["joint_pos"].scale = az.action_scale(az.g1_actuators())
  mc = cfg.commands["motion"]
  mc.motion_file = motion_file
  mc.anchor_body_name = "torso_link"
  mc.body_names = G1_TRACKING_BODIES
  cfg.events["foot_friction"].params["asset_cfg"].geom_names = r"^(left|right)_foot[1-7]_collision$"
  cfg.events["base_com"].params["asset_cfg"].body_names = ("torso_link",)
  cfg.terminations["ee_body_pos"].params["body_names"] = (
    "left_ankle_roll_link", "right_ankle_roll_link", "left_wrist_yaw_link", "right_wrist_yaw_link")
  if not has_state_estimation:
    terms = {k: v for k, v in cfg.observations["policy"].terms.items()
             if k not in ("motion_anchor_pos_b", "base_lin_vel")}
    cfg.observations["policy"] = ObservationGroupCfg(terms=terms, concatenate_terms=True,
                                                     enable_corruption=True)
  if play:
    cfg.episode_length_s = int(1e9)
    cfg.observations["policy"].enable_corruption = False
    cfg.events.pop("push_robot", None)
    mc.pose_range = {}
    mc.velocity_range = {}
    mc.sampling_mode = "start"
  return cfg
