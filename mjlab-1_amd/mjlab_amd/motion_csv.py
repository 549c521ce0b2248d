"""Retargeted-motion pipeline: CSV clip -> tracking motion npz.

Restates `src/mjlab/scripts/csv_to_npz.py:22-179` (MotionLoader: CSV rows of root position,
root quaternion xyzw and joint positions; resampling from the input to the output frame
rate by lerp / slerp; velocities by `torch.gradient` and the SO(3) central difference) and
`run_sim` (`:182-308`: every frame written into the G1 tracking scene as root + joint
state, `Simulation.forward`, the robot's joint and body-link states logged, and the root
link velocities checked against the motion's).  The output npz is the `MotionLoader` schema
of the tracking task (`tasks/tracking/mdp/commands.py:32-68`).

MI355X form: forward kinematics is stateless in qpos / qvel, so the frames are not replayed
one at a time through a single world -- all T frames run as T worlds of one batched
`Simulation.forward` (HIP).  The W&B upload and video rendering of the reference script are
out of scope (no network, no renderer); the file is written locally.
"""

from __future__ import annotations

import numpy as np
import torch

from .math_utils import axis_angle_from_quat, quat_conjugate, quat_mul

# csv_to_npz.py:389-419: the CSV's joint column order
G1_CSV_JOINTS = [
  "left_hip_pitch_joint", "left_hip_roll_joint", "left_hip_yaw_joint", "left_knee_joint",
  "left_ankle_pitch_joint", "left_ankle_roll_joint", "right_hip_pitch_joint",
  "right_hip_roll_joint", "right_hip_yaw_joint", "right_knee_joint", "right_ankle_pitch_joint",
  "right_ankle_roll_joint", "waist_yaw_joint", "waist_roll_joint", "waist_pitch_joint",
  "left_shoulder_pitch_joint", "left_shoulder_roll_joint", "left_shoulder_yaw_joint",
  "left_elbow_joint", "left_wrist_roll_joint", "left_wrist_pitch_joint", "left_wrist_yaw_joint",
  "right_shoulder_pitch_joint", "right_shoulder_roll_joint", "right_shoulder_yaw_joint",
  "right_elbow_joint", "right_wrist_roll_joint", "right_wrist_pitch_joint", "right_wrist_yaw_joint",
]


def quat_slerp_rows(a: torch.Tensor, b: torch.Tensor, tau: torch.Tensor) -> torch.Tensor:
  """Row-wise `quat_slerp` (`utils/lab_api/math.py:1695-1728`, which the reference calls per
  frame), same branch order: tau 0 -> a; tau 1 -> b; |(|a.b| - 1)| < 4 eps -> a; the shorter
  arc (b negated when a.b < 0); angle < 4 eps -> a."""
  eps = torch.finfo(a.dtype).eps * 4.0
  d0 = (a * b).sum(-1)
  flip = d0 < 0.0
  d = torch.where(flip, -d0, d0)
  b2 = torch.where(flip.unsqueeze(-1), -b, b)
  angle = torch.acos(torch.clamp(d, -1, 1))
  isin = 1.0 / torch.sin(angle)
  out = (a * (torch.sin((1.0 - tau) * angle) * isin).unsqueeze(-1)
         + b2 * (torch.sin(tau * angle) * isin).unsqueeze(-1))
  out = torch.where((angle.abs() < eps).unsqueeze(-1), a, out)
  out = torch.where(((d0.abs() - 1.0).abs() < eps).unsqueeze(-1), a, out)
  out = torch.where((tau == 1.0).unsqueeze(-1), b, out)
  return torch.where((tau == 0.0).unsqueeze(-1), a, out)


class CsvMotion:
  """`csv_to_npz.MotionLoader` (`:22-179`), batched over frames."""

  def __init__(self, motion_file: str, input_fps: float, output_fps: float,
               device: torch.device | str = "cpu", line_range: tuple[int, int] | None = None):
    self.input_fps, self.output_fps = input_fps, output_fps
    self.input_dt, self.output_dt = 1.0 / input_fps, 1.0 / output_fps
    self.device = device
    if line_range is None:
      raw = np.loadtxt(motion_file, delimiter=",")
    else:
      raw = np.loadtxt(motion_file, delimiter=",", skiprows=line_range[0] - 1,
                       max_rows=line_range[1] - line_range[0] + 1)
    motion = torch.from_numpy(np.atleast_2d(raw)).to(torch.float32).to(device)
    self.base_pos_in = motion[:, :3]
    self.base_rot_in = motion[:, 3:7][:, [3, 0, 1, 2]]  # xyzw -> wxyz
    self.dof_pos_in = motion[:, 7:]
    self.input_frames = motion.shape[0]
    self.duration = (self.input_frames - 1) * self.input_dt
    self._interpolate()
    self._velocities()

  def _interpolate(self):
    times = torch.arange(0, self.duration, self.output_dt, device=self.device, dtype=torch.float32)
    self.output_frames = times.shape[0]
    phase = times / self.duration
    i0 = (phase * (self.input_frames - 1)).floor().long()
    i1 = torch.minimum(i0 + 1, torch.tensor(self.input_frames - 1, device=self.device))
    blend = phase * (self.input_frames - 1) - i0
    lerp = lambda a, b: a * (1 - blend.unsqueeze(1)) + b * blend.unsqueeze(1)
    self.base_pos = lerp(self.base_pos_in[i0], self.base_pos_in[i1])
    self.base_rot = quat_slerp_rows(self.base_rot_in[i0], self.base_rot_in[i1], blend)
    self.dof_pos = lerp(self.dof_pos_in[i0], self.dof_pos_in[i1])

  def _velocities(self):
    self.base_lin_vel = torch.gradient(self.base_pos, spacing=self.output_dt, dim=0)[0]
    self.dof_vel = torch.gradient(self.dof_pos, spacing=self.output_dt, dim=0)[0]
    q_prev, q_next = self.base_rot[:-2], self.base_rot[2:]
    omega = axis_angle_from_quat(quat_mul(q_next, quat_conjugate(q_prev))) / (2.0 * self.output_dt)
    self.base_ang_vel = torch.cat([omega[:1], omega, omega[-1:]], dim=0)


def csv_to_npz(input_file: str, output_file: str | None = None, input_fps: float = 30.0,
               output_fps: float = 50.0, device: str = "cuda:0",
               line_range: tuple[int, int] | None = None, joint_names=G1_CSV_JOINTS,
               scene_name: str = "g1_tracking", check_root_velocity: bool = True) -> dict:
  """`csv_to_npz.run_sim` + `main`: the motion's frames through the engine's forward
  kinematics, as T worlds of one launch; returns (and writes, given `output_file`) the
  tracking-motion arrays."""
  from .scene import Scene
  from .scenes import load_scene
  from .sim import MujocoCfg, Simulation, SimulationCfg
  from .tracking import write_motion_npz

  motion = CsvMotion(input_file, input_fps, output_fps, device, line_range)
  T = motion.output_frames
  m = load_scene(scene_name)
  sim = Simulation(T, SimulationCfg(mujoco=MujocoCfg(timestep=1.0 / output_fps)), m, device)
  scene = Scene.for_model(m, T, device)
  scene.initialize(m, sim.model, sim.data)
  robot = scene["robot"]
  rd = robot.data
  idx = robot.find_joints(list(joint_names), preserve_order=True)[0]
  # a one-env scene's origin is (0, 0): the reference adds it to the root position
  root = rd.default_root_state[:1].repeat(T, 1)
  root[:, 0:3] = motion.base_pos
  root[:, 3:7] = motion.base_rot
  root[:, 7:10] = motion.base_lin_vel
  root[:, 10:] = motion.base_ang_vel
  robot.write_root_state_to_sim(root)
  jp = rd.default_joint_pos[:1].repeat(T, 1)
  jv = rd.default_joint_vel[:1].repeat(T, 1)
  jp[:, idx] = motion.dof_pos
  jv[:, idx] = motion.dof_vel
  robot.write_joint_state_to_sim(jp, jv)
  sim.forward()
  if check_root_velocity:  # the reference's per-frame asserts (csv_to_npz.py:278-283)
    torch.testing.assert_close(rd.body_link_lin_vel_w[:, 0], motion.base_lin_vel)
    torch.testing.assert_close(rd.body_link_ang_vel_w[:, 0], motion.base_ang_vel)
  out = {
    "fps": np.array([output_fps]),
    "joint_pos": rd.joint_pos.cpu().numpy(), "joint_vel": rd.joint_vel.cpu().numpy(),
    "body_pos_w": rd.body_link_pos_w.cpu().numpy(), "body_quat_w": rd.body_link_quat_w.cpu().numpy(),
    "body_lin_vel_w": rd.body_link_lin_vel_w.cpu().numpy(),
    "body_ang_vel_w": rd.body_link_ang_vel_w.cpu().numpy(),
  }
  if output_file is not None:
    write_motion_npz(output_file, out)
  del sim
  return out
