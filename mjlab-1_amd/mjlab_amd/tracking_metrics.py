"""Motion-tracking evaluation metrics (`src/mjlab/tasks/tracking/mdp/metrics.py:13-101`).

Each function takes a `MotionCommand` (or any object with the same attributes) and returns
one value per env.  `compute_mpkpe` is the same quantity as the command's
`metrics["error_body_pos"]` (tracking.py `_update_metrics`, and the fused tracking kernel's
metric), which tests/test_gpu_tracking_metrics.py checks on the GPU.
"""

from __future__ import annotations

import torch

from .math_utils import quat_error_magnitude


def compute_mpkpe(command) -> torch.Tensor:
  """Mean per-key-body position error in the world frame (`metrics.py:13-22`)."""
  err = command.body_pos_relative_w - command.robot_body_pos_w
  return torch.norm(err, dim=-1).mean(dim=-1)


def compute_root_relative_mpkpe(command) -> torch.Tensor:
  """MPKPE of body positions relative to each side's own anchor (`metrics.py:25-44`):
  invariant to a common translation."""
  ref = command.body_pos_w - command.anchor_pos_w.unsqueeze(1)
  rob = command.robot_body_pos_w - command.robot_anchor_pos_w.unsqueeze(1)
  return torch.norm(ref - rob, dim=-1).mean(dim=-1)


def compute_joint_velocity_error(command) -> torch.Tensor:
  """L2 norm of the joint-velocity error (`metrics.py:47-50`)."""
  return torch.norm(command.joint_vel - command.robot_joint_vel, dim=-1)


def _body_indices(command, names) -> list[int]:
  """Indices of `names` within the command's body list (`metrics.py:88-101`)."""
  return [i for i, n in enumerate(command.cfg.body_names) if n in names]


def compute_ee_position_error(command, ee_body_names: tuple[str, ...]) -> torch.Tensor:
  """Mean position error over the listed end-effector bodies (`metrics.py:53-67`); zeros
  when none of them is tracked."""
  idx = _body_indices(command, ee_body_names)
  if not idx:
    return torch.zeros(command.num_envs, device=command.device)
  err = command.body_pos_relative_w[:, idx] - command.robot_body_pos_w[:, idx]
  return torch.norm(err, dim=-1).mean(dim=-1)


def compute_ee_orientation_error(command, ee_body_names: tuple[str, ...]) -> torch.Tensor:
  """Mean rotation angle between reference and robot over the listed end-effector bodies
  (`metrics.py:70-85`)."""
  idx = _body_indices(command, ee_body_names)
  if not idx:
    return torch.zeros(command.num_envs, device=command.device)
  return quat_error_magnitude(command.body_quat_relative_w[:, idx],
                              command.robot_body_quat_w[:, idx]).mean(dim=-1)
