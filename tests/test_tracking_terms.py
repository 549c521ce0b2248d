"""Tracking-task terms on CPU with a stand-in command (the reference's pattern in
tests/test_rewards.py:75-87: terms called on a mock env holding synthetic tensors).

Pins: quaternion helpers against closed forms (rotation angle, frame inverse), the
yaw-aligned relative targets of `commands.py:384-404` (identity when the robot anchor
equals the motion anchor; pure yaw offset rotates every target about the anchor), the
reward/termination formulas of `tasks/tracking/mdp/{rewards,terminations}.py` and the
6D rotation observation of `observations.py:33-45`.  Parity vs the reference's own
Python is unpinned (importing it was denied)."""

import math
from types import SimpleNamespace as NS

import torch

from mjlab_amd import tracking as tr
from mjlab_amd.math_utils import (matrix_from_quat, quat_error_magnitude, quat_from_euler_xyz,
                                  quat_mul, subtract_frame_transforms, yaw_quat)


def _rand_quat(n, g):
  q = torch.randn(n, 4, generator=g)
  return q / q.norm(dim=-1, keepdim=True)


def test_quat_error_magnitude_is_rotation_angle():
  ang = torch.tensor([0.0, 1e-7, 0.3, 1.0, 3.0])
  z = torch.zeros_like(ang)
  q = quat_from_euler_xyz(z, z, ang)
  e = quat_error_magnitude(q, quat_from_euler_xyz(z, z, z))
  torch.testing.assert_close(e, ang, atol=1e-6, rtol=1e-5)
  # sign-invariant (q and -q are the same rotation)
  torch.testing.assert_close(quat_error_magnitude(-q, q), torch.zeros_like(ang), atol=1e-5, rtol=0)


def test_subtract_frame_transforms_inverse():
  g = torch.Generator().manual_seed(0)
  q01, q02 = _rand_quat(16, g), _rand_quat(16, g)
  t01, t02 = torch.randn(16, 3, generator=g), torch.randn(16, 3, generator=g)
  t12, q12 = subtract_frame_transforms(t01, q01, t02, q02)
  # compose back: T02 = T01 * T12
  from mjlab_amd.math_utils import quat_apply
  torch.testing.assert_close(t01 + quat_apply(q01, t12), t02, atol=1e-5, rtol=1e-5)
  torch.testing.assert_close(matrix_from_quat(quat_mul(q01, q12)), matrix_from_quat(q02),
                             atol=1e-5, rtol=1e-5)


class _Cmd(tr.MotionCommand):
  """MotionCommand with the motion/robot reads replaced by fixed tensors."""

  def __init__(self, nb=3, n=4, seed=0):
    g = torch.Generator().manual_seed(seed)
    self.cfg = NS(body_names=tuple(f"b{i}" for i in range(nb)))
    self.b_pos = torch.randn(n, nb, 3, generator=g)
    self.b_quat = _rand_quat(n * nb, g).view(n, nb, 4)
    self.r_pos = torch.randn(n, nb, 3, generator=g)
    self.r_quat = _rand_quat(n * nb, g).view(n, nb, 4)
    self.body_pos_relative_w = torch.zeros(n, nb, 3)
    self.body_quat_relative_w = torch.zeros(n, nb, 4)
    self.motion_anchor_body_index = 1
    self.robot_anchor_body_index = 1

  body_pos_w = property(lambda s: s.b_pos)
  body_quat_w = property(lambda s: s.b_quat)
  anchor_pos_w = property(lambda s: s.b_pos[:, 1])
  anchor_quat_w = property(lambda s: s.b_quat[:, 1])
  robot_anchor_pos_w = property(lambda s: s.r_pos[:, 1])
  robot_anchor_quat_w = property(lambda s: s.r_quat[:, 1])
  robot_body_pos_w = property(lambda s: s.r_pos)
  robot_body_quat_w = property(lambda s: s.r_quat)


def test_relative_targets_identity_when_anchors_coincide():
  c = _Cmd()
  c.r_pos, c.r_quat = c.b_pos.clone(), c.b_quat.clone()
  c._relative_targets()
  torch.testing.assert_close(c.body_pos_relative_w, c.b_pos, atol=1e-5, rtol=1e-5)
  e = quat_error_magnitude(c.body_quat_relative_w, c.b_quat)
  assert e.abs().max() < 1e-3


def test_relative_targets_yaw_offset():
  """Robot anchor = motion anchor yawed by psi and shifted in xy: every target is the
  motion body rotated by psi about the anchor and shifted; z of the anchor is kept from
  the motion (delta_pos z = motion anchor z)."""
  c = _Cmd(seed=3)
  n = c.b_pos.shape[0]
  psi = torch.tensor([0.3, -1.0, 2.0, 0.0])
  z = torch.zeros(n)
  qy = quat_from_euler_xyz(z, z, psi)
  shift = torch.tensor([0.5, -0.2, 0.7])
  c.r_pos = c.b_pos.clone()
  c.r_pos[:, 1] = c.b_pos[:, 1] + shift
  c.r_quat = c.b_quat.clone()
  c.r_quat[:, 1] = quat_mul(qy, c.b_quat[:, 1])
  c._relative_targets()
  from mjlab_amd.math_utils import quat_apply
  nb = c.b_pos.shape[1]
  anc = c.b_pos[:, 1:2]
  exp = quat_apply(qy[:, None].expand(-1, nb, -1), c.b_pos - anc) + anc
  exp[..., :2] += shift[:2]
  torch.testing.assert_close(c.body_pos_relative_w, exp, atol=1e-5, rtol=1e-5)
  # yaw_quat keeps only the heading of the anchor offset
  yq = yaw_quat(quat_mul(c.r_quat[:, 1], tr.quat_inv(c.b_quat[:, 1])))
  assert quat_error_magnitude(yq, qy).max() < 1e-4


def _env(c):
  return NS(command_manager=NS(get_term=lambda name: c), num_envs=c.b_pos.shape[0],
            scene={"robot": NS(data=NS(gravity_vec_w=torch.tensor([[0.0, 0.0, -1.0]]).repeat(
              c.b_pos.shape[0], 1)))})


def test_reward_and_termination_formulas():
  c = _Cmd(seed=5)
  env = _env(c)
  r = tr.motion_global_anchor_position_error_exp(env, "m", std=0.3)
  exp = torch.exp(-((c.b_pos[:, 1] - c.r_pos[:, 1]) ** 2).sum(-1) / 0.09)
  torch.testing.assert_close(r, exp)
  r = tr.motion_global_anchor_orientation_error_exp(env, "m", std=0.4)
  exp = torch.exp(-quat_error_magnitude(c.b_quat[:, 1], c.r_quat[:, 1]) ** 2 / 0.16)
  torch.testing.assert_close(r, exp)
  c.body_pos_relative_w = c.b_pos + 0.1
  r = tr.motion_relative_body_position_error_exp(env, "m", std=0.3, body_names=("b0", "b2"))
  err = ((c.body_pos_relative_w - c.r_pos)[:, [0, 2]] ** 2).sum(-1).mean(-1)
  torch.testing.assert_close(r, torch.exp(-err / 0.09))
  t = tr.bad_anchor_pos_z_only(env, "m", threshold=0.25)
  torch.testing.assert_close(t, (c.b_pos[:, 1, 2] - c.r_pos[:, 1, 2]).abs() > 0.25)
  t = tr.bad_motion_body_pos_z_only(env, "m", threshold=0.25, body_names=("b2",))
  torch.testing.assert_close(t, (c.body_pos_relative_w[:, 2, 2] - c.r_pos[:, 2, 2]).abs() > 0.25)
  t = tr.bad_anchor_ori(env, NS(name="robot"), "m", threshold=0.8)
  gz = lambda q: matrix_from_quat(q)[..., 2, 2] * -1.0  # projected gravity z = -R[2,2]
  torch.testing.assert_close(t, (gz(c.b_quat[:, 1]) - gz(c.r_quat[:, 1])).abs() > 0.8)


def test_anchor_observations():
  c = _Cmd(seed=7)
  env = _env(c)
  ori = tr.motion_anchor_ori_b(env, "m")
  assert ori.shape == (4, 6)
  # 6D = first two columns of R(robot)^T R(motion), row-major flattened
  R = matrix_from_quat(c.r_quat[:, 1]).transpose(-1, -2) @ matrix_from_quat(c.b_quat[:, 1])
  torch.testing.assert_close(ori, R[..., :2].reshape(4, 6), atol=1e-5, rtol=1e-5)
  pos = tr.motion_anchor_pos_b(env, "m")
  exp = (matrix_from_quat(c.r_quat[:, 1]).transpose(-1, -2) @
         (c.b_pos[:, 1] - c.r_pos[:, 1]).unsqueeze(-1)).squeeze(-1)
  torch.testing.assert_close(pos, exp, atol=1e-5, rtol=1e-5)
  assert tr.robot_body_pos_b(env, "m").shape == (4, 9)
  assert tr.robot_body_ori_b(env, "m").shape == (4, 18)


def test_adaptive_sampling_probabilities():
  """`commands.py:272-290`: uniform floor + replicate-padded causal kernel, normalised."""
  c = _Cmd()
  c.bin_count = 11
  c.cfg = NS(adaptive_uniform_ratio=0.1, adaptive_kernel_size=3, adaptive_lambda=0.8,
             body_names=c.cfg.body_names)
  k = torch.tensor([0.8 ** i for i in range(3)])
  c.kernel = k / k.sum()
  c.bin_failed_count = torch.zeros(11)
  c.bin_failed_count[4] = 1.0
  p = c._sampling_probabilities()
  assert abs(float(p.sum()) - 1.0) < 1e-6
  base = c.bin_failed_count + 0.1 / 11
  padded = torch.cat([base, base[-1:].repeat(2)])
  exp = torch.stack([(padded[i:i + 3] * c.kernel).sum() for i in range(11)])
  torch.testing.assert_close(p, exp / exp.sum())
  assert int(p.argmax()) in (2, 3, 4)  # the failed bin pulls mass onto itself and its predecessors
  assert math.isclose(float(p[5:].min()), float(p[5:].max()), rel_tol=1e-5)


def test_task_registered():
  from mjlab_amd.envs import load_env_cfg
  cfg = load_env_cfg("Mjlab-Tracking-Flat-Unitree-G1")
  assert cfg.decimation == 4 and cfg.episode_length_s == 10.0
  assert cfg.sim.njmax == 250 and cfg.sim.nconmax == 35
  assert cfg.commands["motion"].anchor_body_name == "torso_link"
  assert len(cfg.commands["motion"].body_names) == 14
  play = load_env_cfg("Mjlab-Tracking-Flat-Unitree-G1", play=True)
  assert play.commands["motion"].sampling_mode == "start"
  assert "push_robot" not in play.events
