"""Known answers held by the reference's own tests, restated against this build's managers
and tracking metrics (CPU; the fused-HIP counterparts are in test_gpu_known_answers.py).

  - `tests/test_rewards.py:235-273`: the RewardManager turns NaN / +Inf / -Inf term values
    into 0 (`managers/reward_manager.py:77-91`, nan_to_num after weight * dt);
  - `tests/test_tracking_metrics.py:36-155`: MPKPE, root-relative MPKPE, joint-velocity
    error, end-effector position and orientation errors (`tasks/tracking/mdp/metrics.py`).
The expected values are the reference tests' own numbers.
"""

import math
from types import SimpleNamespace

import pytest
import torch

from mjlab_amd.managers import RewardManager, RewardTermCfg
from mjlab_amd.tracking_metrics import (compute_ee_orientation_error, compute_ee_position_error,
                                        compute_joint_velocity_error, compute_mpkpe,
                                        compute_root_relative_mpkpe)


@pytest.fixture
def mock_env():
  return SimpleNamespace(num_envs=4, device="cpu", max_episode_length_s=10.0, scene=None)


def test_reward_manager_handles_nan_values(mock_env):
  def nan_reward(env):
    r = torch.ones(env.num_envs, device=env.device)
    r[1] = float("nan")
    r[3] = float("inf")
    return r

  manager = RewardManager({"nan_term": RewardTermCfg(func=nan_reward, weight=1.0, params={})}, mock_env)
  rewards = manager.compute(dt=0.01)
  assert not torch.isnan(rewards).any() and not torch.isinf(rewards).any()
  assert rewards[0] == pytest.approx(0.01)
  assert rewards[1] == 0.0
  assert rewards[2] == pytest.approx(0.01)
  assert rewards[3] == 0.0
  # the episode sums and per-term step rewards see the cleaned values too
  assert torch.isfinite(manager._episode_sums["nan_term"]).all()
  assert torch.isfinite(manager._step_reward).all()


def test_reward_manager_handles_neginf_values(mock_env):
  def neginf_reward(env):
    r = torch.ones(env.num_envs, device=env.device)
    r[2] = float("-inf")
    return r

  manager = RewardManager({"neginf_term": RewardTermCfg(func=neginf_reward, weight=1.0, params={})}, mock_env)
  rewards = manager.compute(dt=0.01)
  assert not torch.isinf(rewards).any()
  assert rewards[2] == 0.0


BODIES = ("pelvis", "left_knee", "right_knee", "left_ankle", "right_ankle", "left_wrist", "right_wrist")


@pytest.fixture
def cmd():
  return SimpleNamespace(num_envs=4, device="cpu", cfg=SimpleNamespace(body_names=BODIES))


def test_mpkpe_zero_when_positions_match(cmd):
  p = torch.rand(cmd.num_envs, len(BODIES), 3)
  cmd.body_pos_relative_w, cmd.robot_body_pos_w = p.clone(), p.clone()
  m = compute_mpkpe(cmd)
  assert m.shape == (cmd.num_envs,)
  assert torch.allclose(m, torch.zeros(cmd.num_envs), atol=1e-6)


def test_mpkpe_correct_error(cmd):
  cmd.body_pos_relative_w = torch.zeros(cmd.num_envs, len(BODIES), 3)
  cmd.robot_body_pos_w = torch.zeros(cmd.num_envs, len(BODIES), 3)
  cmd.robot_body_pos_w[:, :, 0] = 1.0
  assert torch.allclose(compute_mpkpe(cmd), torch.ones(cmd.num_envs), atol=1e-6)


def test_r_mpkpe_invariant_to_global_translation(cmd):
  nb = len(BODIES)
  cmd.anchor_pos_w = torch.zeros(cmd.num_envs, 3)
  cmd.body_pos_w = torch.rand(cmd.num_envs, nb, 3)
  cmd.robot_anchor_pos_w = torch.zeros(cmd.num_envs, 3)
  cmd.robot_body_pos_w = cmd.body_pos_w.clone()
  r1 = compute_root_relative_mpkpe(cmd)
  off = torch.tensor([100.0, 200.0, 300.0])
  cmd.anchor_pos_w = off.expand(cmd.num_envs, 3).clone()
  cmd.body_pos_w = cmd.body_pos_w + off
  cmd.robot_anchor_pos_w = off.expand(cmd.num_envs, 3).clone()
  cmd.robot_body_pos_w = cmd.robot_body_pos_w + off
  assert torch.allclose(r1, compute_root_relative_mpkpe(cmd), atol=1e-5)


def test_r_mpkpe_detects_relative_error(cmd):
  nb = len(BODIES)
  cmd.anchor_pos_w = torch.zeros(cmd.num_envs, 3)
  cmd.body_pos_w = torch.zeros(cmd.num_envs, nb, 3)
  cmd.body_pos_w[:, :, 0] = 1.0
  cmd.robot_anchor_pos_w = torch.zeros(cmd.num_envs, 3)
  cmd.robot_body_pos_w = torch.zeros(cmd.num_envs, nb, 3)
  cmd.robot_body_pos_w[:, :, 0] = 2.0
  assert torch.allclose(compute_root_relative_mpkpe(cmd), torch.ones(cmd.num_envs), atol=1e-6)


def test_joint_velocity_error(cmd):
  cmd.joint_vel = torch.zeros(cmd.num_envs, 3)
  cmd.robot_joint_vel = torch.zeros(cmd.num_envs, 3)
  cmd.robot_joint_vel[:, 0] = 3.0
  cmd.robot_joint_vel[:, 1] = 4.0
  assert torch.allclose(compute_joint_velocity_error(cmd), torch.full((cmd.num_envs,), 5.0), atol=1e-6)


def test_ee_position_error_only_uses_specified_bodies(cmd):
  nb = len(BODIES)
  cmd.body_pos_relative_w = torch.zeros(cmd.num_envs, nb, 3)
  cmd.robot_body_pos_w = torch.zeros(cmd.num_envs, nb, 3)
  cmd.robot_body_pos_w[:, 0, :] = 100.0
  cmd.robot_body_pos_w[:, 3, 0] = 1.0
  cmd.robot_body_pos_w[:, 4, 0] = 1.0
  e = compute_ee_position_error(cmd, ("left_ankle", "right_ankle"))
  assert torch.allclose(e, torch.ones(cmd.num_envs), atol=1e-6)


def test_ee_orientation_error_detects_rotation(cmd):
  nb = len(BODIES)
  ident = torch.tensor([1.0, 0.0, 0.0, 0.0])
  cmd.body_quat_relative_w = ident.view(1, 1, 4).expand(cmd.num_envs, nb, 4).clone()
  rot = torch.tensor([0.7071, 0.0, 0.0, 0.7071])
  cmd.robot_body_quat_w = rot.view(1, 1, 4).expand(cmd.num_envs, nb, 4).clone()
  e = compute_ee_orientation_error(cmd, ("left_wrist",))
  assert torch.allclose(e, torch.full((cmd.num_envs,), 3.14159 / 2), atol=0.01)


def test_ee_errors_empty_selection(cmd):
  nb = len(BODIES)
  cmd.body_pos_relative_w = torch.rand(cmd.num_envs, nb, 3)
  cmd.robot_body_pos_w = torch.rand(cmd.num_envs, nb, 3)
  assert (compute_ee_position_error(cmd, ("no_such_body",)) == 0).all()
  assert math.isfinite(float(compute_mpkpe(cmd).sum()))
