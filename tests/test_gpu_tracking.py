"""Tracking task (`Mjlab-Tracking-Flat-Unitree-G1`) on the GPU.

Properties checked (size independent, no reference vectors exist for this path):
  - the synthetic motion is self-consistent: writing frame k's root/joint state and
    running forward reproduces its recorded body poses (the csv_to_npz contract);
  - reference-state init in play mode (no pose/velocity/joint noise, sampling "start")
    puts every robot body exactly on the motion, so the tracking errors are ~0 and the
    exp-kernel rewards are ~1 right after reset;
  - observation sizes match the reference (policy 160, critic 286);
  - per-world body_ipos randomisation (the base_com startup event) reaches the engine;
  - the sync-free graph-captured step equals the eager step on a deterministic config.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TASK = "Mjlab-Tracking-Flat-Unitree-G1"


def _env(device, n, play=False, seed=3):
  from mjlab_amd.envs import ManagerBasedRlEnv, load_env_cfg
  cfg = load_env_cfg(TASK, play=play)
  if play:  # play keeps the joint-position RSI noise (env_cfgs.py:86-98); zero it here
    cfg.commands["motion"].joint_position_range = (0.0, 0.0)
  cfg.scene.num_envs = n
  cfg.seed = seed
  return ManagerBasedRlEnv(cfg, device=device)


def test_motion_is_forward_consistent(gpu_device):
  from mjlab_amd.tracking import MotionLoader, SYNTHETIC_G1_MOTION, ensure_synthetic_motion
  ensure_synthetic_motion(SYNTHETIC_G1_MOTION, gpu_device)
  with np.load(SYNTHETIC_G1_MOTION) as z:
    assert z["joint_pos"].shape == (500, 29) and z["body_pos_w"].shape == (500, 30, 3)
    assert z["body_quat_w"].shape == (500, 30, 4) and float(z["fps"][0]) == 50.0
    jp = z["joint_pos"]
    # joint velocity is the time derivative of joint position (central differences)
    fd = (jp[2:] - jp[:-2]) * 50.0 / 2
    jv = z["joint_vel"][1:-1]
    moving = np.abs(fd) > 0
    assert np.abs(fd - jv)[moving].max() < 0.05
    # root linear velocity = d/dt root position
    bp = z["body_pos_w"][:, 0]
    fdv = (bp[2:] - bp[:-2]) * 25.0
    assert np.abs(fdv - z["body_lin_vel_w"][1:-1, 0]).max() < 2e-3


def test_play_reset_puts_robot_on_motion(gpu_device):
  env = _env(gpu_device, 8, play=True)
  env.reset()
  torch.cuda.synchronize()
  c = env.command_manager.get_term("motion")
  assert int(c.time_steps.max()) == 0
  d = (c.robot_body_pos_w - c.body_pos_w).abs().max().item()
  assert d < 1e-4, d
  from mjlab_amd.math_utils import quat_error_magnitude
  assert quat_error_magnitude(c.robot_body_quat_w, c.body_quat_w).max().item() < 1e-3
  # encoder bias only biases the observation, the joint state is the motion's
  assert (c.robot_joint_pos - c.joint_pos).abs().max().item() < 1e-5
  obs = env.obs_buf
  assert obs["policy"].shape == (8, 160) and obs["critic"].shape == (8, 286)
  # zero tracking error -> exp rewards at 1 (anchor pos / ori terms)
  from mjlab_amd import tracking as tr
  r = tr.motion_global_anchor_position_error_exp(env, "motion", std=0.3)
  assert (r > 0.9999).all()


def test_body_ipos_randomized_per_world(gpu_device):
  env = _env(gpu_device, 16)
  ipos = env.sim.model.body_ipos
  assert ipos.shape[0] == 16
  tid = env.scene["robot"].indexing.body_ids[env.scene["robot"].body_names.index("torso_link")]
  base = env.sim.get_default_field("body_ipos")[tid]
  delta = ipos[:, tid] - base
  assert delta[:, 0].abs().max() <= 0.025 + 1e-6 and delta[:, 1:].abs().max() <= 0.05 + 1e-6
  assert delta.std(0).min() > 0  # distinct per world
  other = [i for i in range(ipos.shape[1]) if i != int(tid)]
  assert torch.equal(ipos[:, other], env.sim.get_default_field("body_ipos")[other].expand(16, -1, -1))


def test_tracking_graph_step_matches_eager(gpu_device):
  """Play config (deterministic: no obs noise, no push, no RSI noise, sampling 'start'):
  K eager steps and K graph-replayed sync-free steps give the same state."""
  n, K = 64, 12
  outs = []
  for graph in (False, True):
    env = _env(gpu_device, n, play=True, seed=11)
    env.reset()
    if graph:
      env.enable_graph(capture=True)
    g = torch.Generator(device=gpu_device).manual_seed(0)
    nact = env.action_manager.total_action_dim
    for _ in range(K):
      obs, rew, term, trunc, _ = env.step(0.3 * (2 * torch.rand(n, nact, device=gpu_device, generator=g) - 1))
    torch.cuda.synchronize()
    outs.append((obs["policy"].clone(), rew.clone(), env.sim.data.qpos.clone()))
  for a, b in zip(*outs):
    torch.testing.assert_close(a, b, atol=1e-4, rtol=1e-4)


def test_tracking_training_graph_step(gpu_device):
  """Training config (noise, pushes, adaptive sampling, RSI) through the captured
  sync-free step: finite outputs, motion-end resampling wraps time steps."""
  n = 128
  env = _env(gpu_device, n)
  env.reset()
  env.enable_graph(capture=True)
  c = env.command_manager.get_term("motion")
  c.time_steps.fill_(c.motion.time_step_total - 3)
  g = torch.Generator(device=gpu_device).manual_seed(0)
  nact = env.action_manager.total_action_dim
  for _ in range(10):
    obs, rew, term, trunc, _ = env.step(2 * torch.rand(n, nact, device=gpu_device, generator=g) - 1)
  torch.cuda.synchronize()
  for v in obs.values():
    assert torch.isfinite(v).all()
  assert torch.isfinite(rew).all()
  assert int(c.time_steps.max()) < c.motion.time_step_total
  assert env.sim.stats()["unsupported"] == 0
