"""Fused HIP managers (mjlab_amd/fused.py, csrc/velocity_task.hip) against the torch
manager path on identical state: rewards, per-term step rewards, terminations, command
update, observations, air-time and swing-height state, and the reset path.

Randomness is neutralised so both paths are deterministic: observation corruption off,
command and push timers pushed out of reach, reset pose ranges zero (the fused kernels
draw from a counter-based hash, the torch path from Philox; RNG streams are not
comparable, their distributions are checked separately).
Tolerances: fp32, the two paths differ only in operation order/FMA contraction:
rewards rtol 1e-4 atol 1e-5; observations atol 1e-4; flags exact."""

import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TASKS = ["Mjlab-Velocity-Flat-Unitree-G1", "Mjlab-Velocity-Flat-Unitree-Go1"]


def _env(task, n, device, fused, zero_reset_ranges=False):
  from mjlab_amd.envs import ManagerBasedRlEnv, load_env_cfg
  cfg = load_env_cfg(task, False)
  cfg.scene.num_envs = n
  cfg.seed = 3
  cfg.observations["policy"].enable_corruption = False
  if zero_reset_ranges:
    cfg.events["reset_base"].params["pose_range"] = {}
  env = ManagerBasedRlEnv(cfg, device=device)
  env.reset()
  env.enable_graph(capture=False, fused=fused)
  assert (env._fused is not None) == fused, getattr(env, "_fused_unsupported", "")
  ct = env.command_manager.get_term("twist")
  ct.time_left.fill_(1e6)
  for tl in env.event_manager._interval_time_left:
    tl.fill_(1e6)
  return env


def _close(a, b, **kw):
  torch.testing.assert_close(a.float(), b.float(), **kw)


@pytest.mark.parametrize("task", TASKS)
def test_fused_step_matches_torch(task, gpu_device):
  n = 128
  et = _env(task, n, gpu_device, fused=False)
  ef = _env(task, n, gpu_device, fused=True)
  g = torch.Generator(device=gpu_device).manual_seed(0)
  nact = et.action_manager.total_action_dim
  for step in range(6):
    a = 0.3 * (2 * torch.rand(n, nact, device=gpu_device, generator=g) - 1)
    ot, rt, tt, ut, _ = et.step(a)
    of, rf, tf, uf, _ = ef.step(a)
    torch.cuda.synchronize()
    assert torch.equal(tt, tf) and torch.equal(ut, uf)
    _close(rt, rf, rtol=1e-4, atol=1e-5)
    _close(et.reward_manager._step_reward, ef.reward_manager._step_reward, rtol=1e-4, atol=1e-4)
    for k in ("policy", "critic"):
      _close(ot[k], of[k], rtol=1e-4, atol=1e-4)
    _close(et.command_manager.get_command("twist"), ef.command_manager.get_command("twist"), rtol=1e-5, atol=1e-6)
    _close(et.sim.data.qpos, ef.sim.data.qpos, rtol=1e-4, atol=1e-4)
  fs_t, fs_f = et.scene["feet_ground_contact"], ef.scene["feet_ground_contact"]
  for k in ("current_air_time", "current_contact_time", "last_air_time", "last_contact_time"):
    _close(fs_t._air[k], fs_f._air[k], atol=1e-6, rtol=0)
  for name in et.reward_manager._term_names:
    _close(et.reward_manager._episode_sums[name], ef.reward_manager._episode_sums[name], rtol=1e-4, atol=1e-5)
  assert torch.equal(et.episode_length_buf, ef.episode_length_buf)


@pytest.mark.parametrize("task", TASKS)
def test_fused_reset_path_matches_torch(task, gpu_device):
  n = 64
  et = _env(task, n, gpu_device, fused=False, zero_reset_ranges=True)
  ef = _env(task, n, gpu_device, fused=True, zero_reset_ranges=True)
  maxlen = et.max_episode_length
  for e in (et, ef):
    e.episode_length_buf[::3] = maxlen - 1  # these envs time out on the next step
  a = torch.zeros(n, et.action_manager.total_action_dim, device=gpu_device)
  _, rt, tt, ut, _ = et.step(a)
  _, rf, tf, uf, _ = ef.step(a)
  torch.cuda.synchronize()
  assert torch.equal(ut, uf) and ut[::3].all()
  assert torch.equal(et.episode_length_buf, ef.episode_length_buf)
  assert (ef.episode_length_buf[::3] == 0).all()
  mask = ut.clone()
  # reset envs: root at default pose + origin, joints at default, velocities zero
  _close(et.sim.data.qpos[mask], ef.sim.data.qpos[mask], rtol=1e-5, atol=1e-5)
  _close(et.sim.data.qvel[mask], ef.sim.data.qvel[mask], rtol=0, atol=1e-6)
  assert (ef.action_manager.action[mask] == 0).all()
  _close(et.reward_manager._reward_buf, ef.reward_manager._reward_buf, rtol=1e-4, atol=1e-5)
  # reset logs: episode-reward means over the reset envs, termination counts
  log_t, log_f = et.extras["log"], ef.extras["log"]
  for k, v in log_t.items():
    if k.startswith("Episode_Reward/") or k.startswith("Episode_Termination/"):
      assert k in log_f, k
      _close(torch.as_tensor(v, device=gpu_device).reshape(()), log_f[k].reshape(()), rtol=1e-4, atol=1e-6)


def test_fused_release_hands_air_time_back(gpu_device):
  """A fused step hands the feet air-time buffers to the engine (mjx_sim_track_air_time);
  switching the env back to the torch managers must turn that off, or air time would
  advance twice per substep (engine phase C + ContactSensor.update).  After the switch the
  env must track air time exactly as an env that never built the fused step."""
  task = "Mjlab-Velocity-Flat-Unitree-G1"
  n = 64
  et = _env(task, n, gpu_device, fused=False)
  ef = _env(task, n, gpu_device, fused=True)
  sensor = ef.scene["feet_ground_contact"]
  assert sensor.engine_owned
  with pytest.raises(RuntimeError):
    sensor.update(0.005)
  ef.enable_graph(capture=False, fused=False)
  assert ef._fused is None and not sensor.engine_owned
  g = torch.Generator(device=gpu_device).manual_seed(1)
  nact = et.action_manager.total_action_dim
  for _ in range(8):
    a = 0.3 * (2 * torch.rand(n, nact, device=gpu_device, generator=g) - 1)
    et.step(a)
    ef.step(a)
  torch.cuda.synchronize()
  fs_t = et.scene["feet_ground_contact"]
  for k in ("current_air_time", "current_contact_time", "last_air_time", "last_contact_time"):
    _close(fs_t._air[k], sensor._air[k], atol=1e-6, rtol=0)
  assert float(sensor._air["current_air_time"].max() + sensor._air["current_contact_time"].max()) > 0


def test_fused_random_draws_in_range(gpu_device):
  """Command resampling and reset events from the counter-based RNG follow the configured
  ranges (velocity_env_cfg.py:120-136 command ranges; reset pose range)."""
  from mjlab_amd.envs import make_env
  n = 4096
  env = make_env("Mjlab-Velocity-Flat-Unitree-Go1", num_envs=n, device=gpu_device, seed=5)
  env.reset()
  env.enable_graph(capture=False, fused=True)
  assert env._fused is not None
  env.episode_length_buf.fill_(env.max_episode_length - 1)  # everyone resets
  env.step(torch.zeros(n, env.action_manager.total_action_dim, device=gpu_device))
  torch.cuda.synchronize()
  ct = env.command_manager.get_term("twist")
  tl = ct.time_left
  assert float(tl.min()) >= 3.0 - 0.02 - 1e-5 and float(tl.max()) <= 8.0
  standing = ct.is_standing_env.float().mean().item()
  heading = ct.is_heading_env.float().mean().item()
  assert abs(standing - 0.1) < 0.03 and abs(heading - 0.3) < 0.04
  c = ct.vel_command_b[~ct.is_standing_env & ~ct.is_heading_env]
  assert float(c[:, 0].min()) >= -1.0 and float(c[:, 0].max()) <= 1.0
  assert abs(float(c[:, 0].mean())) < 0.05
  h = ct.heading_target
  assert float(h.min()) >= -math.pi and float(h.max()) <= math.pi and float(h.std()) > 1.6
