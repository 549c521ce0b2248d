"""Random manager terms on the fused HIP path, as distributions (4096 envs).

The fused kernels draw from a counter-based hash of (seed, env, step, draw), not torch's
Philox stream, so their draws cannot be compared value by value with the torch managers
(test_gpu_fused*.py neutralise them).  Here each random term runs on the fused path and its
draws are isolated exactly, by differencing against a twin env whose only difference is
that the term is off, or against the deterministic reference state:
  - push_by_setting_velocity (`envs/mdp/events.py:209-223`, velocity_env_cfg.py:160):
    root linear velocity x, y += U(-0.5, 0.5); z and the angular velocity unchanged;
    the interval timers resampled in U(1, 3) s;
  - UniformNoiseCfg on the policy observations (`utils/noise/noise_cfg.py:52-77`,
    velocity_env_cfg.py:41-62): per element U(-a, a) with a = 0.5 / 0.2 / 0.05 / 0.01 /
    1.5 for base_lin_vel / base_ang_vel / projected_gravity / joint_pos / joint_vel,
    none on last_action and the command, none on the critic group;
  - reset_root_state_uniform (`envs/mdp/events.py:81-128`): root x, y offsets U(-0.5, 0.5)
    about default + env origin, yaw U(-3.14, 3.14), z / roll / pitch 0, zero velocities;
  - tracking reference-state init (`tasks/tracking/mdp/commands.py:309-375`): root position
    noise x, y U(-0.05, 0.05), z U(-0.01, 0.01); roll / pitch U(-0.1, 0.1), yaw
    U(-0.2, 0.2); root velocity noise per VELOCITY_RANGE; joint noise U(-0.1, 0.1).
Checks per component: support within [lo, hi] (+1e-5), both ends approached (within 5 % of
the width), mean within 5 sigma / sqrt(n) of the centre, variance within 8 % of
(hi - lo)^2 / 12.
"""

import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N = 4096


def _uniform_ok(x, lo, hi, what):
  x = np.asarray(x, dtype=np.float64).reshape(-1)
  n = x.size
  w = hi - lo
  assert x.min() >= lo - 1e-5 and x.max() <= hi + 1e-5, f"{what}: [{x.min()}, {x.max()}] outside [{lo}, {hi}]"
  assert x.min() < lo + 0.05 * w and x.max() > hi - 0.05 * w, f"{what}: does not cover [{lo}, {hi}]"
  sd = w / math.sqrt(12.0)
  assert abs(x.mean() - 0.5 * (lo + hi)) < 5 * sd / math.sqrt(n), f"{what}: mean {x.mean()}"
  assert abs(x.var() / sd ** 2 - 1.0) < 0.08, f"{what}: variance {x.var()} vs {sd ** 2}"


def _velocity_env(device, corruption=False, push_now=False, seed=3):
  from mjlab_amd.envs import ManagerBasedRlEnv, load_env_cfg
  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1", False)
  cfg.scene.num_envs = N
  cfg.seed = seed
  cfg.observations["policy"].enable_corruption = corruption
  env = ManagerBasedRlEnv(cfg, device=device)
  env.reset()
  env.enable_graph(capture=False, fused=True)
  assert env._fused is not None, getattr(env, "_fused_unsupported", "")
  env.command_manager.get_term("twist").time_left.fill_(1e6)
  for tl in env.event_manager._interval_time_left:
    tl.fill_(1e-6 if push_now else 1e6)
  return env


def _zero_action(env):
  return torch.zeros(env.num_envs, env.action_manager.total_action_dim, device=env.device)


def test_fused_push_velocity_distribution(gpu_device):
  ea = _velocity_env(gpu_device, push_now=True)
  eb = _velocity_env(gpu_device, push_now=False)
  ea.step(_zero_action(ea))
  eb.step(_zero_action(eb))
  torch.cuda.synchronize()
  # the push sets qvel from the root link velocity of the step's last mjData (cvel based,
  # EntityData.root_link_vel_w) plus the draw: the twin holds that velocity unpushed
  v0 = eb.scene["robot"].data.root_link_vel_w
  qa = ea.sim.data.qvel
  d = (qa[:, 0:3] - v0[:, 0:3]).cpu().numpy()
  _uniform_ok(d[:, 0], -0.5, 0.5, "push x")
  _uniform_ok(d[:, 1], -0.5, 0.5, "push y")
  assert np.abs(d[:, 2]).max() < 1e-5
  # angular velocity: unchanged (written back in the body frame)
  from mjlab_amd.math_utils import quat_apply
  wa = quat_apply(ea.sim.data.qpos[:, 3:7], qa[:, 3:6])
  torch.testing.assert_close(wa, v0[:, 3:6], atol=1e-4, rtol=1e-4)
  tl = ea.event_manager._interval_time_left[0].cpu().numpy()
  _uniform_ok(tl, 1.0, 3.0, "push interval")


def test_fused_observation_noise_distribution(gpu_device):
  ea = _velocity_env(gpu_device, corruption=True)
  eb = _velocity_env(gpu_device, corruption=False)
  oa, *_ = ea.step(_zero_action(ea))
  ob, *_ = eb.step(_zero_action(eb))
  torch.cuda.synchronize()
  diff = (oa["policy"] - ob["policy"]).cpu().numpy()
  torch.testing.assert_close(oa["critic"], ob["critic"], atol=0, rtol=0)
  nj = ea.action_manager.total_action_dim
  layout = [("base_lin_vel", 3, 0.5), ("base_ang_vel", 3, 0.2), ("projected_gravity", 3, 0.05),
            ("joint_pos", nj, 0.01), ("joint_vel", nj, 1.5), ("actions", nj, 0.0), ("command", 3, 0.0)]
  assert sum(k for _, k, _ in layout) == diff.shape[1]
  c = 0
  for name, k, a in layout:
    block = diff[:, c:c + k]
    if a == 0.0:
      assert np.abs(block).max() == 0.0, f"{name} must not be corrupted"
    else:
      # relative fp32 rounding of value + noise: widen the support check by 1e-5 * |value|
      for j in range(k):
        _uniform_ok(np.clip(block[:, j], -a, a), -a, a, f"noise {name}[{j}]")
      assert np.abs(block).max() <= a * (1 + 1e-5) + 1e-5
    c += k
  # independent draws across elements: correlation of neighbouring columns ~ 0
  jv = diff[:, 9 + nj: 9 + 2 * nj]
  r = np.corrcoef(jv[:, 0], jv[:, 1])[0, 1]
  assert abs(r) < 5 / math.sqrt(N)


def test_fused_reset_pose_distribution(gpu_device):
  env = _velocity_env(gpu_device)
  env.episode_length_buf.fill_(env.max_episode_length - 1)  # every env times out and resets
  env.step(_zero_action(env))
  torch.cuda.synchronize()
  robot = env.scene["robot"]
  q = env.sim.data.qpos
  default = robot.data.default_root_state
  off = (q[:, 0:3] - default[:, 0:3] - env.scene.env_origins).cpu().numpy()
  _uniform_ok(off[:, 0], -0.5, 0.5, "reset x")
  _uniform_ok(off[:, 1], -0.5, 0.5, "reset y")
  assert np.abs(off[:, 2]).max() < 1e-5
  from mjlab_amd.math_utils import quat_conjugate, quat_mul
  rel = quat_mul(quat_conjugate(default[:, 3:7]), q[:, 3:7]).cpu().numpy()  # yaw-only rotation
  assert np.abs(rel[:, 1:3]).max() < 1e-5
  yaw = 2.0 * np.arctan2(rel[:, 3], rel[:, 0])
  yaw = (yaw + np.pi) % (2 * np.pi) - np.pi
  _uniform_ok(yaw, -3.14, 3.14, "reset yaw")
  assert float(env.sim.data.qvel.abs().max()) == 0.0
  jq = robot.indexing.joint_q_adr
  torch.testing.assert_close(q[:, jq], robot.data.default_joint_pos, atol=1e-6, rtol=0)


def test_fused_tracking_rsi_distribution(gpu_device):
  from mjlab_amd.envs import ManagerBasedRlEnv, load_env_cfg
  from mjlab_amd.math_utils import quat_apply, quat_conjugate, quat_mul
  cfg = load_env_cfg("Mjlab-Tracking-Flat-Unitree-G1", False)
  cfg.scene.num_envs = N
  cfg.seed = 3
  mc = cfg.commands["motion"]
  mc.sampling_mode = "start"  # the reference frame of every resample is frame 0
  pr, vr, jr = dict(mc.pose_range), dict(mc.velocity_range), tuple(mc.joint_position_range)
  env = ManagerBasedRlEnv(cfg, device=gpu_device)
  env.reset()
  env.enable_graph(capture=False, fused=True)
  assert env._fused is not None, getattr(env, "_fused_unsupported", "")
  for tl in env.event_manager._interval_time_left:
    tl.fill_(1e6)
  env.episode_length_buf.fill_(env.max_episode_length - 1)
  env.step(_zero_action(env))
  torch.cuda.synchronize()
  ct = env.command_manager.get_term("motion")
  mo = ct.motion
  q, v = env.sim.data.qpos, env.sim.data.qvel
  root_p = mo.body_pos_w[0, 0] + env.scene.env_origins
  dp = (q[:, 0:3] - root_p).cpu().numpy()
  for i, k in enumerate("xyz"):
    _uniform_ok(dp[:, i], *pr[k], f"RSI position {k}")
  rel = quat_mul(q[:, 3:7], quat_conjugate(mo.body_quat_w[0, 0].expand(N, 4)))
  rel = rel * torch.sign(rel[:, :1])
  w, x, y, z = (rel[:, i].double() for i in range(4))
  roll = torch.atan2(2 * (w * x + y * z), 1 - 2 * (x * x + y * y))
  pitch = torch.asin(torch.clamp(2 * (w * y - z * x), -1, 1))
  yaw = torch.atan2(2 * (w * z + x * y), 1 - 2 * (y * y + z * z))
  for ang, k in ((roll, "roll"), (pitch, "pitch"), (yaw, "yaw")):
    _uniform_ok(ang.cpu().numpy(), *pr[k], f"RSI orientation {k}")
  dl = (v[:, 0:3] - mo.body_lin_vel_w[0, 0]).cpu().numpy()
  for i, k in enumerate("xyz"):
    _uniform_ok(dl[:, i], *vr[k], f"RSI linear velocity {k}")
  wa = quat_apply(q[:, 3:7], v[:, 3:6]) - mo.body_ang_vel_w[0, 0]
  da = wa.cpu().numpy()
  for i, k in enumerate(("roll", "pitch", "yaw")):
    _uniform_ok(da[:, i], *vr[k], f"RSI angular velocity {k}")
  robot = env.scene["robot"]
  dj = (q[:, robot.indexing.joint_q_adr] - mo.joint_pos[0]).cpu().numpy()
  lim = robot.data.soft_joint_pos_limits.cpu().numpy()
  jp = q[:, robot.indexing.joint_q_adr].cpu().numpy()
  free = (jp > lim[..., 0] + 1e-6) & (jp < lim[..., 1] - 1e-6)  # not clipped at a soft limit
  assert free.mean() > 0.9
  sel = dj[:, 0][free[:, 0]]
  _uniform_ok(sel, *jr, "RSI joint 0")
  assert np.abs(dj[free]).max() <= max(abs(jr[0]), abs(jr[1])) + 1e-5
