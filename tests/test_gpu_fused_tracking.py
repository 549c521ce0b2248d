"""Fused HIP tracking managers (mjlab_amd/fused_tracking.py, csrc/tracking_task.hip)
against the torch manager path of mjlab_amd/tracking.py on identical state: rewards,
per-term step rewards, terminations, MotionCommand state (time steps, relative body
targets, metrics), observations, the reset path (reference-state init) and the motion-end
resample.

Randomness is neutralised so both paths are deterministic: observation corruption off,
push timers out of reach, RSI pose / velocity / joint noise zero and sampling mode
"start" (the fused kernels draw from a counter-based hash, the torch path from Philox).
The startup randomisation (encoder bias, torso com, foot friction) is seeded identically.
Tolerances: fp32 with different operation order: rewards rtol 1e-4 atol 1e-5;
observations / targets atol 1e-4; flags and time steps exact."""

import pytest
import torch

pytestmark = pytest.mark.gpu

TASK = "Mjlab-Tracking-Flat-Unitree-G1"


def _env(n, device, fused, mode="start", loose=False):
  from mjlab_amd.envs import ManagerBasedRlEnv, load_env_cfg
  cfg = load_env_cfg(TASK, False)
  if loose:  # only time-outs end episodes
    for name, t in cfg.terminations.items():
      if "threshold" in t.params:
        t.params["threshold"] = 1e6
  cfg.scene.num_envs = n
  cfg.seed = 3
  cfg.observations["policy"].enable_corruption = False
  mc = cfg.commands["motion"]
  mc.pose_range, mc.velocity_range = {}, {}
  mc.joint_position_range = (0.0, 0.0)
  mc.sampling_mode = mode
  env = ManagerBasedRlEnv(cfg, device=device)
  env.reset()
  env.enable_graph(capture=False, fused=fused)
  assert (env._fused is not None) == fused, getattr(env, "_fused_unsupported", "")
  for tl in env.event_manager._interval_time_left:
    tl.fill_(1e6)
  return env


def _close(a, b, **kw):
  torch.testing.assert_close(a.float(), b.float(), **kw)


def _compare(et, ef, ot, of, rt, rf, tt, tf, ut, uf):
  assert torch.equal(tt, tf) and torch.equal(ut, uf)
  _close(rt, rf, rtol=1e-4, atol=1e-5)
  _close(et.reward_manager._step_reward, ef.reward_manager._step_reward, rtol=1e-4, atol=1e-4)
  for k in ("policy", "critic"):
    _close(ot[k], of[k], rtol=1e-4, atol=1e-4)
  ct, cf = et.command_manager.get_term("motion"), ef.command_manager.get_term("motion")
  assert torch.equal(ct.time_steps, cf.time_steps)
  _close(ct.body_pos_relative_w, cf.body_pos_relative_w, rtol=1e-5, atol=1e-4)
  _close(ct.body_quat_relative_w, cf.body_quat_relative_w, rtol=1e-5, atol=1e-4)
  for name in ct.metrics:
    if name.startswith("error_"):
      _close(ct.metrics[name], cf.metrics[name], rtol=1e-3, atol=1e-4)
  _close(et.sim.data.qpos, ef.sim.data.qpos, rtol=1e-4, atol=1e-4)
  assert torch.equal(et.episode_length_buf, ef.episode_length_buf)


def test_fused_tracking_step_matches_torch(gpu_device):
  n = 96
  et = _env(n, gpu_device, fused=False)
  ef = _env(n, gpu_device, fused=True)
  g = torch.Generator(device=gpu_device).manual_seed(0)
  nact = et.action_manager.total_action_dim
  for step in range(6):
    a = 0.3 * (2 * torch.rand(n, nact, device=gpu_device, generator=g) - 1)
    ot, rt, tt, ut, _ = et.step(a)
    of, rf, tf, uf, _ = ef.step(a)
    torch.cuda.synchronize()
    _compare(et, ef, ot, of, rt, rf, tt, tf, ut, uf)
  for name in et.reward_manager._term_names:
    _close(et.reward_manager._episode_sums[name], ef.reward_manager._episode_sums[name],
           rtol=1e-4, atol=1e-5)


def test_fused_tracking_reset_and_motion_end(gpu_device):
  """Envs that time out are reset onto the motion start; envs at the last motion frame
  resample at the motion end (reference-state init without a forward)."""
  n = 64
  et = _env(n, gpu_device, fused=False, loose=True)
  ef = _env(n, gpu_device, fused=True, loose=True)
  maxlen = et.max_episode_length
  T = et.command_manager.get_term("motion").motion.time_step_total
  for e in (et, ef):
    e.episode_length_buf[::3] = maxlen - 1                         # time out next step
    e.command_manager.get_term("motion").time_steps[1::3] = T - 1  # motion end next step
  a = torch.zeros(n, et.action_manager.total_action_dim, device=gpu_device)
  ot, rt, tt, ut, _ = et.step(a)
  of, rf, tf, uf, _ = ef.step(a)
  torch.cuda.synchronize()
  assert ut[::3].all()
  _compare(et, ef, ot, of, rt, rf, tt, tf, ut, uf)
  _close(et.sim.data.qvel, ef.sim.data.qvel, rtol=1e-4, atol=1e-4)
  cf = ef.command_manager.get_term("motion")
  assert (cf.time_steps[::3] == 1).all() and (cf.time_steps[1::3] == 0).all()  # reset: 0, then +1
  assert (ef.action_manager.action[::3] == 0).all()
  log_t, log_f = et.extras["log"], ef.extras["log"]
  for k, v in log_t.items():
    if k.startswith(("Episode_Reward/", "Episode_Termination/")):
      _close(torch.as_tensor(v, device=gpu_device).reshape(()), log_f[k].reshape(()),
             rtol=1e-4, atol=1e-6)


def test_fused_tracking_adaptive_sampling(gpu_device):
  """Adaptive sampling from the failure bins: every reset start frame lies in [0, T-1];
  failed bins gain probability (commands.py:258-307) and the sampling metrics are a
  normalised entropy in (0, 1]."""
  n = 2048
  ef = _env(n, gpu_device, fused=True, mode="adaptive")
  c = ef.command_manager.get_term("motion")
  T = c.motion.time_step_total
  c.time_steps.fill_(T // 2)  # a failure here lands in the middle bin
  ef.episode_length_buf.fill_(ef.max_episode_length - 1)
  a = torch.zeros(n, ef.action_manager.total_action_dim, device=gpu_device)
  ef.step(a)
  torch.cuda.synchronize()
  ts = c.time_steps
  assert int(ts.min()) >= 0 and int(ts.max()) <= T - 1
  assert float(ts.float().std()) > T / 8  # spread over the motion, not one frame
  ent = c.metrics["sampling_entropy"]
  assert 0.0 < float(ent.min()) <= 1.0 + 1e-6
