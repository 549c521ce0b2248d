"""SURVEY.md 8f row f4 on CPU: the retargeted-motion pipeline's resampling and velocities
(`scripts/csv_to_npz.py:22-179` restated in mjlab_amd/motion_csv.py) against plain numpy
and per-row `quat_slerp` (`utils/lab_api/math.py:1695-1728`) semantics, and the NaN guard
(`utils/nan_guard.py`) on host tensors: rolling buffer, detection over qpos / qvel / qacc /
qacc_warmstart, one dump with the reference's keys."""

import math
import types

import numpy as np
import pytest
import torch

from mjlab_amd.motion_csv import CsvMotion, quat_slerp_rows
from mjlab_amd.sim import NanGuard, NanGuardCfg, load_nan_dump


def _slerp_ref(q1, q2, tau):
  """quat_slerp, one pair at a time, in the reference's branch order (float32)."""
  eps = float(np.finfo(np.float32).eps) * 4.0
  q1, q2 = q1.astype(np.float32), q2.astype(np.float32).copy()
  if tau == 0.0:
    return q1
  if tau == 1.0:
    return q2
  d = float(np.dot(q1, q2))
  if abs(abs(d) - 1.0) < eps:
    return q1
  if d < 0.0:
    d, q2 = -d, -q2
  ang = math.acos(min(max(d, -1.0), 1.0))
  if abs(ang) < eps:
    return q1
  return q1 * math.sin((1 - tau) * ang) / math.sin(ang) + q2 * math.sin(tau * ang) / math.sin(ang)


def test_row_slerp_matches_the_per_pair_reference():
  rng = np.random.default_rng(0)
  a = rng.normal(size=(64, 4)); a /= np.linalg.norm(a, axis=1, keepdims=True)
  b = rng.normal(size=(64, 4)); b /= np.linalg.norm(b, axis=1, keepdims=True)
  b[5] = a[5]; b[6] = -a[6]  # parallel, antiparallel
  tau = rng.uniform(0, 1, 64).astype(np.float32)
  tau[0], tau[1] = 0.0, 1.0
  got = quat_slerp_rows(torch.tensor(a, dtype=torch.float32), torch.tensor(b, dtype=torch.float32),
                        torch.tensor(tau)).numpy()
  want = np.stack([_slerp_ref(a[i], b[i], float(tau[i])) for i in range(64)])
  np.testing.assert_allclose(got, want, atol=2e-6)


def _write_csv(path, T=31, fps=30.0, nj=29, yaw_rate=0.6):
  t = np.arange(T) / fps
  pos = np.stack([0.3 * t, 0.1 * np.sin(t), 0.75 + 0.01 * t], 1)
  yaw = yaw_rate * t
  quat_xyzw = np.stack([np.zeros(T), np.zeros(T), np.sin(yaw / 2), np.cos(yaw / 2)], 1)
  dof = 0.2 * np.sin(np.outer(t, np.linspace(0.5, 1.5, nj)))
  np.savetxt(path, np.concatenate([pos, quat_xyzw, dof], 1), delimiter=",")
  return t, pos, yaw, dof


def test_csv_motion_resampling_and_velocities(tmp_path):
  f = tmp_path / "clip.csv"
  t, pos, yaw, dof = _write_csv(f)
  m = CsvMotion(str(f), input_fps=30.0, output_fps=50.0)
  # duration (31 - 1) / 30 = 1 s at 50 fps: times 0, 0.02, ..., 0.98
  assert m.output_frames == 50
  to = np.arange(50) * 0.02
  np.testing.assert_allclose(m.base_pos.numpy(), np.stack([np.interp(to, t, pos[:, k]) for k in range(3)], 1),
                             atol=1e-5)
  np.testing.assert_allclose(m.dof_pos[:, 3].numpy(), np.interp(to, t, dof[:, 3]), atol=1e-5)
  # wxyz after the xyzw column swap; yaw slerps linearly between frames
  np.testing.assert_allclose(m.base_rot[:, 0].numpy(), np.cos(0.6 * to / 2), atol=1e-5)
  np.testing.assert_allclose(m.base_rot[:, 3].numpy(), np.sin(0.6 * to / 2), atol=1e-5)
  # torch.gradient (central inside, one-sided at the ends) and the SO(3) central difference
  np.testing.assert_allclose(m.base_lin_vel.numpy(), np.gradient(m.base_pos.numpy(), 0.02, axis=0),
                             atol=1e-4)
  np.testing.assert_allclose(m.base_ang_vel[:, 2].numpy(), 0.6, atol=1e-3)
  np.testing.assert_allclose(m.base_ang_vel[:, :2].numpy(), 0.0, atol=2e-5)  # fp32 log map
  sub = CsvMotion(str(f), 30.0, 50.0, line_range=(2, 11))  # 1-based inclusive rows
  assert sub.input_frames == 10
  np.testing.assert_allclose(sub.base_pos_in[0].numpy(), pos[1], atol=1e-6)


def _data(n, nq=5, nv=4):
  return types.SimpleNamespace(qpos=torch.zeros(n, nq), qvel=torch.zeros(n, nv),
                               qacc=torch.zeros(n, nv), qacc_warmstart=torch.zeros(n, nv))


def test_nan_guard_buffers_and_dumps_once(tmp_path):
  from mjlab_amd.scenes import load_scene
  model = load_scene("go1_velocity")
  guard = NanGuard(NanGuardCfg(enabled=True, buffer_size=3, output_dir=str(tmp_path), max_envs_to_dump=2),
                   num_envs=6, model=model)
  d = _data(6, model.nq, model.nv)
  for k in range(5):
    with guard.watch(d):
      d.qpos += 1.0
  assert guard.last_dump is None and len(guard.buffer) == 3
  with guard.watch(d):
    d.qacc_warmstart[4, 1] = float("inf")
    d.qvel[1, 0] = float("nan")
  assert guard.last_dump is not None
  states, meta = load_nan_dump(str(tmp_path / "nan_dump_latest.npz"))
  assert sorted(states) == ["states_step_000003", "states_step_000004", "states_step_000005"]
  assert meta["nan_env_ids"] == [1, 4] and meta["dumped_env_ids"] == [1, 4]
  assert meta["state_size"] == model.nq + model.nv and meta["detection_step"] == 6
  s5 = states["states_step_000005"]  # captured before the step that went bad
  assert s5.shape == (2, model.nq + model.nv)
  np.testing.assert_array_equal(s5[:, :model.nq], 5.0)
  assert (tmp_path / "model_latest.npz").exists()
  # once per run
  with guard.watch(d):
    pass
  assert len(list(tmp_path.glob("nan_dump_2*.npz"))) == 1
  off = NanGuard(NanGuardCfg(), 6, model)
  with off.watch(d):
    pass
  assert not off.enabled
