"""SURVEY.md 8f row f4 on the GPU: csv_to_npz through the engine's forward kinematics (all
frames as worlds of one launch) and the NaN guard around Simulation.step."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_csv_to_npz_records_the_clip(gpu_device, tmp_path):
  from mjlab_amd.motion_csv import G1_CSV_JOINTS, CsvMotion, csv_to_npz
  from mjlab_amd.tracking import MotionLoader
  T, fps = 31, 30.0
  t = np.arange(T) / fps
  pos = np.stack([0.3 * t, 0.05 * np.sin(t), 0.76 + 0.0 * t], 1)
  yaw = 0.5 * t
  quat_xyzw = np.stack([np.zeros(T), np.zeros(T), np.sin(yaw / 2), np.cos(yaw / 2)], 1)
  dof = 0.15 * np.sin(np.outer(t, np.linspace(0.5, 1.5, len(G1_CSV_JOINTS))))
  csv = tmp_path / "clip.csv"
  np.savetxt(csv, np.concatenate([pos, quat_xyzw, dof], 1), delimiter=",")
  out_file = tmp_path / "motion.npz"
  out = csv_to_npz(str(csv), str(out_file), device=gpu_device)  # asserts the root velocities
  m = CsvMotion(str(csv), 30.0, 50.0)
  assert out["joint_pos"].shape == (50, 29) and out["body_pos_w"].shape[0] == 50
  np.testing.assert_allclose(out["body_pos_w"][:, 0], m.base_pos.numpy(), atol=1e-5)
  q = out["body_quat_w"][:, 0]
  q = q * np.sign(q[:, :1] * m.base_rot[:, :1].numpy() + 1e-12)
  np.testing.assert_allclose(q, m.base_rot.numpy(), atol=1e-5)
  assert float(out["fps"][0]) == 50.0
  mot = MotionLoader(str(out_file), torch.arange(out["body_pos_w"].shape[1]), device=gpu_device)
  assert mot.time_step_total == 50
  # robot joint order: the CSV columns land on their named joints
  from mjlab_amd.scenes import load_scene
  names = [n.split("/")[-1] for n in load_scene("g1_tracking").names["joint"] if n.startswith("robot/")]
  names = [n for n in names if n != "floating_base_joint"]
  k = names.index("left_knee_joint")
  np.testing.assert_allclose(out["joint_pos"][:, k], m.dof_pos[:, G1_CSV_JOINTS.index("left_knee_joint")].numpy(),
                             atol=1e-6)


def test_nan_guard_dumps_the_bad_world(gpu_device, tmp_path):
  from mjlab_amd.scenes import load_scene
  from mjlab_amd.sim import MujocoCfg, NanGuardCfg, Simulation, SimulationCfg, load_nan_dump
  m = load_scene("go1_velocity")
  cfg = SimulationCfg(nconmax=48, njmax=160, mujoco=MujocoCfg(timestep=0.005),
                      nan_guard=NanGuardCfg(enabled=True, buffer_size=4, output_dir=str(tmp_path)))
  sim = Simulation(8, cfg, m, gpu_device)
  sim.data.qpos[:] = torch.as_tensor(m.key_qpos, dtype=torch.float32)
  for _ in range(6):
    sim.step()
  assert sim.nan_guard.last_dump is None
  sim.data.qvel[3, 2] = float("nan")
  sim.step()
  assert sim.nan_guard.last_dump is not None
  states, meta = load_nan_dump(str(tmp_path / "nan_dump_latest.npz"))
  assert meta["nan_env_ids"] == [3] and len(states) == 4
  last = states[max(states)]
  assert last.shape == (1, m.nq + m.nv) and np.isnan(last[0, m.nq + 2])
