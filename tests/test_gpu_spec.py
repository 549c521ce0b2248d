"""Model-specialised step kernels (csrc/specs.inc).

The shipped task scenes must run on their specialised kernels, and those kernels must
agree with the generic kernels (same source, run-time dims) on the same inputs.  Both
paths are checked against the fp64 oracle by test_gpu_parity.py (nconmax 48 / njmax 160
select the specialisation there; other capacities run the generic kernels)."""

import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _spec(sim):
  from mjlab_amd._lib import lib
  return int(lib().mjx_sim_spec(sim._sim))


@pytest.mark.parametrize("task", ["Mjlab-Velocity-Flat-Unitree-G1", "Mjlab-Velocity-Flat-Unitree-Go1",
                                  "Mjlab-Tracking-Flat-Unitree-G1", "Mjlab-Jump-Flat-Unitree-G1",
                                  "Mjlab-Jump-Hfield-Unitree-G1"])
def test_shipped_tasks_use_specialised_kernels(task, gpu_device):
  from mjlab_amd.envs import make_env
  env = make_env(task, num_envs=8, device=gpu_device, seed=0)
  assert _spec(env.sim) > 0, f"{task} fell back to the generic kernels (regenerate specs.inc)"


def _make_sim(scene, n, generic):
  from mjlab_amd.scenes import load_scene
  from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
  m = load_scene(scene)
  old = os.environ.get("MJX355_NO_SPEC")
  if generic:
    os.environ["MJX355_NO_SPEC"] = "1"
  try:
    sim = Simulation(n, SimulationCfg(nconmax=48, njmax=160, mujoco=MujocoCfg(
        timestep=m.timestep, iterations=10, ls_iterations=20)), m, "cuda:0")
  finally:
    if old is None:
      os.environ.pop("MJX355_NO_SPEC", None)
    else:
      os.environ["MJX355_NO_SPEC"] = old
  return m, sim


@pytest.mark.parametrize("scene", ["g1_velocity", "go1_velocity"])
def test_specialised_matches_generic(scene, gpu_device):
  n = 64
  m, s_spec = _make_sim(scene, n, generic=False)
  _, s_gen = _make_sim(scene, n, generic=True)
  assert _spec(s_spec) > 0 and _spec(s_gen) == 0
  rng = np.random.default_rng(5)
  q = np.tile(m.key_qpos, (n, 1))
  q[:, 2] -= rng.uniform(0.0, 0.06, n)  # press into the ground: contacts and limits
  qv = rng.normal(0, 0.3, (n, m.nv))
  jq = [m.jnt_qposadr[j] for j in m.actuator_trnid]
  ctrl = q[:, jq] + rng.uniform(-0.2, 0.2, (n, m.nu))
  for s in (s_spec, s_gen):
    s.data.qpos[:] = torch.tensor(q, dtype=torch.float32)
    s.data.qvel[:] = torch.tensor(qv, dtype=torch.float32)
    s.data.ctrl[:] = torch.tensor(ctrl, dtype=torch.float32)
  s_spec.step()
  s_gen.step()
  torch.cuda.synchronize()
  assert s_spec.stats()["max_ncon"] > 0
  for f in ("qpos", "qvel", "qacc", "sensordata", "xpos", "cvel"):
    a = getattr(s_spec.data, f).cpu().numpy()
    b = getattr(s_gen.data, f).cpu().numpy()
    scale = max(1.0, float(np.abs(b).max()))
    assert np.abs(a - b).max() <= 1e-4 * scale, f"{scene} {f}: spec vs generic {np.abs(a - b).max()}"
