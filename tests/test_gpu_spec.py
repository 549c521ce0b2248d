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


def test_spec_built_motor_velocity_position_actuators(gpu_device):
  """A model built with the MjSpec-like surface (mjlab_amd/spec.py): motor, velocity and
  position actuators (`utils/spec.py:91-202`) with their ctrl / force clamps, on the GPU
  against the oracle (actuator_force, qacc_smooth, one step)."""
  from mjlab_amd import spec as S
  from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
  from parity_util import oracle_step
  sp = S.Spec()
  b = sp.worldbody.add_body(name="base", pos=(0, 0, 1.0))
  for k, ax in enumerate(([0, 1, 0], [1, 0, 0], [0, 1, 0])):
    b = b.add_body(name=f"l{k}", pos=(0, 0, -0.15) if k else (0, 0, 0))
    b.add_joint(name=f"j{k}", axis=ax, range=[-1.5, 1.5], damping=0.05)
    b.add_geom(name=f"g{k}", type=S.mjtGeom.mjGEOM_CAPSULE, size=[0.03, 0.06], pos=(0, 0, -0.07),
               mass=0.4, contype=0, conaffinity=0)
  S.create_motor_actuator(sp, "j0", effort_limit=2.0, gear=1.5, armature=0.01)
  S.create_velocity_actuator(sp, "j1", damping=0.8, effort_limit=1.0, armature=0.01)
  S.create_position_actuator(sp, "j2", stiffness=20.0, damping=1.0, effort_limit=3.0,
                             armature=0.01)
  m = sp.compile()
  n = 32
  rng = np.random.default_rng(2)
  q = rng.uniform(-1.2, 1.2, (n, m.nq))
  qv = rng.normal(0, 1.5, (n, m.nv))
  ctrl = rng.uniform(-4, 4, (n, m.nu))
  cfg = SimulationCfg(nconmax=8, njmax=16,
                      mujoco=MujocoCfg(timestep=m.timestep, iterations=10, ls_iterations=20))
  sim = Simulation(n, cfg, m, gpu_device)
  d = sim.data
  d.qpos[:] = torch.as_tensor(q, dtype=torch.float32)
  d.qvel[:] = torch.as_tensor(qv, dtype=torch.float32)
  d.ctrl[:] = torch.as_tensor(ctrl, dtype=torch.float32)
  d.qacc_warmstart.zero_()
  sim.step()
  torch.cuda.synchronize()
  ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=True, nconmax=8, njmax=16)
  af = d.actuator_force.cpu().numpy()
  qa = d.qacc.cpu().numpy()
  clipped = 0
  for i, r in enumerate(ref):
    np.testing.assert_allclose(af[i], r["actuator_force"], atol=1e-4, rtol=1e-5)
    clipped += int(np.isclose(np.abs(r["actuator_force"]), [2.0, 1.0, 3.0]).any())
    sc = max(1.0, np.abs(r["qacc"]).max())
    np.testing.assert_allclose(qa[i], r["qacc"], atol=1e-3 * sc)
  assert clipped >= n // 4  # the force clamps are exercised
