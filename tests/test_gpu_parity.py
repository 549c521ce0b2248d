"""GPU (libmjx355, fp32) vs CPU oracle (fp64) parity on the hot path.

Tolerances (fp32 engine vs fp64 restatement, one step from identical inputs):
  kinematics (xpos, subtree_com, xquat): atol 2e-5
  velocities (cvel): atol 1e-4 + 1e-4*|v|
  smooth dynamics (qacc_smooth): rtol 1e-3 of max|qacc_smooth| per world
  constrained qacc / next qvel: rtol 2e-3 of the per-world scale (max|qacc|, >=1)
  sensors: same as the quantity they read.
Contact count must match exactly unless a contact distance is within 1e-5 of zero.
Newton iteration count: within 1 of the oracle in every world, equal in >= 90%.
"""

import numpy as np
import pytest
import torch

from parity_util import g1_states, oracle_step

pytestmark = pytest.mark.gpu


def _sim(scene, n, device):
  from mjlab_amd.scenes import load_scene
  from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
  m = load_scene(scene)
  cfg = SimulationCfg(nconmax=48, njmax=160,
                      mujoco=MujocoCfg(timestep=m.timestep, iterations=10, ls_iterations=20))
  return m, Simulation(n, cfg, m, device)


def _load(sim, q, qv, ctrl, qws=None):
  d = sim.data
  d.qpos[:] = torch.as_tensor(q, dtype=torch.float32)
  d.qvel[:] = torch.as_tensor(qv, dtype=torch.float32)
  d.ctrl[:] = torch.as_tensor(ctrl, dtype=torch.float32)
  d.qacc_warmstart[:] = 0 if qws is None else torch.as_tensor(qws, dtype=torch.float32)


@pytest.mark.parametrize("scene", ["g1_velocity", "go1_velocity"])
def test_forward_kinematics_parity(scene, gpu_device):
  m, sim = _sim(scene, 32, gpu_device)
  q, qv, ctrl = g1_states(m, 32, seed=1) if scene.startswith("g1") else _go1_states(m, 32)
  _load(sim, q, qv, ctrl)
  sim.forward()
  torch.cuda.synchronize()
  ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=False)
  d = sim.data
  xpos = d.xpos.cpu().numpy()
  stc = d.subtree_com.cpu().numpy()
  cvel = d.cvel.cpu().numpy()
  qs = d.qacc_smooth.cpu().numpy()
  for i, r in enumerate(ref):
    np.testing.assert_allclose(xpos[i], r["xpos"], atol=2e-5)
    np.testing.assert_allclose(stc[i], r["subtree_com"], atol=2e-5)
    np.testing.assert_allclose(cvel[i], r["cvel"], atol=1e-4, rtol=1e-4)
    sc = max(1.0, np.abs(r["qacc_smooth"]).max())
    np.testing.assert_allclose(qs[i], r["qacc_smooth"], atol=1e-3 * sc)


def _go1_states(m, n, seed=3):
  rng = np.random.default_rng(seed)
  q = np.tile(m.key_qpos, (n, 1))
  q[:, 2] += rng.uniform(-0.03, 0.02, n)
  q[:, 7:] += rng.uniform(-0.1, 0.1, (n, m.nq - 7))
  qv = rng.normal(0, 0.3, (n, m.nv))
  jq = np.array([m.jnt_qposadr[j] for j in m.actuator_trnid])
  ctrl = q[:, jq] + rng.uniform(-0.2, 0.2, (n, m.nu))
  return q, qv, ctrl


@pytest.mark.parametrize("scene", ["g1_velocity", "go1_velocity"])
def test_step_parity(scene, gpu_device):
  n = 48
  m, sim = _sim(scene, n, gpu_device)
  q, qv, ctrl = g1_states(m, n, seed=2) if scene.startswith("g1") else _go1_states(m, n)
  _load(sim, q, qv, ctrl)
  sim.step()
  torch.cuda.synchronize()
  ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=True)
  d = sim.data
  ncon = d.ncon.cpu().numpy()
  qacc = d.qacc.cpu().numpy()
  qvel = d.qvel.cpu().numpy()
  qpos = d.qpos.cpu().numpy()
  sens = d.sensordata.cpu().numpy()
  af = d.actuator_force.cpu().numpy()
  niter = d.solver_niter.cpu().numpy()
  ncontact_worlds = 0
  niter_equal = 0
  for i, r in enumerate(ref):
    assert ncon[i] == r["ncon"], f"world {i}: ncon {ncon[i]} vs {r['ncon']}"
    ncontact_worlds += r["ncon"] > 0
    sc = max(1.0, np.abs(r["qacc"]).max())
    np.testing.assert_allclose(qacc[i], r["qacc"], atol=2e-3 * sc, err_msg=f"qacc world {i}")
    np.testing.assert_allclose(qvel[i], r["qvel"], atol=2e-3 * sc * m.timestep + 1e-5)
    np.testing.assert_allclose(qpos[i], r["qpos"], atol=2e-3 * sc * m.timestep ** 2 + 1e-5)  # h x the qvel bound
    np.testing.assert_allclose(af[i], r["actuator_force"], atol=1e-3, rtol=1e-4)
    ssc = max(1.0, np.abs(r["sensordata"]).max())
    np.testing.assert_allclose(sens[i], r["sensordata"], atol=3e-3 * ssc, err_msg=f"sens {i}")
    # Newton stopping: same iteration count as the fp64 oracle (fp32 rounding floors on
    # MuJoCo's gradient/improvement tests), at most one off
    assert abs(int(niter[i]) - r["niter"]) <= 1, f"world {i}: niter {niter[i]} vs {r['niter']}"
    niter_equal += int(niter[i]) == r["niter"]
  assert ncontact_worlds > 0
  assert niter_equal >= 0.9 * n


@pytest.mark.parametrize("maxmatch", [1, 3])
def test_contact_sensor_maxmatch(maxmatch, gpu_device):
  """SimulationCfg.contact_sensor_maxmatch (`sim/sim.py:95,141`) reaches the engine: each
  contact sensor reduces over (and counts) its first `maxmatch` matching contacts.  The G1
  foot sensors (found + net force over each foot's 4-14 contacts) then differ from the
  64-match values, and the engine matches the oracle run with the same cap."""
  from mjlab_amd.scenes import load_scene
  from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
  n = 48
  m = load_scene("g1_velocity")
  cfg = SimulationCfg(nconmax=48, njmax=160, contact_sensor_maxmatch=maxmatch,
                      mujoco=MujocoCfg(timestep=m.timestep, iterations=10, ls_iterations=20))
  sim = Simulation(n, cfg, m, gpu_device)
  assert m.contact_maxmatch == maxmatch
  q, qv, ctrl = g1_states(m, n, seed=2)
  _load(sim, q, qv, ctrl)
  sim.step()
  torch.cuda.synchronize()
  ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=True)
  m.contact_maxmatch = 64
  full = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=True)
  d = sim.data
  ncon = d.ncon.cpu().numpy()
  sens = d.sensordata.cpu().numpy()
  truncated = 0
  for i, r in enumerate(ref):
    assert ncon[i] == r["ncon"], f"world {i}: ncon {ncon[i]} vs {r['ncon']}"
    ssc = max(1.0, np.abs(r["sensordata"]).max())
    np.testing.assert_allclose(sens[i], r["sensordata"], atol=3e-3 * ssc, err_msg=f"sens {i}")
    truncated += not np.allclose(r["sensordata"], full[i]["sensordata"])
  assert truncated > n // 4


def test_contact_sensor_maxmatch_rejects_zero(gpu_device):
  from mjlab_amd.scenes import load_scene
  from mjlab_amd.sim import Simulation, SimulationCfg
  with pytest.raises(ValueError, match="contact_sensor_maxmatch"):
    Simulation(4, SimulationCfg(contact_sensor_maxmatch=0), load_scene("g1_velocity"), gpu_device)
