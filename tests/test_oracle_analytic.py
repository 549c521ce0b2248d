"""Pin the CPU oracle (oracle/oracle.c) with analytic answers and with the known-answer
values of the reference's own tests.  Physics trajectories are otherwise unpinned: no
reference test compares mj_step numerically and MuJoCo-C is absent.

  - actuator force law: tests/test_spec_utils.py:26-102 (torque = -kp (q - target) with
    the setpoint NOT clipped to the joint range; force clipped to +-effort_limit);
  - free fall: with actuation removed, every body accelerates at g, and the integrator is
    semi-implicit Euler (MuJoCo's Euler/implicitfast update qvel then qpos);
  - static contact: a robot holding its keyframe on the plane carries its weight through
    the feet (sum of foot net forces = M g);
  - OpenMP determinism: worlds are independent, results do not depend on thread count.
"""

import copy

import numpy as np
import pytest

import oracle_lib as ol
from mjlab_amd.scenes import load_scene


@pytest.fixture(scope="module")
def go1():
  return load_scene("go1_velocity")


def _unactuated(m):
  m2 = copy.deepcopy(m)
  m2.arrays["actuator_gainprm"] = np.zeros_like(m.actuator_gainprm)
  m2.arrays["actuator_biasprm"] = np.zeros_like(m.actuator_biasprm)
  return m2


def _jq(m):
  return np.array([m.jnt_qposadr[j] for j in m.actuator_trnid])


def test_free_fall_acceleration(go1):
  m = _unactuated(go1)
  q = np.array(go1.key_qpos, dtype=np.float64)
  q[2] = 5.0  # far above the plane: no contacts
  out = ol.forward(m, q)
  assert out["ncon"] == 0
  g = np.array([0.0, 0.0, -9.81])
  np.testing.assert_allclose(out["qacc"][:3], g, atol=1e-9)
  np.testing.assert_allclose(out["qacc"][3:], 0.0, atol=1e-9)
  np.testing.assert_allclose(out["qacc_smooth"], out["qacc"], atol=1e-12)


def test_free_fall_semi_implicit_euler(go1):
  m = _unactuated(go1)
  q = np.array(go1.key_qpos, dtype=np.float64)
  q[2] = 5.0
  h, K = m.timestep, 40
  qs, qv = q.copy(), np.zeros(m.nv)
  for _ in range(K):
    out = ol.forward(m, qs, qv, step=True)
    qs, qv = out["qpos"], out["qvel"]
  # v_k = -g h k ; z_K = z0 - g h^2 K(K+1)/2
  assert qv[2] == pytest.approx(-9.81 * h * K, rel=1e-12)
  assert qs[2] == pytest.approx(5.0 - 9.81 * h * h * K * (K + 1) / 2, rel=1e-12)
  np.testing.assert_allclose(qs[3:7], q[3:7], atol=1e-12)   # no rotation
  np.testing.assert_allclose(qs[7:], q[7:], atol=1e-12)     # joints unchanged


def test_position_actuator_setpoint_beyond_limit(go1):
  """test_spec_utils.py:26-67: commanding beyond the joint limit is not clipped."""
  m = go1
  u = 0
  j = m.actuator_trnid[u]
  kp = m.actuator_gainprm[u][0]
  q = np.array(m.key_qpos, dtype=np.float64)
  q[2] = 5.0
  a = m.jnt_qposadr[j]
  q[a] = 0.5
  upper = m.jnt_range[j][1]
  ctrl = q[_jq(m)].copy()
  ctrl[u] = upper + 0.6           # beyond the range, still below the effort limit
  assert kp * (ctrl[u] - q[a]) < m.actuator_forcerange[u][1]
  f = ol.forward(m, q, ctrl=ctrl)["actuator_force"][u]
  assert f == pytest.approx(-kp * (q[a] - ctrl[u]), rel=1e-9)
  f_at_limit = ol.forward(m, q, ctrl=np.where(np.arange(m.nu) == u, upper, ctrl))["actuator_force"][u]
  assert abs(f) > abs(f_at_limit) + 1e-6


def test_position_actuator_force_clipped_to_effort(go1):
  """test_spec_utils.py:69-102: force saturates at +-effort_limit."""
  m = go1
  q = np.array(m.key_qpos, dtype=np.float64)
  q[2] = 5.0
  ctrl = q[_jq(m)] + 3.0
  out = ol.forward(m, q, ctrl=ctrl)
  np.testing.assert_allclose(out["actuator_force"], m.actuator_forcerange[:, 1], rtol=1e-12)
  ctrl = q[_jq(m)] - 3.0
  out = ol.forward(m, q, ctrl=ctrl)
  np.testing.assert_allclose(out["actuator_force"], m.actuator_forcerange[:, 0], rtol=1e-12)


def test_damping_term_of_position_actuator(go1):
  """force = kp ctrl - kp q - kd qd  (biasprm = [0, -kp, -kd])."""
  m = go1
  q = np.array(m.key_qpos, dtype=np.float64)
  q[2] = 5.0
  qv = np.zeros(m.nv)
  u = 2
  j = m.actuator_trnid[u]
  qv[m.jnt_dofadr[j]] = 0.7
  ctrl = q[_jq(m)].copy()
  f = ol.forward(m, q, qv, ctrl=ctrl)["actuator_force"][u]
  assert f == pytest.approx(m.actuator_biasprm[u][2] * 0.7, rel=1e-9)


def test_standing_robot_carries_its_weight(go1):
  """Static equilibrium: the constraint force on the root's vertical dof equals M g.
  qfrc_constraint = M qacc - qfrc_smooth and, on the free joint's translational dofs,
  qfrc_smooth = -qfrc_bias (no actuator, passive or applied force acts there).
  The feet (contact sensors, netforce) carry most of it; in this pose the rear calf
  capsules also touch the plane (non-foot geoms collide: go1_constants.py:120-128)."""
  m = go1
  nw = 1
  q = np.tile(np.array(m.key_qpos, dtype=np.float64), (nw, 1))
  qv = np.zeros((nw, m.nv))
  qws = np.zeros((nw, m.nv))
  ctrl = np.ascontiguousarray(q[:, _jq(m)])
  tm = np.zeros(nw)
  ol.rollout(m, q, qv, qws, ctrl, tm, 400, outputs=False)  # settle for 2 s
  out = ol.forward(m, q[0], qv[0], qws[0], ctrl[0])
  weight = float(np.sum(m.body_mass)) * 9.81
  fz_total = (out["qM"] @ out["qacc"])[2] + out["qfrc_bias"][2]
  assert fz_total == pytest.approx(weight, rel=0.02)
  fz_feet = 0.0
  for s, name in enumerate(m.names["sensor"]):
    if name.startswith("feet_ground_contact") and name.endswith("_force"):
      fz_feet += out["sensordata"][m.sensor_adr[s] + 2]
  assert 0.85 * weight < abs(fz_feet) <= fz_total * 1.001
  assert np.linalg.norm(qv[0][:3]) < 0.05  # at rest


def test_rollout_independent_of_thread_count(go1):
  m = go1
  rng = np.random.default_rng(0)
  nw = 8
  base = np.tile(np.array(m.key_qpos, dtype=np.float64), (nw, 1))
  base[:, 2] += rng.uniform(0.0, 0.05, nw)
  res = []
  for threads in (1, 4):
    q = base.copy()
    qv = np.ascontiguousarray(rng.normal(0, 0.0, (nw, m.nv)))
    qws = np.zeros((nw, m.nv))
    ctrl = np.ascontiguousarray(q[:, _jq(m)] + 0.05)
    tm = np.zeros(nw)
    ol.rollout(m, q, qv, qws, ctrl, tm, 20, nthreads=threads, outputs=False)
    res.append((q, qv, tm))
  np.testing.assert_array_equal(res[0][0], res[1][0])
  np.testing.assert_array_equal(res[0][1], res[1][1])
  np.testing.assert_allclose(res[0][2], 20 * m.timestep)


@pytest.mark.parametrize("k", [1, 2, 5])
def test_contact_sensor_maxmatch_counts(k):
  """contact_sensor_maxmatch (sim/sim.py:95,141): a `found` sensor reports min(matches, k)
  and a sensor whose matches fit under k is unchanged."""
  from parity_util import g1_states, oracle_step
  m = load_scene("g1_velocity")
  n = 16
  q, qv, c = g1_states(m, n, seed=2)
  full = oracle_step(m, q, qv, np.zeros_like(qv), c, step=False)
  m.contact_maxmatch = k
  cap = oracle_step(m, q, qv, np.zeros_like(qv), c, step=False)
  st = np.asarray(m.arrays["sensor_type"]).ravel()
  ip = np.asarray(m.arrays["sensor_intprm"]).reshape(-1, 3)
  adr = np.asarray(m.arrays["sensor_adr"]).ravel()
  dim = np.asarray(m.arrays["sensor_dim"]).ravel()
  fsens = [s for s in range(m.nsensor) if st[s] == 4 and ip[s, 0] & 1]
  assert fsens
  capped = 0
  for a, b in zip(full, cap):
    for s in fsens:
      nf = a["sensordata"][adr[s]]
      assert b["sensordata"][adr[s]] == min(nf, k)
      capped += nf > k
      if nf <= k:  # every match kept: the whole sensor is unchanged
        np.testing.assert_array_equal(a["sensordata"][adr[s]:adr[s] + dim[s]],
                                      b["sensordata"][adr[s]:adr[s] + dim[s]])
  assert capped > 0
