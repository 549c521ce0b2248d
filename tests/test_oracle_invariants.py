"""The oracle pinned by classical mechanics rather than by its own formulas (tests/invariants.py;
SURVEY.md section 7 build step 1: pendulum period, energy drift).

Each check uses only the compiled masses / inertias, the position-level kinematics and
finite differences, so a misconception shared by the oracle's CRB / RNE / solver and the
engine (which mirrors them) would fail here."""

import copy

import numpy as np
import pytest

import invariants as inv
from mjlab_amd.scenes import load_scene
from oracle_sim import OracleData


@pytest.fixture(scope="module")
def g1():
  return load_scene("g1_velocity")


def _random_state(m, seed, vscale=1.0, z=50.0):
  rng = np.random.default_rng(seed)
  q = np.array(m.key_qpos, float)
  q[2] = z
  q[7:] += rng.uniform(-0.3, 0.3, m.nq - 7)
  ang = rng.normal(0, 0.3, 3)
  q[3:7] = inv.integrate_pos(m, q, np.r_[np.zeros(3), ang, np.zeros(m.nv - 6)], 1.0)[3:7]
  v = rng.normal(0, vscale, m.nv)
  return q, v


def test_pendulum_small_angle_period():
  m = inv.pendulum(L=0.5)
  T = inv.pendulum_period(m)
  od = OracleData(m)
  od.qpos[0] = 0.02
  ts, th = [], []
  for k in range(int(4 * T / m.timestep)):
    od.step()
    ts.append(od.time)
    th.append(od.qpos[0])
  Tn = inv.zero_crossing_period(ts, th)
  # semi-implicit Euler shifts the period by O((w h)^2) ~ 1e-5 at h = 1 ms; the amplitude
  # correction theta0^2 / 16 is 2.5e-5
  assert Tn == pytest.approx(T, rel=2e-4)
  assert max(abs(x) for x in th) == pytest.approx(0.02, rel=1e-2)  # no damping: amplitude kept


@pytest.mark.parametrize("seed", [0, 1])
def test_kinetic_energy_from_body_twists(g1, seed):
  """1/2 v'Mv (CRB mass matrix) == sum of body kinetic energies from finite-difference twists."""
  m = inv.free_floating(g1)
  od = OracleData(m)
  q, v = _random_state(m, seed)
  M = inv.mass_matrix(od, q)
  xi, R = inv.body_pose(od, q)
  vb, wb = inv.fd_twists(od, q, v)
  ke_bodies = inv.kinetic_energy_bodies(m, R, vb, wb, v)
  assert 0.5 * v @ M @ v == pytest.approx(ke_bodies, rel=1e-8)
  # and the oracle's com-based velocities (cvel) describe the same twists
  od.qpos[:], od.qvel[:] = q, v
  od.forward()
  vc, wc = inv.twists_from_cvel(m, od.xipos, od.subtree_com, od.cvel)
  np.testing.assert_allclose(vc[1:], vb[1:], atol=1e-7)
  np.testing.assert_allclose(wc[1:], wb[1:], atol=1e-7)


def test_kinetic_energy_hinge_tree():
  m = inv.hinge_tree()
  od = OracleData(m)
  rng = np.random.default_rng(3)
  q, v = rng.uniform(-1, 1, m.nq), rng.normal(0, 2, m.nv)
  M = inv.mass_matrix(od, q)
  xi, R = inv.body_pose(od, q)
  vb, wb = inv.fd_twists(od, q, v)
  assert 0.5 * v @ M @ v == pytest.approx(inv.kinetic_energy_bodies(m, R, vb, wb, v), rel=1e-8)


def test_bias_forces_from_lagrange_hinge_tree():
  """qfrc_bias (RNE) == d/dt(M) v - dT/dq + dU/dq (finite differences of M(q) and U(q))
  on every dof of a branching hinge tree with skewed axes, armature and gravity."""
  m = inv.hinge_tree()
  od = OracleData(m)
  rng = np.random.default_rng(4)
  for _ in range(3):
    q, v = rng.uniform(-1.5, 1.5, m.nq), rng.normal(0, 2, m.nv)
    od.qpos[:], od.qvel[:] = q, v
    od.forward()
    bias = od.qfrc_bias.copy()
    lag = inv.lagrange_bias(od, q, v, range(m.nv))
    want = np.array([lag[i] for i in range(m.nv)])
    np.testing.assert_allclose(bias, want, rtol=1e-6, atol=1e-6 * max(1.0, np.abs(want).max()))


def test_bias_forces_from_lagrange_g1(g1):
  """The same on the free-floating G1 for every dof with a true coordinate: the free
  joint's three translations and the 29 hinges (the free joint's rotational dofs are
  quasi-velocities, whose equations carry Boltzmann-Hamel terms)."""
  m = inv.free_floating(g1, gravity=(0.0, 0.0, -inv.G))
  od = OracleData(m)
  q, v = _random_state(m, 7, vscale=0.7)
  od.qpos[:], od.qvel[:] = q, v
  od.forward()
  bias = od.qfrc_bias.copy()
  rows = [0, 1, 2] + list(range(6, m.nv))
  lag = inv.lagrange_bias(od, q, v, rows)
  for i in rows:
    assert bias[i] == pytest.approx(lag[i], rel=1e-5, abs=1e-5 * max(1.0, abs(lag[i]))), f"dof {i}"


def _energy_drift(m, q0, v0, h, T=1.0):
  m = copy.copy(m)
  m.timestep = h
  m.integrator = 0  # Euler (semi-implicit)
  od = OracleData(m)
  od.qpos[:], od.qvel[:] = q0, v0

  def energy():
    q, v = od.qpos.copy(), od.qvel.copy()
    M = inv.mass_matrix(od, q)
    xi, _ = inv.body_pose(od, q)
    return 0.5 * v @ M @ v + inv.potential(m, xi)

  q, v = od.qpos.copy(), od.qvel.copy()
  E0 = energy()
  od.qpos[:], od.qvel[:] = q, v
  worst = 0.0
  for k in range(int(round(T / h))):
    od.step()
    if k % 10 == 9:
      q, v = od.qpos.copy(), od.qvel.copy()
      worst = max(worst, abs(energy() - E0))
      od.qpos[:], od.qvel[:] = q, v
  return worst, E0, 0.5 * v0 @ inv.mass_matrix(od, q0) @ v0


def test_energy_drift_first_order(g1):
  """Unactuated, undamped, contact-free G1 for 1 s of semi-implicit Euler steps.  Without
  gravity the energy is kept to O(h) (small, and halved with h).  In gravity the drift is the
  integrator's free-fall error, 1/2 M g^2 h T (v_k = -g h k, z_k = -g h^2 k (k + 1) / 2),
  again halved with h."""
  for grav in ((0.0, 0.0, 0.0), (0.0, 0.0, -inv.G)):
    m = inv.free_floating(g1, gravity=grav)
    q, v = _random_state(m, 11, vscale=1.0)
    d1, E0, ke = _energy_drift(m, q, v, 0.005)
    d2, _, _ = _energy_drift(m, q, v, 0.0025)
    assert 1.8 < d1 / d2 < 2.2, (grav, d1, d2)
    if grav[2] == 0.0:
      assert d1 < 0.02 * ke, (d1, ke)
      internal = d1
    else:
      free_fall = 0.5 * float(np.sum(m.body_mass)) * inv.G ** 2 * 0.005 * 1.0
      assert abs(d1 - free_fall) <= 0.05 * free_fall + internal, (d1, free_fall)


def _momenta_at(od, q, v):
  m = od.model
  od.qpos[:], od.qvel[:] = q, v
  od.forward()
  vb, wb = inv.twists_from_cvel(m, od.xipos, od.subtree_com, od.cvel)
  return inv.momenta(m, od.xipos, od.ximat.reshape(-1, 3, 3), vb, wb)


@pytest.mark.parametrize("gravity", [0.0, -inv.G])
def test_momentum_rate_equals_external_force(g1, gravity):
  """Newton-Euler for the whole free-floating G1 (no contacts, limits or actuators): the
  oracle's forward dynamics qacc must give dP/dt = M_total g and dL/dt = 0 about the com.
  The rates are central differences of the momenta along the motion (q(t +- e) from v and
  qacc), with body twists from cvel (pinned by the kinetic-energy test above)."""
  m = inv.free_floating(g1, gravity=(0.0, 0.0, gravity))
  od = OracleData(m)
  q, v = _random_state(m, 5, vscale=1.5)
  od.qpos[:], od.qvel[:] = q, v
  od.forward()
  a = od.qacc.copy()
  e = 1e-4
  Mt, _, Pp, Lp = _momenta_at(od, inv.integrate_pos(m, q, e * v + 0.5 * e * e * a, 1.0), v + e * a)
  _, _, Pm, Lm = _momenta_at(od, inv.integrate_pos(m, q, -e * v + 0.5 * e * e * a, 1.0), v - e * a)
  dP, dL = (Pp - Pm) / (2 * e), (Lp - Lm) / (2 * e)
  scale = Mt * max(1.0, float(np.abs(a).max()))
  np.testing.assert_allclose(dP, [0.0, 0.0, Mt * gravity], atol=1e-5 * scale)
  np.testing.assert_allclose(dL, 0.0, atol=1e-5 * scale)


def test_momentum_drift_first_order_zero_gravity(g1):
  """Over 1 s of semi-implicit Euler steps without gravity the momenta drift O(h): the
  largest deviation along the trajectory halves with h."""
  m0 = inv.free_floating(g1, gravity=(0.0, 0.0, 0.0))
  q, v = _random_state(m0, 5, vscale=1.5)
  drift = []
  for h in (0.005, 0.0025):
    m = copy.copy(m0)
    m.integrator, m.timestep = 0, h
    od = OracleData(m)
    _, _, P0, L0 = _momenta_at(od, q, v)
    od.qpos[:], od.qvel[:] = q, v
    dp = dl = 0.0
    for k in range(int(round(1.0 / h))):
      od.step()
      if k % int(round(0.05 / h)) == 0:
        qq, vv = od.qpos.copy(), od.qvel.copy()
        _, _, P1, L1 = _momenta_at(od, qq, vv)
        dp, dl = max(dp, np.linalg.norm(P1 - P0)), max(dl, np.linalg.norm(L1 - L0))
        od.qpos[:], od.qvel[:] = qq, vv
    drift.append((dp, dl))
    assert dp <= 2e-2 * np.linalg.norm(P0) and dl <= 5e-2 * np.linalg.norm(L0), drift
  for k in range(2):
    assert 1.7 < drift[0][k] / drift[1][k] < 2.3, drift


@pytest.mark.parametrize("mu", [0.3, 0.5])
def test_incline_stick_and_slip(mu):
  """Coulomb friction on an incline (a cube, so tan(theta) < 1 keeps it from tipping):
  below the pyramidal cone's inscribed bound (tan(theta) = 0.6 mu < mu / sqrt(2) for any
  tangent frame) it holds, up to the soft contact's steady creep (MuJoCo's friction rows are
  regularised: a small slip velocity proportional to the tangential load, mm/s here);
  above the cone (tan(theta) = 1.5 mu) it slides with a = g (sin theta - mu cos theta)."""
  m = inv.incline(np.arctan(0.6 * mu), mu)
  od = OracleData(m)
  od.qpos[:] = m.key_qpos
  for _ in range(500):  # 1 s
    od.step()
  assert abs(od.qvel[0]) < 5e-3 and abs(od.qpos[0]) < 5e-3
  th = np.arctan(1.5 * mu)
  m = inv.incline(th, mu)
  od = OracleData(m)
  od.qpos[:] = m.key_qpos
  for _ in range(100):
    od.step()
  v0, t0 = od.qvel[0], od.time
  for _ in range(400):
    od.step()
  a = (od.qvel[0] - v0) / (od.time - t0)
  assert a == pytest.approx(inv.G * (np.sin(th) - mu * np.cos(th)), rel=3e-2)
  assert abs(od.qpos[2] - 0.1) < 5e-3  # sliding on the plane, not tipping over or sinking


# (timeconst, dampratio, constant impedance d)
SOFT_CASES = [(0.02, 1.0, 0.95), (0.05, 0.3, 0.5), (0.04, 0.5, 0.7)]


def soft_start(tc, dr, d, R=0.1, margin=0.005):
  """(model, omega, r_eq, e0, steps): the oscillator's parameters and a start below the
  equilibrium that keeps the contact detected (r < 0) and pushing for the whole run."""
  m = inv.soft_sphere(tc, dr, solimp=(d, d, 0.001, 0.5, 2.0), margin=margin, R=R)
  omega = 1.0 / (tc * dr)
  r_eq = -(1.0 - d) * inv.G / omega ** 2
  e0 = -1e-3 if dr >= 1.0 else 0.4 * r_eq  # underdamped: overshoots by < |e0| < |r_eq|
  n = int(round((6.0 / omega if dr >= 1.0 else 3.0 * 2 * np.pi / omega) / m.timestep))
  return m, omega, r_eq, e0, n


@pytest.mark.parametrize("tc,dr,d", SOFT_CASES)
def test_soft_contact_is_the_documented_oscillator(tc, dr, d):
  """A frictionless sphere resting on a plane with a constant impedance d, started below its
  equilibrium with no velocity: the penetration follows the damped oscillator of natural
  frequency 1 / (tc dr) and damping ratio dr about r_eq = -(1 - d) g / omega^2 (the
  constraint's position is dist - margin)."""
  R, margin = 0.1, 0.005
  m, omega, r_eq, e0, n = soft_start(tc, dr, d, R, margin)
  od = OracleData(m)
  q = np.array(m.key_qpos, float)
  q[2] = R + margin + r_eq + e0
  od.qpos[:] = q
  od.qvel[:] = 0.0
  z = np.empty(n)
  for k in range(n):
    od.step()
    z[k] = od.qpos[2]
  t = (np.arange(n) + 1) * m.timestep
  e = z - (R + margin + r_eq)
  ref = inv.damped_oscillator(e0, omega, dr, t)
  # semi-implicit Euler at h omega <= 0.007: measured 0.16-0.30 % of e0
  assert np.abs(e - ref).max() <= 0.01 * abs(e0), (np.abs(e - ref).max(), e0)
  assert np.abs(od.qvel[[0, 1, 3, 4, 5]]).max() < 1e-9  # no lateral / rotational motion


def test_soft_contact_resting_penetration_follows_solimp():
  """With solimp's sigmoid impedance (width 2 mm) the sphere comes to rest at the depth
  where d(r)^2 K r = -(1 - d(r)) g, K = 1 / (dmax tc dr)^2 -- the documented impedance
  curve, found here by bisection."""
  solimp = (0.5, 0.95, 0.002, 0.5, 2.0)
  tc, dr, R, margin = 0.02, 1.0, 0.1, 0.0
  m = inv.soft_sphere(tc, dr, solimp=solimp, h=2e-4, margin=margin, R=R)
  K = 1.0 / (solimp[1] * tc * dr) ** 2
  f = lambda r: inv.solimp_impedance(solimp, r) ** 2 * K * r + (1 - inv.solimp_impedance(solimp, r)) * inv.G
  lo, hi = -0.05, 0.0  # f(lo) < 0 < f(hi)
  for _ in range(100):
    mid = 0.5 * (lo + hi)
    lo, hi = (mid, hi) if f(mid) < 0 else (lo, mid)
  r_eq = 0.5 * (lo + hi)
  od = OracleData(m)
  q = np.array(m.key_qpos, float)
  q[2] = R
  od.qpos[:] = q
  od.qvel[:] = 0.0
  for _ in range(5000):  # 1 s: >> the 20 ms time constant
    od.step()
  assert abs(od.qvel[2]) < 1e-6
  assert od.qpos[2] - R == pytest.approx(r_eq, rel=1e-3, abs=1e-7), (od.qpos[2] - R, r_eq)
  # the impedance matters: a constant d = dmax would rest elsewhere
  d = solimp[1]
  assert abs(r_eq - (-(1 - d) * inv.G / (d * d * K))) > 1e-5
