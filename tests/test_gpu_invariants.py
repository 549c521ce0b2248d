"""The engine checked once against the classical-mechanics invariants that pin the oracle
(tests/invariants.py, tests/test_oracle_invariants.py).  fp32 engine,
so the tolerances are fp32-scaled; each quantity the engine does not expose (M) comes from
the oracle, which the CPU tests pin independently."""

import numpy as np
import pytest
import torch

import invariants as inv
from mjlab_amd.scenes import load_scene
from oracle_sim import OracleData

pytestmark = pytest.mark.gpu


def _sim(m, n, device):
  from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
  cfg = MujocoCfg(timestep=float(m.timestep), integrator="euler" if m.integrator == 0 else "implicitfast",
                  gravity=tuple(float(g) for g in m.gravity), iterations=int(m.iterations),
                  ls_iterations=int(m.ls_iterations), tolerance=float(m.tolerance))
  return Simulation(n, SimulationCfg(nconmax=48, njmax=160, mujoco=cfg), m, device)


def _set(sim, q, v):
  sim.data.qpos[:] = torch.as_tensor(np.atleast_2d(q), dtype=torch.float32)
  sim.data.qvel[:] = torch.as_tensor(np.atleast_2d(v), dtype=torch.float32)
  sim.data.qacc_warmstart.zero_()
  sim.data.ctrl.zero_()


def _np(t):
  return t.double().cpu().numpy()


@pytest.fixture(scope="module")
def g1():
  return load_scene("g1_velocity")


def _state(m, seed, vscale=1.0):
  rng = np.random.default_rng(seed)
  q = np.array(m.key_qpos, float)
  q[2] = 50.0
  q[7:] += rng.uniform(-0.3, 0.3, m.nq - 7)
  q[3:7] = inv.integrate_pos(m, q, np.r_[np.zeros(3), rng.normal(0, 0.3, 3), np.zeros(m.nv - 6)], 1.0)[3:7]
  return q, rng.normal(0, vscale, m.nv)


def test_gpu_pendulum_period(gpu_device):
  m = inv.pendulum(L=0.5)
  T = inv.pendulum_period(m)
  amps = np.array([0.01, 0.02, 0.03, -0.02])
  sim = _sim(m, len(amps), gpu_device)
  _set(sim, amps[:, None], np.zeros((len(amps), 1)))
  nstep = int(4 * T / m.timestep)
  trace = torch.zeros(nstep, len(amps), device=sim.data.qpos.device)
  for k in range(nstep):
    sim.step()
    trace[k] = sim.data.qpos[:, 0]
  th = _np(trace)
  t = (np.arange(nstep) + 1) * m.timestep
  for w, a in enumerate(amps):
    sgn = np.sign(a)
    assert inv.zero_crossing_period(t, sgn * th[:, w]) == pytest.approx(T, rel=5e-4), f"world {w}"
    assert np.abs(th[:, w]).max() == pytest.approx(abs(a), rel=1e-2)


def test_gpu_twists_kinetic_energy_and_bias(g1, gpu_device):
  """The engine's cvel (body twists) against finite-difference twists, its kinetic energy
  against 1/2 v'Mv, and its qfrc_bias against Lagrange's equations, on free-floating G1
  states."""
  m = inv.free_floating(g1)
  od = OracleData(m)
  n = 3
  states = [_state(m, s) for s in range(n)]
  sim = _sim(m, n, gpu_device)
  _set(sim, np.array([s[0] for s in states]), np.array([s[1] for s in states]))
  sim.forward()
  torch.cuda.synchronize()
  d = sim.data
  xipos, ximat, stc, cvel = (_np(getattr(d, f)) for f in ("xipos", "ximat", "subtree_com", "cvel"))
  bias = _np(d.qfrc_bias)
  for w, (q, v) in enumerate(states):
    q32 = _np(d.qpos[w])
    v32 = _np(d.qvel[w])
    vb, wb = inv.fd_twists(od, q32, v32)
    vg, wg = inv.twists_from_cvel(m, xipos[w], stc[w], cvel[w])
    scale = max(1.0, float(np.abs(vb).max()), float(np.abs(wb).max()))
    np.testing.assert_allclose(vg[1:], vb[1:], atol=2e-5 * scale)
    np.testing.assert_allclose(wg[1:], wb[1:], atol=2e-5 * scale)
    ke = inv.kinetic_energy_bodies(m, ximat[w].reshape(-1, 3, 3), vg, wg, v32)
    M = inv.mass_matrix(od, q32)
    assert ke == pytest.approx(0.5 * v32 @ M @ v32, rel=1e-4)
    rows = [0, 1, 2] + list(range(6, m.nv))
    lag = inv.lagrange_bias(od, q32, v32, rows)
    bscale = max(1.0, max(abs(x) for x in lag.values()))
    for i in rows:
      assert abs(bias[w][i] - lag[i]) <= 1e-4 * bscale, f"world {w} dof {i}: {bias[w][i]} vs {lag[i]}"


@pytest.mark.parametrize("gravity", [0.0, -inv.G])
def test_gpu_momentum_rate(g1, gravity, gpu_device):
  """The engine's forward dynamics: dP/dt = M_total g and dL/dt = 0 about the com."""
  m = inv.free_floating(g1, gravity=(0.0, 0.0, gravity))
  od = OracleData(m)
  q, v = _state(m, 5, vscale=1.5)
  sim = _sim(m, 1, gpu_device)
  _set(sim, q, v)
  sim.forward()
  torch.cuda.synchronize()
  q, v, a = _np(sim.data.qpos[0]), _np(sim.data.qvel[0]), _np(sim.data.qacc[0])

  def mom(qq, vv):
    od.qpos[:], od.qvel[:] = qq, vv
    od.forward()
    vb, wb = inv.twists_from_cvel(m, od.xipos, od.subtree_com, od.cvel)
    return inv.momenta(m, od.xipos, od.ximat.reshape(-1, 3, 3), vb, wb)

  e = 1e-4
  Mt, _, Pp, Lp = mom(inv.integrate_pos(m, q, e * v + 0.5 * e * e * a, 1.0), v + e * a)
  _, _, Pm, Lm = mom(inv.integrate_pos(m, q, -e * v + 0.5 * e * e * a, 1.0), v - e * a)
  scale = Mt * max(1.0, float(np.abs(a).max()))
  np.testing.assert_allclose((Pp - Pm) / (2 * e), [0.0, 0.0, Mt * gravity], atol=1e-4 * scale)
  np.testing.assert_allclose((Lp - Lm) / (2 * e), 0.0, atol=1e-4 * scale)


def test_gpu_energy_drift_first_order(g1, gpu_device):
  """Zero gravity, unactuated, contact-free G1: the engine's semi-implicit Euler keeps the
  energy to O(h) over 1 s (halving h halves the largest deviation)."""
  m0 = inv.free_floating(g1, gravity=(0.0, 0.0, 0.0))
  q, v = _state(m0, 11)
  od = OracleData(m0)
  drift = []
  for h in (0.005, 0.0025):
    m = inv.free_floating(g1, gravity=(0.0, 0.0, 0.0))
    m.integrator, m.timestep = 0, h
    sim = _sim(m, 1, gpu_device)
    _set(sim, q, v)
    q32, v32 = _np(sim.data.qpos[0]), _np(sim.data.qvel[0])
    nstep = int(round(1.0 / h))
    every = int(round(0.05 / h))
    qs, vs = [], []
    for k in range(nstep):
      sim.step()
      if k % every == every - 1:
        qs.append(sim.data.qpos[0].clone())
        vs.append(sim.data.qvel[0].clone())
    torch.cuda.synchronize()

    def energy(qq, vv):
      return 0.5 * vv @ inv.mass_matrix(od, qq) @ vv

    E0 = energy(q32, v32)
    worst = max(abs(energy(_np(a), _np(b)) - E0) for a, b in zip(qs, vs))
    drift.append(worst)
    assert worst < 0.02 * E0, (h, worst, E0)
  assert 1.7 < drift[0] / drift[1] < 2.3, drift


@pytest.mark.parametrize("mu", [0.3, 0.5])
def test_gpu_incline_stick_and_slip(mu, gpu_device):
  for ratio, slides in ((0.6, False), (1.5, True)):
    th = np.arctan(ratio * mu)
    m = inv.incline(th, mu)
    sim = _sim(m, 2, gpu_device)
    _set(sim, np.tile(m.key_qpos, (2, 1)), np.zeros((2, m.nv)))
    for _ in range(100):
      sim.step()
    torch.cuda.synchronize()
    v0 = _np(sim.data.qvel[:, 0])
    for _ in range(400):
      sim.step()
    torch.cuda.synchronize()
    v1, x, z = _np(sim.data.qvel[:, 0]), _np(sim.data.qpos[:, 0]), _np(sim.data.qpos[:, 2])
    if slides:
      a = (v1 - v0) / (400 * m.timestep)
      np.testing.assert_allclose(a, inv.G * (np.sin(th) - mu * np.cos(th)), rtol=3e-2)
      assert np.all(np.abs(z - 0.1) < 5e-3)
    else:
      assert np.all(np.abs(v1) < 5e-3) and np.all(np.abs(x) < 5e-3)


@pytest.mark.parametrize("case", range(3))
def test_gpu_soft_contact_is_the_documented_oscillator(case, gpu_device):
  """The engine's soft contact against the damped oscillator its solref defines
  (tests/test_oracle_invariants.py::test_soft_contact_is_the_documented_oscillator)."""
  from test_oracle_invariants import SOFT_CASES, soft_start
  tc, dr, d = SOFT_CASES[case]
  R, margin = 0.1, 0.005
  m, omega, r_eq, e0, n = soft_start(tc, dr, d, R, margin)
  sim = _sim(m, 1, gpu_device)
  q = np.array(m.key_qpos, float)
  q[2] = R + margin + r_eq + e0
  _set(sim, q, np.zeros(m.nv))
  z = torch.zeros(n, device=sim.data.qpos.device, dtype=torch.float64)
  for k in range(n):
    sim.step()
    z[k] = sim.data.qpos[0, 2]
  t = (np.arange(n) + 1) * m.timestep
  e = z.cpu().numpy() - (R + margin + r_eq)
  ref = inv.damped_oscillator(e0, omega, dr, t)
  # fp32 positions near 0.1 m: ulp 7e-9 m, a few percent of |e0| >= 4.4e-4 m at most
  assert np.abs(e - ref).max() <= 0.02 * abs(e0), (np.abs(e - ref).max(), e0)


def test_gpu_soft_contact_resting_penetration_follows_solimp(gpu_device):
  solimp = (0.5, 0.95, 0.002, 0.5, 2.0)
  tc, dr, R = 0.02, 1.0, 0.1
  m = inv.soft_sphere(tc, dr, solimp=solimp, h=2e-4, margin=0.0, R=R)
  K = 1.0 / (solimp[1] * tc * dr) ** 2
  f = lambda r: inv.solimp_impedance(solimp, r) ** 2 * K * r + (1 - inv.solimp_impedance(solimp, r)) * inv.G
  lo, hi = -0.05, 0.0
  for _ in range(100):
    mid = 0.5 * (lo + hi)
    lo, hi = (mid, hi) if f(mid) < 0 else (lo, mid)
  r_eq = 0.5 * (lo + hi)
  sim = _sim(m, 1, gpu_device)
  q = np.array(m.key_qpos, float)
  q[2] = R
  _set(sim, q, np.zeros(m.nv))
  for _ in range(5000):
    sim.step()
  torch.cuda.synchronize()
  zr = float(sim.data.qpos[0, 2]) - R
  assert zr == pytest.approx(r_eq, rel=2e-3, abs=2e-7), (zr, r_eq)
