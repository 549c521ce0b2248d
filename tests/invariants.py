"""Physical invariants that pin the dynamics by routes that share none of the oracle's
formulas (test infrastructure; SURVEY.md section 7 build step 1).

The oracle (oracle/oracle.c) and the engine (csrc/engine_impl.h) share one formulation:
composite-rigid-body M, recursive Newton-Euler bias forces, the contact / Newton problem.  The
checks here use only the model's masses, inertias and the position-level kinematics
(body frames), and classical mechanics:

  - the small-angle period of a hinge pendulum, T = 2 pi sqrt(I_pivot / (m g L));
  - kinetic energy: 1/2 v'Mv against the sum over bodies of 1/2 m |v_com|^2 + 1/2 w'Iw
    (+ 1/2 armature v^2), with every body's twist from finite differences of its pose along
    the motion (no cvel, no CRB);
  - Lagrange's equations: qfrc_bias against d/dt(M) v - dT/dq + dU/dq by central finite
    differences of M(q) and of U(q) = -sum m_b g . x_b (no RNE);
  - conservation: energy of an unactuated contact-free system under semi-implicit Euler
    drifts O(h) (halving h halves it); linear and angular momentum about the centre of
    mass of a free-floating system without gravity;
  - Coulomb friction: a box on an incline sticks when tan(theta) < mu / sqrt(2) (the
    pyramidal cone's inscribed bound) and slides with a = g (sin theta - mu cos theta) when
    tan(theta) > mu;
  - the soft-contact model's documented behaviour (MuJoCo "Computation: soft constraints"):
    a frictionless contact with solref (timeconst, dampratio) and a constant impedance d
    makes the penetration r a damped oscillator, r'' = (1 - d) a0 + d (-B r' - K d r) with
    d^2 K = 1 / (timeconst dampratio)^2 and d B = 2 / timeconst, i.e. natural frequency
    1 / (timeconst dampratio) and damping ratio dampratio, about the equilibrium
    r_eq = (1 - d) a0 / omega^2; and with solimp's sigmoid impedance d(r) the resting
    penetration solves d(r)^2 K r = -(1 - d(r)) g.  These are closed forms of the model's
    definition (no constraint Jacobian, no solver), checked on trajectories.
"""

from __future__ import annotations

import copy

import numpy as np

from mjlab_amd.spec import Spec

G = 9.81


# ----------------------------------------------------------------------------- models
PENDULUM_XML = """
<mujoco>
  <option timestep="0.001" integrator="Euler"/>
  <worldbody>
    <body name="pendulum" pos="0 0 2">
      <joint name="hinge" type="hinge" axis="0 1 0"/>
      <geom name="rod" type="capsule" fromto="0 0 0 0 0 -{L}" size="0.01" mass="0.3"
        contype="0" conaffinity="0"/>
      <geom name="bob" type="sphere" pos="0 0 -{L}" size="0.05" mass="1.0"
        contype="0" conaffinity="0"/>
    </body>
  </worldbody>
</mujoco>
"""

# a branching hinge tree with skewed axes and offset inertias (no contacts)
TREE_XML = """
<mujoco>
  <worldbody>
    <body name="base" pos="0 0 1">
      <joint name="j0" type="hinge" axis="0 0 1"/>
      <geom type="box" size="0.1 0.05 0.04" mass="2.0" contype="0" conaffinity="0"/>
      <body name="a1" pos="0.15 0 0">
        <joint name="j1" type="hinge" axis="0 1 0"/>
        <geom type="capsule" fromto="0 0 0 0.3 0 0.05" size="0.03" mass="1.2" contype="0" conaffinity="0"/>
        <body name="a2" pos="0.3 0 0.05" quat="0.9238795 0 0.3826834 0">
          <joint name="j2" type="hinge" axis="1 0.4 0.2" armature="0.01"/>
          <geom type="box" size="0.12 0.03 0.02" pos="0.1 0.02 0" mass="0.7" contype="0" conaffinity="0"/>
          <body name="a3" pos="0.22 0 0">
            <joint name="j3" type="hinge" axis="0 0.6 0.8"/>
            <geom type="sphere" size="0.05" pos="0.05 0.03 -0.02" mass="0.4" contype="0" conaffinity="0"/>
          </body>
        </body>
      </body>
      <body name="b1" pos="-0.15 0 0">
        <joint name="k1" type="hinge" axis="1 0 0"/>
        <geom type="capsule" fromto="0 0 0 -0.2 0.1 -0.1" size="0.025" mass="0.9" contype="0" conaffinity="0"/>
        <body name="b2" pos="-0.2 0.1 -0.1">
          <joint name="k2" type="hinge" axis="0.3 -0.5 0.8"/>
          <geom type="cylinder" size="0.03 0.08" pos="0 0 -0.08" mass="0.5" contype="0" conaffinity="0"/>
        </body>
      </body>
    </body>
  </worldbody>
</mujoco>
"""

INCLINE_XML = """
<mujoco>
  <option timestep="0.002"/>
  <worldbody>
    <geom name="floor" type="plane" size="5 5 0.1" friction="{mu} 0.005 0.0001"/>
    <body name="box" pos="0 0 0.1">
      <freejoint name="box_joint"/>
      <geom name="box_geom" type="box" size="0.1 0.1 0.1" mass="1.0" friction="{mu} 0.005 0.0001"/>
    </body>
  </worldbody>
</mujoco>
"""


# a frictionless sphere on a plane, both geoms with one solref / solimp / margin
SPHERE_XML = """
<mujoco>
  <option timestep="{h}" integrator="Euler"/>
  <worldbody>
    <geom name="floor" type="plane" size="5 5 0.1" condim="1" solref="{tc} {dr}"
      solimp="{solimp}" margin="{margin}"/>
    <body name="ball" pos="0 0 1">
      <freejoint name="ball_joint"/>
      <geom name="ball_geom" type="sphere" size="{R}" mass="{mass}" condim="1"
        solref="{tc} {dr}" solimp="{solimp}" margin="{margin}"/>
    </body>
  </worldbody>
</mujoco>
"""


def soft_sphere(tc: float, dr: float, solimp=(0.95, 0.95, 0.001, 0.5, 2.0), h: float = 1e-4,
                margin: float = 0.005, R: float = 0.1, mass: float = 2.0):
  spec = Spec.from_string(SPHERE_XML.format(h=h, tc=tc, dr=dr, solimp=" ".join(str(v) for v in solimp),
                                            margin=margin, R=R, mass=mass))
  spec.option.update(timestep=h, integrator="euler")
  return spec.compile()


def solimp_impedance(solimp, r: float) -> float:
  """MuJoCo's documented impedance d(r): x = |r| / width clipped to [0, 1], the sigmoid
  y(x) = x^p / mid^(p-1) below the midpoint and 1 - (1-x)^p / (1-mid)^(p-1) above it,
  d = dmin + y (dmax - dmin)."""
  dmin, dmax, width, mid, p = solimp
  x = min(1.0, abs(r) / width)
  if x <= mid:
    y = x ** p / mid ** (p - 1)
  else:
    y = 1.0 - (1.0 - x) ** p / (1.0 - mid) ** (p - 1)
  return dmin + y * (dmax - dmin)


def damped_oscillator(e0: float, omega: float, zeta: float, t: np.ndarray) -> np.ndarray:
  """e(t) of e'' + 2 zeta omega e' + omega^2 e = 0 from e(0) = e0, e'(0) = 0."""
  if zeta >= 1.0:
    return e0 * (1.0 + omega * t) * np.exp(-omega * t)
  wd = omega * np.sqrt(1.0 - zeta * zeta)
  return e0 * np.exp(-zeta * omega * t) * (np.cos(wd * t) + zeta * omega / wd * np.sin(wd * t))


def pendulum(L: float = 0.5):
  spec = Spec.from_string(PENDULUM_XML.format(L=L))
  spec.option.update(timestep=0.001, integrator="euler")
  return spec.compile()


def hinge_tree(gravity=(0.0, 0.0, -G)):
  spec = Spec.from_string(TREE_XML)
  spec.option.update(gravity=tuple(gravity))
  return spec.compile()


def incline(theta: float, mu: float):
  """Box on a plane under gravity tilted by theta about y (the incline's frame)."""
  spec = Spec.from_string(INCLINE_XML.format(mu=mu))
  spec.option.update(timestep=0.002, gravity=(G * np.sin(theta), 0.0, -G * np.cos(theta)))
  return spec.compile()


def free_floating(model, gravity=None):
  """An unactuated, limit-free, contact-free copy of a robot model (no collision pairs, no
  joint limits, no actuator gains), optionally with another gravity."""
  m = copy.deepcopy(model)
  m.arrays["actuator_gainprm"] = np.zeros_like(m.arrays["actuator_gainprm"])
  m.arrays["actuator_biasprm"] = np.zeros_like(m.arrays["actuator_biasprm"])
  m.arrays["jnt_limited"] = np.zeros_like(m.arrays["jnt_limited"])
  m.arrays["pair_geom1"] = np.zeros(0, np.int32)
  m.arrays["pair_geom2"] = np.zeros(0, np.int32)
  m.npair = 0
  if gravity is not None:
    m.gravity = np.asarray(gravity, float)
  return m


# ----------------------------------------------------------------------------- kinematics
def quat_mul(a, b):
  w1, x1, y1, z1 = a
  w2, x2, y2, z2 = b
  return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                   w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


def integrate_pos(m, qpos, qvel, dt):
  """qpos advanced by qvel over dt along MuJoCo's joint conventions (free joint: world
  linear velocity, body-frame angular velocity; hinge / slide: q += v dt)."""
  q = np.array(qpos, float)
  for j in range(m.njnt):
    a, d, t = int(m.jnt_qposadr[j]), int(m.jnt_dofadr[j]), int(m.jnt_type[j])
    if t == 0:
      q[a:a + 3] += dt * qvel[d:d + 3]
      w = np.asarray(qvel[d + 3:d + 6], float) * dt
      th = np.linalg.norm(w)
      dq = np.array([np.cos(th / 2), *(w / th * np.sin(th / 2))]) if th > 0 else np.array([1.0, 0, 0, 0])
      qq = quat_mul(q[a + 3:a + 7], dq)
      q[a + 3:a + 7] = qq / np.linalg.norm(qq)
    else:
      q[a] += dt * qvel[d]
  return q


def body_pose(od, qpos):
  """(xipos [nb, 3], ximat [nb, 3, 3]) at qpos: the oracle's position stage only."""
  od.qpos[:] = qpos
  od.qvel[:] = 0.0
  od.forward()
  return od.xipos.copy(), od.ximat.reshape(-1, 3, 3).copy()


def fd_twists(od, qpos, qvel, eps=1e-6):
  """Every body's com velocity and world angular velocity by central differences of its
  pose along the motion (q(t +- eps))."""
  m = od.model
  xp, Rp = body_pose(od, integrate_pos(m, qpos, qvel, eps))
  xm, Rm = body_pose(od, integrate_pos(m, qpos, qvel, -eps))
  v = (xp - xm) / (2 * eps)
  w = np.zeros_like(v)
  for b in range(m.nbody):
    # R(t+e) R(t-e)^T = exp(2 e [w]x): the skew part over 4 e
    S = Rp[b] @ Rm[b].T
    w[b] = np.array([S[2, 1] - S[1, 2], S[0, 2] - S[2, 0], S[1, 0] - S[0, 1]]) / (4 * eps)
  return v, w


def kinetic_energy_bodies(m, ximat, v, w, qvel):
  """sum_b 1/2 m_b |v_b|^2 + 1/2 w_b' (R I_b R') w_b, plus the armature (rotor) term."""
  ke = 0.0
  for b in range(1, m.nbody):
    R = ximat[b]
    I = R @ np.diag(m.body_inertia[b]) @ R.T
    ke += 0.5 * m.body_mass[b] * v[b] @ v[b] + 0.5 * w[b] @ I @ w[b]
  return ke + 0.5 * float(np.sum(np.asarray(m.dof_armature) * np.asarray(qvel) ** 2))


def mass_matrix(od, qpos):
  od.qpos[:] = qpos
  od.qvel[:] = 0.0
  od.forward()
  return od.qM.copy()


def potential(m, xipos):
  return -float(np.sum(np.asarray(m.body_mass)[:, None] * np.asarray(m.gravity)[None, :] * xipos))


def lagrange_bias(od, qpos, qvel, rows, eps=1e-6):
  """d/dt(M) v - dT/dq_i + dU/dq_i for the dofs `rows` whose coordinate is a true
  generalized coordinate (translational free-joint dofs, hinges, slides): central
  differences of M(q) along the motion and along each coordinate, and of U(q)."""
  m = od.model
  Mp = mass_matrix(od, integrate_pos(m, qpos, qvel, eps))
  Mm = mass_matrix(od, integrate_pos(m, qpos, qvel, -eps))
  Mdot_v = (Mp - Mm) @ qvel / (2 * eps)
  out = {}
  for i in rows:
    e = np.zeros(m.nv)
    e[i] = 1.0
    qp, qm = integrate_pos(m, qpos, e, eps), integrate_pos(m, qpos, e, -eps)
    dM = (mass_matrix(od, qp) - mass_matrix(od, qm)) / (2 * eps)
    xp, _ = body_pose(od, qp)
    xm, _ = body_pose(od, qm)
    dU = (potential(m, xp) - potential(m, xm)) / (2 * eps)
    out[i] = Mdot_v[i] - 0.5 * qvel @ dM @ qvel + dU
  return out


def momenta(m, xipos, ximat, v, w):
  """(total mass, com, linear momentum, angular momentum about the com)."""
  mass = np.asarray(m.body_mass)[1:]
  M = float(mass.sum())
  c = (mass[:, None] * xipos[1:]).sum(0) / M
  P = (mass[:, None] * v[1:]).sum(0)
  L = np.zeros(3)
  for b in range(1, m.nbody):
    R = ximat[b]
    I = R @ np.diag(m.body_inertia[b]) @ R.T
    L += I @ w[b] + m.body_mass[b] * np.cross(xipos[b] - c, v[b])
  return M, c, P, L


def twists_from_cvel(m, xipos, subtree_com, cvel):
  """Body com velocity / angular velocity from MuJoCo's com-based cvel ([w; v] of the point
  at the root's subtree com, `entity/data.py:20-31`)."""
  root = np.asarray(m.body_rootid)
  w = cvel[:, 0:3]
  v = cvel[:, 3:6] + np.cross(w, xipos - subtree_com[root])
  return v, w


def pendulum_period(m) -> float:
  """Small-angle period of the compiled pendulum from its inertia alone."""
  b = 1
  L = float(np.linalg.norm(m.body_ipos[b]))  # com distance from the hinge (at the body origin)
  ax = np.asarray(m.jnt_axis[0], float)
  from mjlab_amd.compiler.mjcf import quat_to_mat
  R = quat_to_mat(m.body_iquat[b])
  I_cm = float(ax @ (R @ np.diag(m.body_inertia[b]) @ R.T) @ ax)
  I = I_cm + float(m.body_mass[b]) * L * L + float(m.dof_armature[0])
  return 2 * np.pi * np.sqrt(I / (float(m.body_mass[b]) * G * L))


def zero_crossing_period(t, theta) -> float:
  """Mean period from the upward zero crossings (linear interpolation)."""
  t, theta = np.asarray(t), np.asarray(theta)
  idx = np.nonzero((theta[:-1] < 0) & (theta[1:] >= 0))[0]
  tc = t[idx] - theta[idx] * (t[idx + 1] - t[idx]) / (theta[idx + 1] - theta[idx])
  assert tc.size >= 3, "fewer than three crossings"
  return float(np.mean(np.diff(tc)))
