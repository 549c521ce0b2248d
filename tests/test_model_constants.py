"""Compiled-scene checks pinned to the reference's robot constants and its own constant tests.

Expected values are restated from the reference sources (read as text):
  asset_zoo/robots/unitree_g1/g1_constants.py:100-187 (actuator groups, NATURAL_FREQ =
  10*2*3.1415926535, DAMPING_RATIO 2, effort limits), :207-220 (KNEES_BENT_KEYFRAME),
  :229-234 (FULL_COLLISION), :287-295 (G1_ACTION_SCALE = 0.25*effort/stiffness);
  asset_zoo/robots/unitree_go1/go1_constants.py:37-133;
  tests/test_g1_constants.py:37-141 (the properties asserted there);
  SURVEY.md section 8(a) a6/a15 for the derived kp/kd/scale numbers and scene dimensions.
"""

import math
import re

import numpy as np
import pytest

from mjlab_amd.scenes import load_scene

OMEGA = 10 * 2.0 * 3.1415926535  # NATURAL_FREQ as written in the reference (truncated pi)

# (joint regexes, kp, kd, effort): g1_constants.py:134-187, values per SURVEY a6
G1_GROUPS = [
  ((".*_elbow_joint", ".*_shoulder_pitch_joint", ".*_shoulder_roll_joint",
    ".*_shoulder_yaw_joint", ".*_wrist_roll_joint"), 14.2506, 0.90722, 25.0),
  ((".*_hip_pitch_joint", ".*_hip_yaw_joint", "waist_yaw_joint"), 40.1792, 2.55789, 88.0),
  ((".*_hip_roll_joint", ".*_knee_joint"), 99.0984, 6.30880, 139.0),
  ((".*_wrist_pitch_joint", ".*_wrist_yaw_joint"), 16.7783, 1.06814, 5.0),
  (("waist_pitch_joint", "waist_roll_joint"), 2 * 14.2506, 2 * 0.90722, 50.0),
  ((".*_ankle_pitch_joint", ".*_ankle_roll_joint"), 2 * 14.2506, 2 * 0.90722, 50.0),
]
GO1_ROTOR = 0.000111842  # go1_constants.py:43
GO1_GROUPS = [
  ((".*_hip_joint", ".*_thigh_joint"), GO1_ROTOR * 6 ** 2, 23.7),
  ((".*_calf_joint",), GO1_ROTOR * 9 ** 2, 35.55),
]


@pytest.fixture(scope="module")
def g1():
  return load_scene("g1_velocity")


@pytest.fixture(scope="module")
def go1():
  return load_scene("go1_velocity")


def _short(n):
  return n.split("/", 1)[1] if "/" in n else n  # entity prefix "robot/"


def _actuator_joint_names(m):
  jn = m.names["joint"]
  return [_short(jn[j]) for j in m.actuator_trnid]


def _group_of(name, groups):
  hits = [g for g in groups if any(re.fullmatch(p, name) for p in g[0])]
  assert len(hits) == 1, (name, hits)
  return hits[0]


def test_g1_dimensions(g1):
  """nq 36, nv 35, nu 29, nbody 32, ngeom 69, ~502 pairs, nsensordata 21."""
  assert (g1.nq, g1.nv, g1.nu, g1.nbody, g1.njnt) == (36, 35, 29, 32, 30)
  assert g1.ngeom == 69
  assert g1.npair == 502
  assert g1.nsensordata == 21


def test_go1_dimensions(go1):
  assert (go1.nq, go1.nv, go1.nu, go1.nbody) == (19, 18, 12, 15)
  assert go1.ngeom == 44
  assert go1.npair == 30
  assert go1.nsensordata == 54


def test_g1_actuator_parameters(g1):
  """test_g1_constants.py:37-50 + :128-141: gain/bias/forcerange per actuator group,
  ctrllimited False and forcelimited True everywhere."""
  names = _actuator_joint_names(g1)
  assert len(names) == 29
  for u, name in enumerate(names):
    _, kp, kd, effort = _group_of(name, G1_GROUPS)
    assert g1.actuator_gainprm[u][0] == pytest.approx(kp, rel=2e-5)
    assert g1.actuator_biasprm[u][1] == pytest.approx(-kp, rel=2e-5)
    assert g1.actuator_biasprm[u][2] == pytest.approx(-kd, rel=2e-5)
    assert tuple(g1.actuator_forcerange[u]) == pytest.approx((-effort, effort))
    assert g1.actuator_ctrllimited[u] == 0
    assert g1.actuator_forcelimited[u] == 1


def test_g1_armature_is_reflected_inertia(g1):
  """armature = kp / omega^2 per group (STIFFNESS = ARMATURE * NATURAL_FREQ**2)."""
  names = _actuator_joint_names(g1)
  for u, name in enumerate(names):
    _, kp, _, _ = _group_of(name, G1_GROUPS)
    dof = g1.jnt_dofadr[g1.actuator_trnid[u]]
    assert g1.dof_armature[dof] == pytest.approx(kp / OMEGA ** 2, rel=2e-5)


def test_go1_actuator_parameters(go1):
  """go1_constants.py:49-81: kp = I w^2, kd = 2*zeta*I*w with I = rotor * gear^2."""
  for u, name in enumerate(_actuator_joint_names(go1)):
    _, inertia, effort = _group_of(name, [(g[0], g[1], g[2]) for g in GO1_GROUPS])
    kp, kd = inertia * OMEGA ** 2, 2 * 2.0 * inertia * OMEGA
    assert go1.actuator_gainprm[u][0] == pytest.approx(kp, rel=1e-6)
    assert go1.actuator_biasprm[u][1] == pytest.approx(-kp, rel=1e-6)
    assert go1.actuator_biasprm[u][2] == pytest.approx(-kd, rel=1e-6)
    assert tuple(go1.actuator_forcerange[u]) == pytest.approx((-effort, effort))
  # SURVEY a6 numbers
  assert GO1_GROUPS[0][1] * OMEGA ** 2 == pytest.approx(15.8952, rel=1e-5)
  assert GO1_GROUPS[1][1] * OMEGA ** 2 == pytest.approx(35.7643, rel=1e-5)


def test_action_scales():
  """G1_ACTION_SCALE / GO1_ACTION_SCALE = 0.25 * effort / stiffness (SURVEY a15 values)."""
  from mjlab_amd.asset_zoo import action_scale, g1_actuators, go1_actuators
  s = action_scale(g1_actuators())
  expect = {".*_elbow_joint": 0.438577, ".*_hip_pitch_joint": 0.547546,
            ".*_knee_joint": 0.350661, ".*_wrist_yaw_joint": 0.0745009,
            "waist_roll_joint": 0.438577, ".*_ankle_pitch_joint": 0.438577}
  for k, v in expect.items():
    assert s[k] == pytest.approx(v, rel=2e-5), k
  s = action_scale(go1_actuators())
  assert s[".*_hip_joint"] == pytest.approx(0.372753, rel=2e-5)
  assert s[".*_calf_joint"] == pytest.approx(0.248502, rel=2e-5)


def test_g1_keyframe(g1):
  """KNEES_BENT_KEYFRAME (g1_constants.py:207-220), test_g1_constants.py:52-78."""
  q = np.asarray(g1.key_qpos)
  np.testing.assert_array_equal(q[:3], [0, 0, 0.76])
  np.testing.assert_array_equal(q[3:7], [1, 0, 0, 0])
  expect = {".*_hip_pitch_joint": -0.312, ".*_knee_joint": 0.669, ".*_ankle_pitch_joint": -0.363,
            ".*_elbow_joint": 0.6, "left_shoulder_roll_joint": 0.2,
            "left_shoulder_pitch_joint": 0.2, "right_shoulder_roll_joint": -0.2,
            "right_shoulder_pitch_joint": 0.2}
  for j, name in enumerate(g1.names["joint"]):
    name = _short(name)
    if g1.jnt_type[j] == 0:  # free joint
      continue
    want = 0.0
    for pat, v in expect.items():
      if re.match(pat, name):  # resolve_expr: first match wins
        want = v
        break
    assert q[g1.jnt_qposadr[j]] == pytest.approx(want, rel=1e-5), name


def test_go1_keyframe(go1):
  q = np.asarray(go1.key_qpos)
  np.testing.assert_allclose(q[:3], [0, 0, 0.278])
  expect = {".*thigh_joint": 0.9, ".*calf_joint": -1.8, ".*R_hip_joint": 0.1, ".*L_hip_joint": -0.1}
  for j, name in enumerate(go1.names["joint"]):
    name = _short(name)
    if go1.jnt_type[j] == 0:
      continue
    want = [v for p, v in expect.items() if re.match(p, name)]
    assert q[go1.jnt_qposadr[j]] == pytest.approx(want[0] if want else 0.0), name


FOOT = r"^(left|right)_foot[1-7]_collision$"


def test_g1_foot_collision_geoms(g1):
  """test_g1_constants.py:81-118: 14 foot capsules, condim 3, priority 1, friction 0.6;
  other *_collision geoms condim 1."""
  names = [_short(n) for n in g1.names["geom"]]
  feet = [i for i, n in enumerate(names) if re.match(FOOT, n)]
  assert len(feet) == 14
  for i in feet:
    assert g1.geom_condim[i] == 3
    assert g1.geom_priority[i] == 1
    assert g1.geom_friction[i][0] == pytest.approx(0.6)
  for i, n in enumerate(names):
    if "_collision" in n and not re.match(FOOT, n):
      assert g1.geom_condim[i] == 1, n


def test_go1_foot_solimp(go1):
  """go1_constants.py:117-127: feet condim 3, priority 1, friction 0.6, solimp (.9,.95,.023)."""
  names = [_short(n) for n in go1.names["geom"]]
  feet = [i for i, n in enumerate(names) if re.match(r"^[FR][LR]_foot_collision$", n)]
  assert len(feet) == 4
  for i in feet:
    assert _foot_ok(go1, i)


def _foot_ok(m, i):
  return (m.geom_condim[i] == 3 and m.geom_priority[i] == 1
          and m.geom_friction[i][0] == pytest.approx(0.6)
          and tuple(m.geom_solimp[i][:3]) == pytest.approx((0.9, 0.95, 0.023)))


def test_sensor_layout(g1):
  """G1 sensordata = gyro 3 + velocimeter 3 + accelerometer 3 + subtreeangmom 3 +
  feet (found 1 + force 3) x 2 + self_collision found 1 = 21."""
  dims = sorted(int(d) for d in g1.sensor_dim)
  assert sum(dims) == 21
  assert dims.count(3) == 6 and dims.count(1) == 3


def test_constant_fields(g1):
  """_set_const: subtree mass at the root equals total mass; invweights positive."""
  total = float(np.sum(g1.body_mass))
  assert g1.body_subtreemass[0] == pytest.approx(total)
  assert np.all(np.asarray(g1.dof_invweight0) > 0)
  assert math.isfinite(float(g1.meaninertia)) and g1.meaninertia > 0
