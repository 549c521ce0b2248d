"""Capsule-capsule narrowphase of the oracle (MuJoCo's mjc_CapsuleCapsule,
engine_collision_primitive.c, restated in oracle.c col_capsule_capsule and in the engine's
capsule_capsule): crossed capsules give one contact at the closest points; parallel
capsules give up to two, from the segment ends; non-parallel closest points agree with a
brute-force minimisation of the segment distance."""

import numpy as np
import pytest

import oracle_lib as ol
from mjlab_amd.compiler.mjcf import parse_mjcf_string
from mjlab_amd.compiler.model import EntitySpec, compile_scene

R, H = 0.05, 0.2  # radius, half length

_TWO = f"""<mujoco><worldbody>
  <body name="a" pos="0 0 0"><freejoint/>
    <inertial pos="0 0 0" mass="1" diaginertia="0.01 0.01 0.01"/>
    <geom name="ca" type="capsule" size="{R} {H}"/></body>
  <body name="b" pos="0 0 1"><freejoint/>
    <inertial pos="0 0 0" mass="1" diaginertia="0.01 0.01 0.01"/>
    <geom name="cb" type="capsule" size="{R} {H}"/></body>
</worldbody></mujoco>"""


def two_capsules():
  ent = EntitySpec("pair", parse_mjcf_string(_TWO))
  return compile_scene([ent], terrain="none", timestep=0.005)


def quat_axis(axis):
  """Unit quaternion turning local z onto `axis`."""
  a = np.asarray(axis, float) / np.linalg.norm(axis)
  z = np.array([0.0, 0.0, 1.0])
  c = float(z @ a)
  if c < -1 + 1e-12:
    return np.array([0.0, 1.0, 0.0, 0.0])
  v = np.cross(z, a)
  q = np.array([1.0 + c, *v])
  return q / np.linalg.norm(q)


def state(pa, axa, pb, axb):
  q = np.zeros(14)
  q[0:3], q[3:7] = pa, quat_axis(axa)
  q[7:10], q[10:14] = pb, quat_axis(axb)
  return q


@pytest.fixture(scope="module")
def model():
  return two_capsules()


def test_scene_has_the_pair(model):
  assert model.npair == 1


def test_crossed_capsules_one_contact(model):
  q = state((0, 0, 0), (1, 0, 0), (0.05, 0.02, 0.09), (0, 1, 0))
  f = ol.forward(model, q)
  assert f["ncon"] == 1
  c = f["contact"][0]
  assert c[2] == pytest.approx(0.09 - 2 * R, abs=1e-12)
  np.testing.assert_allclose(c[3:6], [0.05, 0.0, R - 0.005], atol=1e-12)
  np.testing.assert_allclose(c[6:9], [0, 0, 1], atol=1e-12)


def test_parallel_capsules_two_contacts_from_the_ends(model):
  # cap a on x in [-0.2, 0.2], cap b on x in [-0.1, 0.3], 0.09 above: a's +x end and b's -x
  # end are over the other segment (depth -0.01); a's -x end and b's +x end are not
  q = state((0, 0, 0), (1, 0, 0), (0.1, 0, 0.09), (1, 0, 0))
  f = ol.forward(model, q)
  assert f["ncon"] == 2
  c = f["contact"]
  np.testing.assert_allclose(c[:, 2], [-0.01, -0.01], atol=1e-12)
  np.testing.assert_allclose(c[:, 3], [0.2, -0.1], atol=1e-12)
  np.testing.assert_allclose(c[:, 5], [R - 0.005] * 2, atol=1e-12)
  np.testing.assert_allclose(c[:, 6:9], [[0, 0, 1]] * 2, atol=1e-12)
  # anti-parallel axes are parallel too: each of a's ends is over one of b's ends
  q = state((0, 0, 0), (1, 0, 0), (0.0, 0, 0.095), (-1, 0, 0))
  f = ol.forward(model, q)
  assert f["ncon"] == 2
  np.testing.assert_allclose(np.sort(f["contact"][:, 3]), [-0.2, 0.2], atol=1e-12)
  np.testing.assert_allclose(f["contact"][:, 2], [-0.005, -0.005], atol=1e-12)


def test_collinear_end_to_end(model):
  q = state((0, 0, 0), (1, 0, 0), (0.55, 0, 0.0), (1, 0, 0))  # segment ends 0.15 apart
  assert ol.forward(model, q)["ncon"] == 0
  # segment ends 0.05 apart: a's +x end against b's -x end is found from both sides (x1 = 1,
  # then x2 = -1 with x1 clipped back to 1) -- MuJoCo's algorithm returns that contact twice
  q = state((0, 0, 0), (1, 0, 0), (0.45, 0, 0.0), (1, 0, 0))
  f = ol.forward(model, q)
  assert f["ncon"] == 2
  np.testing.assert_allclose(f["contact"][0], f["contact"][1], atol=1e-15)
  assert f["contact"][0, 2] == pytest.approx(0.05 - 2 * R, abs=1e-12)
  np.testing.assert_allclose(f["contact"][0, 6:9], [1, 0, 0], atol=1e-12)


def _seg_dist_brute(p1, a1, p2, a2, n=401):
  t = np.linspace(-1, 1, n)
  P = p1[None, :] + t[:, None] * a1[None, :]
  Q = p2[None, :] + t[:, None] * a2[None, :]
  d = np.linalg.norm(P[:, None, :] - Q[None, :, :], axis=-1)
  i, j = np.unravel_index(np.argmin(d), d.shape)
  # refine on a local grid
  ti = np.linspace(max(-1, t[i] - 0.01), min(1, t[i] + 0.01), 201)
  tj = np.linspace(max(-1, t[j] - 0.01), min(1, t[j] + 0.01), 201)
  P = p1[None, :] + ti[:, None] * a1[None, :]
  Q = p2[None, :] + tj[:, None] * a2[None, :]
  return float(np.linalg.norm(P[:, None, :] - Q[None, :, :], axis=-1).min())


def test_general_closest_points_match_brute_force(model):
  rng = np.random.default_rng(3)
  hits = 0
  for _ in range(40):
    pa = rng.uniform(-0.05, 0.05, 3)
    pb = pa + rng.uniform(-0.15, 0.15, 3)
    axa, axb = rng.normal(size=3), rng.normal(size=3)
    q = state(pa, axa, pb, axb)
    f = ol.forward(model, q)
    A1 = H * np.asarray(axa) / np.linalg.norm(axa)
    A2 = H * np.asarray(axb) / np.linalg.norm(axb)
    dist = _seg_dist_brute(pa, A1, pb, A2) - 2 * R
    if f["ncon"] == 0:
      assert dist > -1e-6
      continue
    hits += 1
    assert f["ncon"] == 1
    assert f["contact"][0, 2] == pytest.approx(dist, abs=2e-6)
  assert hits >= 10
