"""MJCF compiler breadth: MuJoCo's `inertiafromgeom` -- bodies without
an <inertial> (compiler default "auto"), or every body ("true"), take mass, centre of mass
and principal inertia from their geoms at the geom density or explicit mass; "false" keeps
them massless.  Closed forms of the primitive inertias; the shipped robot scenes, whose
bodies all carry <inertial>, compile unchanged (tests/test_model_constants.py)."""

import numpy as np
import pytest

from mjlab_amd.compiler.mjcf import parse_mjcf_string
from mjlab_amd.compiler.model import EntitySpec, compile_scene

_XML = """<mujoco><compiler angle="radian" {opt}/><worldbody>
  <body name="box" pos="0 0 1"><freejoint/>
    <geom type="box" size="0.1 0.2 0.3"/></body>
  <body name="pair" pos="1 0 1"><freejoint/>
    <geom type="sphere" size="0.1" pos="0.2 0 0"/>
    <geom type="sphere" size="0.1" pos="-0.2 0 0" mass="2"/></body>
  <body name="cap" pos="2 0 1"><freejoint/>
    <inertial pos="0 0 0" mass="7" diaginertia="1 1 1"/>
    <geom type="capsule" size="0.05 0.2" density="500"/></body>
</worldbody></mujoco>"""


def _compile(opt=""):
  m = compile_scene([EntitySpec("e", parse_mjcf_string(_XML.format(opt=opt)))], terrain="none")
  ids = {n.split("/")[-1]: i for i, n in enumerate(m.names["body"])}
  return m, ids


def test_auto_takes_geoms_where_no_inertial():
  m, ids = _compile()
  b = ids["box"]
  mass = 1000.0 * 0.2 * 0.4 * 0.6
  assert m.body_mass[b] == pytest.approx(mass)
  want = np.sort(mass / 12 * np.array([0.4 ** 2 + 0.6 ** 2, 0.2 ** 2 + 0.6 ** 2, 0.2 ** 2 + 0.4 ** 2]))
  np.testing.assert_allclose(np.sort(m.body_inertia[b]), want, rtol=1e-12)
  np.testing.assert_allclose(m.body_ipos[b], 0.0, atol=1e-12)
  p = ids["pair"]
  m1 = 1000.0 * 4 / 3 * np.pi * 0.1 ** 3
  assert m.body_mass[p] == pytest.approx(m1 + 2.0)
  com = (m1 * 0.2 - 2.0 * 0.2) / (m1 + 2.0)
  np.testing.assert_allclose(m.body_ipos[p], [com, 0, 0], atol=1e-12)
  ixx = 0.4 * 0.01 * (m1 + 2.0)
  iyy = ixx + m1 * (0.2 - com) ** 2 + 2.0 * (0.2 + com) ** 2
  np.testing.assert_allclose(np.sort(m.body_inertia[p]), np.sort([ixx, iyy, iyy]), rtol=1e-10)
  c = ids["cap"]  # explicit <inertial> wins under "auto"
  assert m.body_mass[c] == pytest.approx(7.0)


def test_true_overrides_inertial_and_false_keeps_massless():
  m, ids = _compile('inertiafromgeom="true"')
  c = ids["cap"]
  r, h = 0.05, 0.4
  vs, vc = 4 / 3 * np.pi * r ** 3, np.pi * r * r * h
  assert m.body_mass[c] == pytest.approx(500.0 * (vs + vc))
  ixy = 500.0 * (vc * (3 * r * r + h * h) / 12 + vs * (0.4 * r * r + h * h / 4 + 3 * r * h / 8))
  izz = 500.0 * (vc * r * r / 2 + vs * 0.4 * r * r)
  np.testing.assert_allclose(np.sort(m.body_inertia[c]), np.sort([ixy, ixy, izz]), rtol=1e-10)
  # "false": the inertial-less free bodies stay massless, which MuJoCo's compiler rejects
  with pytest.raises(ValueError, match="mass and inertia of moving bodies"):
    _compile('inertiafromgeom="false"')
