"""A MjSpec-like editing surface over the MJCF compiler (`compiler/`), for code that builds or
edits models programmatically the way the reference does with `mujoco.MjSpec`
(`src/mjlab/utils/spec.py`, `src/mjlab/entity/entity.py:127-207`,
`src/mjlab/scene/scene.py:30-198`).

Only what the engine runs is modelled: a body tree with free / hinge / slide joints,
primitive geoms, sites, mocap bodies, joint-transmission actuators with fixed gain and
affine bias, keyframes, `attach` with a name prefix, and `compile()` to the flat `Model`
the engine and the oracle load.  Enum names follow MuJoCo's (`mjtJoint.mjJNT_HINGE` ...).
Anything else raises at the call that asks for it.

    spec = Spec()
    body = spec.worldbody.add_body(name="b")
    body.add_joint(name="j", type=mjtJoint.mjJNT_SLIDE, axis=[0, 0, 1], range=[-1, 1])
    body.add_geom(type=mjtGeom.mjGEOM_BOX, size=[0.1, 0.1, 0.1], mass=1.0)
    create_position_actuator(spec, "j", stiffness=100.0, damping=10.0)
    model = spec.compile()

The helpers at the bottom restate `src/mjlab/utils/spec.py` on this surface.
"""

from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Callable

import numpy as np

from .compiler.mjcf import (_GEOM_DEFAULTS, _JOINT_DEFAULTS, _SITE_DEFAULTS, XBody, XGeom,
                            XJoint, XModel, XSite, parse_mjcf_string, quat_normalize)
from .compiler.model import ActuatorSpec, EntitySpec, Model, compile_scene


class mjtJoint:  # noqa: N801 - MuJoCo's enum names
  mjJNT_FREE, mjJNT_BALL, mjJNT_SLIDE, mjJNT_HINGE = 0, 1, 2, 3


class mjtGeom:  # noqa: N801
  mjGEOM_PLANE, mjGEOM_HFIELD, mjGEOM_SPHERE, mjGEOM_CAPSULE = 0, 1, 2, 3
  mjGEOM_ELLIPSOID, mjGEOM_CYLINDER, mjGEOM_BOX, mjGEOM_MESH = 4, 5, 6, 7


class mjtLimited:  # noqa: N801
  mjLIMITED_FALSE, mjLIMITED_TRUE, mjLIMITED_AUTO = 0, 1, 2


class mjtTrn:  # noqa: N801
  mjTRN_JOINT = 0


class mjtDyn:  # noqa: N801
  mjDYN_NONE = 0


class mjtGain:  # noqa: N801
  mjGAIN_FIXED = 0


class mjtBias:  # noqa: N801
  mjBIAS_NONE, mjBIAS_AFFINE = 0, 1


_JOINT_NAMES = {0: "free", 1: "ball", 2: "slide", 3: "hinge"}
_GEOM_NAMES = {0: "plane", 1: "hfield", 2: "sphere", 3: "capsule", 4: "ellipsoid",
               5: "cylinder", 6: "box", 7: "mesh"}
_LIMITED = {0: "false", 1: "true", 2: "auto"}


def _vec(v, n=None) -> tuple:
  t = tuple(float(x) for x in np.asarray(v, float).reshape(-1))
  return t if n is None else (t + (0.0,) * n)[:n]


class _Elem:
  """Attribute view over an MJCF element's resolved attribute dict (joint / geom / site)."""

  _KIND: dict = {}

  def __init__(self, x):
    object.__setattr__(self, "_x", x)

  @property
  def name(self) -> str:
    return self._x.name

  @name.setter
  def name(self, v: str) -> None:
    self._x.name = v

  def __getattr__(self, k):
    a = self._x.attrs
    if k == "type":
      return {v: i for i, v in self._KIND.items()}[a["type"]]
    if k == "limited":
      return {v: i for i, v in _LIMITED.items()}[a.get("limited", "auto")]
    if k in a:
      v = a[k]
      return np.array(v, float) if isinstance(v, tuple) else v
    raise AttributeError(k)

  def __setattr__(self, k, v):
    a = self._x.attrs
    if k == "name":
      self._x.name = v
    elif k == "type":
      a["type"] = self._KIND[int(v)]
    elif k == "limited":
      a["limited"] = _LIMITED[int(v)]
    elif isinstance(v, (list, tuple, np.ndarray)):
      a[k] = _vec(v)
    else:
      a[k] = v


class SpecJoint(_Elem):
  _KIND = _JOINT_NAMES


class SpecGeom(_Elem):
  _KIND = _GEOM_NAMES


class SpecSite(_Elem):
  _KIND = {2: "sphere"}


class SpecBody:
  """`MjsBody` subset: children bodies, joints, geoms, sites; mocap; frames."""

  def __init__(self, spec: "Spec", x: XBody):
    self._spec, self._x = spec, x

  name = property(lambda self: self._x.name)
  pos = property(lambda self: np.array(self._x.pos, float))
  quat = property(lambda self: np.array(self._x.quat, float))
  mocap = property(lambda self: bool(self._x.mocap))

  # MjsBody.mass / ipos / inertia: the body's <inertial> (bodies whose inertia comes from their
  # geoms have none to edit; give them one first)
  def _inertial(self) -> dict:
    if self._x.inertial is None:
      raise NotImplementedError(f"body '{self.name}': no explicit <inertial> to edit")
    return self._x.inertial

  @property
  def mass(self) -> float:
    return float(self._x.inertial.get("mass", 0.0)) if self._x.inertial is not None else 0.0

  @mass.setter
  def mass(self, v: float) -> None:
    self._inertial()["mass"] = float(v)

  @property
  def ipos(self) -> np.ndarray:
    return np.array(self._inertial().get("pos", (0.0, 0.0, 0.0)), float)

  @ipos.setter
  def ipos(self, v) -> None:
    self._inertial()["pos"] = _vec(v, 3)

  @property
  def inertia(self) -> np.ndarray:
    return np.array(self._inertial().get("diaginertia", (0.0, 0.0, 0.0)), float)

  @inertia.setter
  def inertia(self, v) -> None:
    inr = self._inertial()
    inr.pop("fullinertia", None)
    inr["diaginertia"] = _vec(v, 3)

  def add_body(self, name: str = "", pos=(0, 0, 0), quat=(1, 0, 0, 0), mocap: bool = False,
               mass: float | None = None, ipos=(0, 0, 0), inertia=None) -> "SpecBody":
    xb = XBody(name, np.array(_vec(pos, 3)), quat_normalize(_vec(quat, 4)), None, mocap=mocap)
    if mass is not None:
      xb.inertial = dict(mass=float(mass), pos=_vec(ipos, 3),
                         diaginertia=_vec(inertia if inertia is not None else (0, 0, 0), 3))
    self._x.children.append(xb)
    return SpecBody(self._spec, xb)

  def add_joint(self, name: str = "", type: int = mjtJoint.mjJNT_HINGE, **kw) -> SpecJoint:
    if int(type) == mjtJoint.mjJNT_BALL:
      raise NotImplementedError("ball joints")
    attrs = dict(_JOINT_DEFAULTS, type=_JOINT_NAMES[int(type)])
    j = XJoint(name, attrs)
    self._x.joints.append(j)
    sj = SpecJoint(j)
    for k, v in kw.items():
      setattr(sj, k, v)
    return sj

  def add_freejoint(self, name: str = "") -> SpecJoint:
    return self.add_joint(name, mjtJoint.mjJNT_FREE)

  def add_geom(self, name: str = "", type: int = mjtGeom.mjGEOM_SPHERE, **kw) -> SpecGeom:
    g = XGeom(name, dict(_GEOM_DEFAULTS, type=_GEOM_NAMES[int(type)]))
    self._x.geoms.append(g)
    sg = SpecGeom(g)
    for k, v in kw.items():
      setattr(sg, k, v)
    return sg

  def add_site(self, name: str = "", **kw) -> SpecSite:
    s = XSite(name, dict(_SITE_DEFAULTS))
    self._x.sites.append(s)
    ss = SpecSite(s)
    for k, v in kw.items():
      setattr(ss, k, v)
    return ss

  def add_frame(self, pos=(0, 0, 0), quat=(1, 0, 0, 0)) -> "SpecFrame":
    return SpecFrame(self, np.array(_vec(pos, 3)), quat_normalize(_vec(quat, 4)))


@dataclass
class SpecFrame:
  """`MjsFrame`: an attachment point (body + local pose) for `Spec.attach`."""
  body: SpecBody
  pos: np.ndarray
  quat: np.ndarray


@dataclass
class SpecActuator:
  """`MjsActuator` subset: joint transmission, no dynamics, fixed gain, none/affine bias."""
  name: str
  target: str
  trntype: int = mjtTrn.mjTRN_JOINT
  dyntype: int = mjtDyn.mjDYN_NONE
  gaintype: int = mjtGain.mjGAIN_FIXED
  biastype: int = mjtBias.mjBIAS_NONE
  gainprm: np.ndarray = field(default_factory=lambda: np.array([1.0] + [0.0] * 9))
  biasprm: np.ndarray = field(default_factory=lambda: np.zeros(10))
  gear: np.ndarray = field(default_factory=lambda: np.array([1.0, 0, 0, 0, 0, 0]))
  ctrllimited: bool = False
  ctrlrange: np.ndarray = field(default_factory=lambda: np.zeros(2))
  forcelimited: bool = False
  forcerange: np.ndarray = field(default_factory=lambda: np.zeros(2))
  inheritrange: float = 0.0

  def to_actuator_spec(self) -> ActuatorSpec:
    if self.trntype != mjtTrn.mjTRN_JOINT or self.dyntype != mjtDyn.mjDYN_NONE:
      raise NotImplementedError(f"actuator '{self.name}': only joint transmission, no dynamics")
    if self.gaintype != mjtGain.mjGAIN_FIXED:
      raise NotImplementedError(f"actuator '{self.name}': only fixed gain")
    if np.any(np.asarray(self.gainprm)[1:3] != 0):
      raise NotImplementedError(f"actuator '{self.name}': fixed gain uses gainprm[0] only")
    affine = self.biastype == mjtBias.mjBIAS_AFFINE
    if not affine and self.biastype != mjtBias.mjBIAS_NONE:
      raise NotImplementedError(f"actuator '{self.name}': bias none or affine")
    if np.any(np.asarray(self.gear)[1:] != 0):
      raise NotImplementedError(f"actuator '{self.name}': joint gear is gear[0]")
    bias = tuple(float(x) for x in np.asarray(self.biasprm)[:3]) if affine else (0.0, 0.0, 0.0)
    return ActuatorSpec(self.name, self.target, gain=float(self.gainprm[0]), bias=bias,
                        gear=float(self.gear[0]), ctrllimited=bool(self.ctrllimited),
                        ctrlrange=tuple(float(x) for x in self.ctrlrange),
                        forcelimited=bool(self.forcelimited),
                        forcerange=tuple(float(x) for x in self.forcerange),
                        inheritrange=float(self.inheritrange))


@dataclass
class SpecKey:
  name: str
  qpos: np.ndarray
  ctrl: np.ndarray


class Spec:
  """`mujoco.MjSpec` subset (module docstring)."""

  def __init__(self, xml: XModel | None = None):
    if xml is None:
      xml = XModel("", XBody("world", np.zeros(3), np.array([1.0, 0, 0, 0]), None), [], [],
                   True, "xyz")
    self._xml = xml
    self.actuators: list[SpecActuator] = []
    self.keys: list[SpecKey] = []
    self.option = dict(timestep=0.002, iterations=100, ls_iterations=50, tolerance=1e-8,
                       ls_tolerance=0.01, impratio=1.0, integrator="implicitfast",
                       gravity=(0.0, 0.0, -9.81))

  @staticmethod
  def from_string(text: str) -> "Spec":
    return Spec(parse_mjcf_string(text))

  @staticmethod
  def from_file(path: str) -> "Spec":
    with open(path) as f:
      return Spec.from_string(f.read())

  def copy(self) -> "Spec":
    return copy.deepcopy(self)

  @property
  def worldbody(self) -> SpecBody:
    return SpecBody(self, self._xml.world)

  def _walk(self):
    stack = [self._xml.world]
    while stack:
      b = stack.pop(0)
      yield b
      stack[0:0] = b.children

  @property
  def bodies(self) -> list[SpecBody]:
    return [SpecBody(self, b) for b in self._walk()]

  @property
  def joints(self) -> list[SpecJoint]:
    return [SpecJoint(j) for b in self._walk() for j in b.joints]

  @property
  def geoms(self) -> list[SpecGeom]:
    return [SpecGeom(g) for b in self._walk() for g in b.geoms]

  @property
  def sites(self) -> list[SpecSite]:
    return [SpecSite(s) for b in self._walk() for s in b.sites]

  def joint(self, name: str) -> SpecJoint:
    for j in self.joints:
      if j.name == name:
        return j
    raise KeyError(f"no joint '{name}'")

  def body(self, name: str) -> SpecBody:
    for b in self.bodies:
      if b.name == name:
        return b
    raise KeyError(f"no body '{name}'")

  def geom(self, name: str) -> SpecGeom:
    for g in self.geoms:
      if g.name == name:
        return g
    raise KeyError(f"no geom '{name}'")

  def actuator(self, name: str) -> SpecActuator:
    for a in self.actuators:
      if a.name == name:
        return a
    raise KeyError(f"no actuator '{name}'")

  def add_actuator(self, name: str = "", target: str = "", **kw) -> SpecActuator:
    a = SpecActuator(name, target)
    for k, v in kw.items():
      setattr(a, k, v)
    self.actuators.append(a)
    return a

  def add_key(self, name: str = "", qpos=None, ctrl=None) -> SpecKey:
    k = SpecKey(name, np.asarray(qpos if qpos is not None else [], float),
                np.asarray(ctrl if ctrl is not None else [], float))
    self.keys.append(k)
    return k

  def delete(self, obj) -> None:
    if isinstance(obj, SpecKey):
      self.keys.remove(obj)
    elif isinstance(obj, SpecActuator):
      self.actuators.remove(obj)
    else:
      raise NotImplementedError(f"delete {type(obj).__name__}")

  def attach(self, child: "Spec", prefix: str = "", frame: SpecFrame | None = None) -> None:
    """`MjSpec.attach`: the child's world children (bodies, world geoms / sites) hang off
    `frame` (default: this world body) with every name prefixed; actuators and sensors come
    along, retargeted.  Keyframes do not (MuJoCo: delete them first, re-add on the parent)."""
    if child.keys:
      raise ValueError("attach: the child spec still has keyframes")
    src = copy.deepcopy(child._xml)

    def rename(b: XBody):
      b.name = prefix + b.name if b.name else b.name
      for e in b.joints + b.geoms + b.sites:
        e.name = prefix + e.name if e.name else e.name
      for c in b.children:
        rename(c)
    for c in src.world.children:
      rename(c)
    for e in src.world.geoms + src.world.sites:
      e.name = prefix + e.name if e.name else e.name
    if frame is None:
      host = self._xml.world
      fpos, fquat = np.zeros(3), np.array([1.0, 0, 0, 0])
    else:
      host, fpos, fquat = frame.body._x, frame.pos, frame.quat
    from .compiler.mjcf import quat_mul, quat_to_mat
    R = quat_to_mat(fquat)
    for c in src.world.children:
      c.pos = fpos + R @ np.asarray(c.pos, float)
      c.quat = quat_normalize(quat_mul(fquat, c.quat))
      host.children.append(c)
    if src.world.geoms or src.world.sites:
      if frame is not None or fpos.any():
        raise NotImplementedError("attach: child world geoms / sites under a frame")
      host.geoms += src.world.geoms
      host.sites += src.world.sites
    self._xml.excludes += [(prefix + a, prefix + b) for a, b in src.excludes]
    for tag, attrs in src.sensors:
      self._xml.sensors.append((tag, {k: (prefix + v if k in ("site", "body", "joint", "objname", "name")
                                          else v) for k, v in attrs.items()}))
    for a in child.actuators:
      b = copy.deepcopy(a)
      b.name, b.target = prefix + a.name, prefix + a.target
      self.actuators.append(b)

  def compile(self, terrain: str = "none") -> Model:
    """`MjSpec.compile()`: the flat model (names unprefixed; keyframe 0 -> `key_qpos`)."""
    acts = tuple(a.to_actuator_spec() for a in self.actuators)
    ent = EntitySpec("", self._xml, actuators=acts)
    m = compile_scene([ent], terrain=terrain, **self.option)
    m.arrays["key_qpos"] = np.asarray(m.arrays["qpos0"], float).copy()  # MjSpec: no key -> qpos0
    if self.keys and self.keys[0].qpos.size:
      if self.keys[0].qpos.size != m.nq:
        raise ValueError(f"keyframe '{self.keys[0].name}': qpos size {self.keys[0].qpos.size} != nq {m.nq}")
      m.arrays["key_qpos"] = self.keys[0].qpos.astype(float).copy()
    return m


# --------------------------------------------------------------------------- utils/spec.py
def auto_wrap_fixed_base_mocap(spec_fn: Callable[[], Spec]) -> Callable[[], Spec]:
  """`src/mjlab/utils/spec.py:9-51`: a fixed-base entity is wrapped in a mocap body so each
  environment can place it; floating-base or already-mocap specs pass through."""

  def wrapper() -> Spec:
    original = spec_fn()
    if get_free_joint(original) is not None:
      return original
    bodies = original.bodies
    if len(bodies) > 1 and bodies[1].mocap:
      return original
    keys = [(k.qpos.copy(), k.ctrl.copy(), k.name) for k in original.keys]
    for k in list(original.keys):
      original.delete(k)
    wrapped = Spec()
    wrapped.option = dict(original.option)
    mocap = wrapped.worldbody.add_body(name="mocap_base", mocap=True)
    wrapped.attach(original, prefix="", frame=mocap.add_frame())
    for qpos, ctrl, name in keys:
      wrapped.add_key(name=name, qpos=qpos, ctrl=ctrl)
    return wrapped

  return wrapper


def get_non_free_joints(spec: Spec) -> tuple[SpecJoint, ...]:
  """`utils/spec.py:54-61`."""
  return tuple(j for j in spec.joints if j.type != mjtJoint.mjJNT_FREE)


def get_free_joint(spec: Spec) -> SpecJoint | None:
  """`utils/spec.py:64-71`."""
  for j in spec.joints:
    if j.type == mjtJoint.mjJNT_FREE:
      return j
  return None


def disable_collision(geom: SpecGeom) -> None:
  """`utils/spec.py:74-77`."""
  geom.contype = 0
  geom.conaffinity = 0


def is_joint_limited(jnt: SpecJoint) -> bool:
  """`utils/spec.py:80-88` (mjLIMITED_AUTO: limited iff range[0] < range[1], autolimits)."""
  lim = jnt.limited
  if lim == mjtLimited.mjLIMITED_TRUE:
    return True
  if lim == mjtLimited.mjLIMITED_AUTO:
    r = jnt.range
    return bool(r[0] < r[1])
  return False


def create_motor_actuator(spec: Spec, joint_name: str, *, effort_limit: float, gear: float = 1.0,
                          armature: float = 0.0, frictionloss: float = 0.0) -> SpecActuator:
  """`utils/spec.py:91-119`: <motor>, ctrl and force limited to +-effort_limit."""
  a = spec.add_actuator(name=joint_name, target=joint_name)
  a.trntype, a.dyntype = mjtTrn.mjTRN_JOINT, mjtDyn.mjDYN_NONE
  a.gaintype, a.biastype = mjtGain.mjGAIN_FIXED, mjtBias.mjBIAS_NONE
  a.gear[0] = gear
  a.forcelimited = True
  a.forcerange[:] = (-effort_limit, effort_limit)
  a.ctrllimited = True
  a.ctrlrange[:] = (-effort_limit, effort_limit)
  spec.joint(joint_name).armature = armature
  spec.joint(joint_name).frictionloss = frictionloss
  return a


def create_position_actuator(spec: Spec, joint_name: str, *, stiffness: float, damping: float,
                             effort_limit: float | None = None, armature: float = 0.0,
                             frictionloss: float = 0.0) -> SpecActuator:
  """`utils/spec.py:122-165`: <position> with ctrllimited False (setpoints beyond the joint
  limits are allowed), force limited when effort_limit is given."""
  a = spec.add_actuator(name=joint_name, target=joint_name)
  a.trntype, a.dyntype = mjtTrn.mjTRN_JOINT, mjtDyn.mjDYN_NONE
  a.gaintype, a.biastype = mjtGain.mjGAIN_FIXED, mjtBias.mjBIAS_AFFINE
  a.gainprm[0] = stiffness
  a.biasprm[1] = -stiffness
  a.biasprm[2] = -damping
  a.ctrllimited = False
  if effort_limit is not None:
    a.forcelimited = True
    a.forcerange[:] = (-effort_limit, effort_limit)
  else:
    a.forcelimited = False
  spec.joint(joint_name).armature = armature
  spec.joint(joint_name).frictionloss = frictionloss
  return a


def create_velocity_actuator(spec: Spec, joint_name: str, *, damping: float,
                             effort_limit: float | None = None, armature: float = 0.0,
                             frictionloss: float = 0.0, inheritrange: float = 1.0) -> SpecActuator:
  """`utils/spec.py:168-202`: <velocity>, gain = damping, bias = -damping * velocity."""
  a = spec.add_actuator(name=joint_name, target=joint_name)
  a.trntype, a.dyntype = mjtTrn.mjTRN_JOINT, mjtDyn.mjDYN_NONE
  a.gaintype, a.biastype = mjtGain.mjGAIN_FIXED, mjtBias.mjBIAS_AFFINE
  a.inheritrange = inheritrange
  a.ctrllimited = True
  a.gainprm[0] = damping
  a.biasprm[2] = -damping
  if effort_limit is not None:
    a.forcelimited = True
    a.forcerange[:] = (-effort_limit, effort_limit)
  else:
    a.forcelimited = False
  spec.joint(joint_name).armature = armature
  spec.joint(joint_name).frictionloss = frictionloss
  return a
