"""Scene compiler: parsed MJCF entities + mjlab scene edits -> one flat SoA `Model`.

Replaces the reference's MjSpec assembly + `spec.compile()` for the subset the
velocity / tracking / jump tasks need:

* scene layout: world, terrain body with a plane geom
  (`src/mjlab/terrains/terrain_importer.py:153-161`), then each entity attached
  with prefix ``"<name>/"`` (`src/mjlab/scene/scene.py:154-179`);
* `CollisionCfg.edit_spec` (`src/mjlab/utils/spec_config.py:210-238`);
* position actuators (`src/mjlab/utils/spec.py:122-165`) added per actuator cfg in
  cfg order, joints in natural order (`src/mjlab/entity/entity.py:155-168`);
* contact sensors (`src/mjlab/sensor/contact_sensor.py:159-197,472-533`);
* MuJoCo's `mj_setConst` quantities the solver consumes (subtree mass,
  `dof_invweight0`, `body_invweight0`, `meaninertia`) computed at `qpos0`.

Everything is float64 on the host; the HIP engine converts to fp32 when the model
is uploaded.
"""

from __future__ import annotations

import re
from dataclasses import dataclass, field

import numpy as np

from .mjcf import (GEOM_TYPES, JOINT_TYPES, XBody, XGeom, XModel, geom_frame, quat_mul,
                   quat_normalize, quat_to_mat)

# sensor types (values shared with include/mjx355.h)
SENS_GYRO, SENS_VELOCIMETER, SENS_ACCELEROMETER, SENS_SUBTREEANGMOM, SENS_CONTACT = 0, 1, 2, 3, 4
SENS_FRAMEPOS, SENS_FRAMEQUAT, SENS_JOINTPOS, SENS_JOINTVEL = 5, 6, 7, 8
_SENSOR_TAGS = {"gyro": SENS_GYRO, "velocimeter": SENS_VELOCIMETER,
                "accelerometer": SENS_ACCELEROMETER, "subtreeangmom": SENS_SUBTREEANGMOM,
                "framepos": SENS_FRAMEPOS, "framequat": SENS_FRAMEQUAT,
                "jointpos": SENS_JOINTPOS, "jointvel": SENS_JOINTVEL}
_SENSOR_DIM = {SENS_GYRO: 3, SENS_VELOCIMETER: 3, SENS_ACCELEROMETER: 3,
               SENS_SUBTREEANGMOM: 3, SENS_FRAMEPOS: 3, SENS_FRAMEQUAT: 4,
               SENS_JOINTPOS: 1, SENS_JOINTVEL: 1}
OBJ_BODY, OBJ_XBODY, OBJ_GEOM, OBJ_SITE, OBJ_JOINT, OBJ_NONE = 1, 2, 5, 6, 3, 0
CONTACT_FIELD_DIM = {"found": 1, "force": 3, "torque": 3, "dist": 1, "pos": 3, "normal": 3,
                     "tangent": 3}
CONTACT_FIELD_BIT = {"found": 0, "force": 1, "torque": 2, "dist": 3, "pos": 4, "normal": 5,
                     "tangent": 6}
CONTACT_REDUCE = {"none": 0, "mindist": 1, "maxforce": 2, "netforce": 3}

MINVAL = 1e-15


@dataclass
class PositionActuatorGroup:
  """`BuiltinPositionActuatorCfg` (`src/mjlab/actuator/builtin_actuator.py:27-42`)."""
  joint_names_expr: tuple[str, ...]
  stiffness: float
  damping: float
  effort_limit: float | None = None
  armature: float = 0.0
  frictionloss: float = 0.0


@dataclass
class MotorActuatorGroup:
  """`BuiltinMotorActuatorCfg` (`src/mjlab/actuator/builtin_actuator.py:80-97`): a <motor>
  per joint, `create_motor_actuator` (`src/mjlab/utils/spec.py:91-119`): force = ctrl,
  ctrl and force both limited to +-effort_limit."""
  joint_names_expr: tuple[str, ...]
  effort_limit: float
  gear: float = 1.0
  armature: float = 0.0
  frictionloss: float = 0.0


@dataclass
class VelocityActuatorGroup:
  """`BuiltinVelocityActuatorCfg` (`src/mjlab/actuator/builtin_actuator.py:130-147`): a
  <velocity> per joint, `create_velocity_actuator` (`src/mjlab/utils/spec.py:168-202`):
  force = damping * (ctrl - qvel), ctrl limited through `inheritrange` (the joint range about
  its middle), force limited when effort_limit is given."""
  joint_names_expr: tuple[str, ...]
  damping: float
  effort_limit: float | None = None
  armature: float = 0.0
  frictionloss: float = 0.0
  inheritrange: float = 1.0


@dataclass
class ActuatorSpec:
  """One joint-transmission actuator with fixed gain and affine bias (the MjsActuator subset
  the engine runs, `mjlab_amd.spec.SpecActuator.to_actuator_spec`): force = gain * ctrl + b0 +
  b1 * length + b2 * velocity, length = gear * qpos, velocity = gear * qvel; ctrl clamped to
  ctrlrange when ctrllimited, force to forcerange when forcelimited; inheritrange > 0 sets
  ctrlrange from the joint's range (MuJoCo compiler semantics).  `joint` is unprefixed."""
  name: str
  joint: str
  gain: float = 1.0
  bias: tuple = (0.0, 0.0, 0.0)
  gear: float = 1.0
  ctrllimited: bool = False
  ctrlrange: tuple = (0.0, 0.0)
  forcelimited: bool = False
  forcerange: tuple = (0.0, 0.0)
  inheritrange: float = 0.0


@dataclass
class CollisionEdit:
  """`CollisionCfg` (`src/mjlab/utils/spec_config.py:137-238`)."""
  geom_names_expr: tuple[str, ...]
  contype: int | dict = 1
  conaffinity: int | dict = 1
  condim: int | dict = 3
  priority: int | dict = 0
  friction: tuple | dict | None = None
  solref: tuple | dict | None = None
  solimp: tuple | dict | None = None
  disable_other_geoms: bool = True


@dataclass
class ContactSensorSpec:
  """Flattened `ContactSensorCfg` after pattern expansion."""
  name: str
  primary_mode: str            # geom | body | subtree
  primary_names: list[str]     # fully prefixed names
  secondary_mode: str | None
  secondary_name: str | None   # fully prefixed or None (any)
  fields: tuple[str, ...]
  reduce: str
  num_slots: int


@dataclass
class BuiltinSensorSpec:
  """A builtin sensor added by the scene config (`sensor/builtin_sensor.py:279-305`): MJCF tag
  (gyro, accelerometer, jointpos, ...), its object attribute ({"site" | "body" | "joint":
  prefixed name}) and the sensor's full name."""
  tag: str
  attrs: dict
  name: str


@dataclass
class EntitySpec:
  name: str
  xml: XModel
  collisions: tuple = ()
  actuators: tuple = ()
  init_pos: tuple = (0.0, 0.0, 0.0)
  init_rot: tuple = (1.0, 0.0, 0.0, 0.0)
  init_joint_pos: dict | None = None
  key_qpos: np.ndarray | None = None  # the entity's own keyframe qpos (init joint_pos=None)


@dataclass
class HFieldSpec:
  """Heightfield geom (config 5): elevation grid normalised to [0,1]."""
  name: str
  pos: tuple
  size: tuple                  # (sx/2, sy/2, z_max, base)
  data: np.ndarray             # (nrow, ncol) float in [0,1]


@dataclass
class BoxSpec:
  """Static box geom of a generated terrain (`terrains/primitive_terrains.py`): world
  position and half sizes (MuJoCo box size)."""
  name: str
  pos: tuple
  size: tuple


@dataclass
class Model:
  """Flat structure-of-arrays model; field names follow MuJoCo's mjModel."""
  nq: int = 0
  nv: int = 0
  nu: int = 0
  nbody: int = 0
  njnt: int = 0
  ngeom: int = 0
  nsite: int = 0
  nsensor: int = 0
  nsensordata: int = 0
  npair: int = 0
  nhfield: int = 0
  nhfielddata: int = 0
  # options (MujocoCfg, src/mjlab/sim/sim.py:42-79)
  timestep: float = 0.002
  gravity: np.ndarray = field(default_factory=lambda: np.array([0.0, 0.0, -9.81]))
  iterations: int = 100
  ls_iterations: int = 50
  tolerance: float = 1e-8
  ls_tolerance: float = 0.01
  impratio: float = 1.0
  integrator: int = 1      # 0 euler, 1 implicitfast
  cone: int = 0            # 0 pyramidal, 1 elliptic (unsupported)
  contact_maxmatch: int = 64  # SimulationCfg.contact_sensor_maxmatch (sim/sim.py:95,141)
  solver: int = 2          # 2 newton
  meaninertia: float = 1.0
  arrays: dict = field(default_factory=dict)
  names: dict = field(default_factory=dict)

  def __getattr__(self, item):
    arrays = self.__dict__.get("arrays")
    if arrays is not None and item in arrays:
      return arrays[item]
    raise AttributeError(item)

  def name2id(self, kind: str, name: str) -> int:
    return self.names[kind].index(name)


def _resolve(value, names, default):
  """`resolve_field` of mjlab's spec_config (utils/string.py:5-38): scalar or
  {regex: value} per name; first pattern that matches at the START of the name wins
  (re.match semantics, so ".*_collision" also covers "FR_thigh_collision1")."""
  if isinstance(value, dict):
    out = []
    for n in names:
      v = default
      for pat, val in value.items():
        if re.match(pat, n):
          v = val
          break
      out.append(v)
    return out
  return [value] * len(names)


def _filter_exp(exprs, names):
  """`filter_exp` (utils/string.py:24-30): prefix match (re.match)."""
  return [n for n in names if any(re.match(e, n) for e in exprs)]


def _group_actuator(grp, name: str) -> dict:
  """Builtin actuator group -> one actuator record per joint (`src/mjlab/utils/spec.py:
  91-202`: motor, position, velocity)."""
  rec = dict(name=name, joint=name, gear=1.0, gain=0.0, bias=(0.0, 0.0, 0.0), ctrllim=False,
             crange=(0.0, 0.0), forcelim=False, frange=(0.0, 0.0), inherit=0.0)
  eff = grp.effort_limit
  if isinstance(grp, PositionActuatorGroup):
    rec.update(gain=grp.stiffness, bias=(0.0, -grp.stiffness, -grp.damping))
  elif isinstance(grp, MotorActuatorGroup):
    rec.update(gain=1.0, gear=grp.gear, ctrllim=True, crange=(-eff, eff))
  elif isinstance(grp, VelocityActuatorGroup):
    rec.update(gain=grp.damping, bias=(0.0, 0.0, -grp.damping), inherit=grp.inheritrange)
  else:
    raise TypeError(f"unsupported actuator group {type(grp).__name__}")
  if eff is not None:
    rec.update(forcelim=True, frange=(-eff, eff))
  return rec


def _find_names(exprs, names):
  """Entity.find_joints / resolve_matching_names (lab_api/string.py:227): full match."""
  return [n for n in names if any(re.fullmatch(e, n) for e in exprs)]


class _Builder:
  def __init__(self):
    self.bodies = []   # dicts
    self.joints = []
    self.geoms = []
    self.sites = []

  def add_body(self, name, parent, pos, quat, inertial, mocap=False):
    self.bodies.append(dict(name=name, parent=parent, pos=np.asarray(pos, float),
                            quat=quat_normalize(quat), inertial=inertial, mocap=mocap))
    return len(self.bodies) - 1


def _geom_inertia(attrs: dict, xml: XModel):
  """Mass, frame and principal inertia of one geom at its density (or explicit mass), as
  MuJoCo's geom inertia for sphere / capsule / cylinder / box / ellipsoid; None for the
  massless types (plane, hfield) and meshes (volume unavailable without the mesh)."""
  t = attrs["type"]
  if t not in ("sphere", "capsule", "cylinder", "box", "ellipsoid"):
    return None
  pos, quat, size = geom_frame(attrs, xml.angle_deg, xml.eulerseq)
  r = float(size[0])
  if t == "sphere":
    vol, unit = 4.0 / 3.0 * np.pi * r ** 3, np.full(3, 0.4 * r * r)
  elif t == "capsule":
    h = 2.0 * float(size[1])  # cylinder length; two hemispheres of radius r at its ends
    vs, vc = 4.0 / 3.0 * np.pi * r ** 3, np.pi * r * r * h
    vol = vs + vc
    ixy = (vc * (3 * r * r + h * h) / 12 + vs * (0.4 * r * r + h * h / 4 + 3 * r * h / 8)) / vol
    unit = np.array([ixy, ixy, (vc * r * r / 2 + vs * 0.4 * r * r) / vol])
  elif t == "cylinder":
    h = 2.0 * float(size[1])
    vol = np.pi * r * r * h
    unit = np.array([(3 * r * r + h * h) / 12, (3 * r * r + h * h) / 12, r * r / 2])
  elif t == "box":
    a, b, c = (2.0 * float(x) for x in size[:3])
    vol = a * b * c
    unit = np.array([b * b + c * c, a * a + c * c, a * a + b * b]) / 12
  else:  # ellipsoid
    a, b, c = (float(x) for x in size[:3])
    vol = 4.0 / 3.0 * np.pi * a * b * c
    unit = np.array([b * b + c * c, a * a + c * c, a * a + b * b]) / 5
  mass = float(attrs["mass"]) if "mass" in attrs else float(attrs.get("density", 1000.0)) * vol
  return mass, np.asarray(pos, float), quat_to_mat(quat), mass * unit


def _inertial_from_geoms(b: XBody, xml: XModel):
  """MuJoCo's inertiafromgeom: the body's mass, centre of mass and principal inertia from
  its geoms (parallel-axis sum about the com, eigen-decomposed into ipos / iquat / diag)."""
  for x in b.geoms:
    # MuJoCo includes a mesh's volume; without the mesh this compiler cannot, and dropping
    # the geom would give silently wrong dynamics
    if x.attrs.get("type") == "mesh" and (float(x.attrs.get("mass", 0.0)) > 0.0 or
                                          float(x.attrs.get("density", 1000.0)) > 0.0):
      raise NotImplementedError(
        f"body '{b.name}': inertia from geoms needs the volume of mesh geom "
        f"'{x.attrs.get('name', '?')}' (nonzero density or mass); give the body an <inertial>")
  parts = [g for g in (_geom_inertia(x.attrs, xml) for x in b.geoms) if g is not None and g[0] > 0]
  if not parts:
    return None
  mass = sum(p[0] for p in parts)
  com = sum(p[0] * p[1] for p in parts) / mass
  I = np.zeros((3, 3))
  for m, pos, R, diag in parts:
    d = pos - com
    I += R @ np.diag(diag) @ R.T + m * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
  w, V = np.linalg.eigh(I)
  if np.linalg.det(V) < 0:
    V[:, 0] = -V[:, 0]
  from .mjcf import mat_to_quat
  return dict(mass=mass, ipos=com, iquat=quat_normalize(mat_to_quat(V)), inertia=w)


def _inertial(b: XBody, xml: XModel | None = None):
  mode = xml.inertiafromgeom if xml is not None else "false"
  if mode == "true" or (mode == "auto" and b.inertial is None):
    fg = _inertial_from_geoms(b, xml)
    if fg is not None:
      return fg
  if b.inertial is None:
    return dict(mass=0.0, ipos=np.zeros(3), iquat=np.array([1.0, 0, 0, 0]), inertia=np.zeros(3))
  inr = b.inertial
  ipos = np.asarray(inr.get("pos", (0, 0, 0)), float)
  mass = float(inr.get("mass", 0.0))
  if "fullinertia" in inr:
    xx, yy, zz, xy, xz, yz = inr["fullinertia"]
    I = np.array([[xx, xy, xz], [xy, yy, yz], [xz, yz, zz]])
    w, V = np.linalg.eigh(I)
    if np.linalg.det(V) < 0:
      V[:, 0] = -V[:, 0]
    from .mjcf import mat_to_quat
    iquat = quat_mul(quat_normalize(inr.get("quat", (1, 0, 0, 0))), mat_to_quat(V))
    inertia = w
  else:
    iquat = quat_normalize(inr.get("quat", (1, 0, 0, 0)))
    inertia = np.asarray(inr.get("diaginertia", (0, 0, 0)), float)
  return dict(mass=mass, ipos=ipos, iquat=iquat, inertia=inertia)


def compile_scene(entities: list[EntitySpec], *, terrain: str = "plane",
                  hfields: list[HFieldSpec] | None = None,
                  terrain_geoms: list | None = None,
                  contact_sensors: list[ContactSensorSpec] = (),
                  timestep=0.002, iterations=100, ls_iterations=50, tolerance=1e-8,
                  ls_tolerance=0.01, impratio=1.0, integrator="implicitfast",
                  gravity=(0.0, 0.0, -9.81), cone="pyramidal") -> Model:
  """Assemble and compile a scene.  Body/geom ordering follows MuJoCo's depth-first
  spec order: world, terrain, then each attached entity.  terrain: "plane", "generator"
  (terrain_geoms: the TerrainGenerator's HFieldSpec / BoxSpec geoms in generation order,
  on the static `terrain` body, `terrains/terrain_generator.py:93-114`), "hfield" (the
  same with heightfields only) or "none"."""
  if cone != "pyramidal":
    raise NotImplementedError("only pyramidal friction cones are supported")
  B = _Builder()
  B.add_body("world", -1, np.zeros(3), np.array([1.0, 0, 0, 0]), None)
  geoms, sites, joints = [], [], []
  excludes = []
  xml_sensors = []
  keyframe_parts = []  # (qposadr, values)
  actuators = []

  def add_geom(body, name, attrs, xml):
    pos, quat, size = geom_frame(attrs, xml.angle_deg, xml.eulerseq) if xml else (
      np.asarray(attrs["pos"], float), quat_normalize(attrs["quat"]), np.asarray(attrs["size"], float))
    g = dict(body=body, name=name, type=GEOM_TYPES[attrs["type"]], size=size, pos=pos,
             quat=quat, contype=int(attrs["contype"]), conaffinity=int(attrs["conaffinity"]),
             condim=int(attrs["condim"]), priority=int(attrs["priority"]),
             friction=np.array(list(attrs["friction"]) + [0.005, 0.0001][len(attrs["friction"]) - 1:]
                               if len(attrs["friction"]) < 3 else attrs["friction"][:3], float),
             solmix=float(attrs["solmix"]), solref=np.array(attrs["solref"], float),
             solimp=np.array(list(attrs["solimp"]) + [0.5, 2.0][len(attrs["solimp"]) - 3:]
                             if len(attrs["solimp"]) < 5 else attrs["solimp"][:5], float),
             margin=float(attrs["margin"]), gap=float(attrs["gap"]), hfield=-1)
    geoms.append(g)
    return g

  # ---------------------------------------------------------------- terrain
  if terrain == "plane":
    tb = B.add_body("terrain", 0, np.zeros(3), np.array([1.0, 0, 0, 0]), None)
    from .mjcf import _GEOM_DEFAULTS
    add_geom(tb, "terrain", dict(_GEOM_DEFAULTS, type="plane", size=(0.0, 0.0, 0.01)), None)
  elif terrain in ("hfield", "generator"):
    tb = B.add_body("terrain", 0, np.zeros(3), np.array([1.0, 0, 0, 0]), None)
    from .mjcf import _GEOM_DEFAULTS
    tgeoms = list(terrain_geoms if terrain_geoms is not None else (hfields or []))
    hfields = [t for t in tgeoms if isinstance(t, HFieldSpec)]
    hi = 0
    for tg in tgeoms:
      if isinstance(tg, HFieldSpec):
        g = add_geom(tb, tg.name, dict(_GEOM_DEFAULTS, type="hfield", pos=tg.pos,
                                        size=(tg.size[0], tg.size[1], tg.size[2])), None)
        g["hfield"] = hi
        hi += 1
      else:
        add_geom(tb, tg.name, dict(_GEOM_DEFAULTS, type="box", pos=tg.pos, size=tg.size), None)
  elif terrain is not None and terrain != "none":
    raise ValueError(f"unknown terrain {terrain}")

  # ---------------------------------------------------------------- entities
  for ent in entities:
    prefix = f"{ent.name}/" if ent.name else ""
    xml = ent.xml
    # entity-level geom edits (CollisionCfg), applied on unprefixed names
    all_geom_names = []

    def collect(b: XBody):
      for g in b.geoms:
        all_geom_names.append(g.name)
      for c in b.children:
        collect(c)
    for c in xml.world.children:
      collect(c)
    edits = {}
    for ce in ent.collisions:
      subset = _filter_exp(ce.geom_names_expr, [n for n in all_geom_names if n])
      res = {k: _resolve(getattr(ce, k), subset, d) for k, d in
             dict(condim=3, contype=1, conaffinity=1, priority=0, friction=None, solref=None,
                  solimp=None).items()}
      for i, n in enumerate(subset):
        e = edits.setdefault(n, {})
        for k in ("condim", "contype", "conaffinity", "priority"):
          e[k] = res[k][i]
        for k in ("friction", "solref", "solimp"):
          if res[k][i] is not None:
            e[k] = tuple(res[k][i])
      if ce.disable_other_geoms:
        for n in all_geom_names:
          if n not in subset:
            edits.setdefault(("__disable__", n) if not n else n, {}).update(contype=0, conaffinity=0)
      # unnamed geoms are "other geoms" too
      if ce.disable_other_geoms:
        edits["__unnamed__"] = dict(contype=0, conaffinity=0)

    qposadr = 0 if not joints else None  # recomputed later
    joint_name_order = []

    def walk(xb: XBody, parent: int):
      bid = B.add_body(prefix + xb.name, parent, xb.pos, xb.quat, _inertial(xb, xml), xb.mocap)
      for j in xb.joints:
        joints.append(dict(body=bid, name=prefix + j.name, attrs=j.attrs))
        if j.attrs["type"] != "free":
          joint_name_order.append(j.name)
      for g in xb.geoms:
        attrs = dict(g.attrs)
        if g.name:
          attrs.update({k: v for k, v in edits.get(g.name, {}).items()})
        elif "__unnamed__" in edits:
          attrs.update(edits["__unnamed__"])
        if attrs.get("friction") is not None and len(attrs["friction"]) < 3:
          f = list(attrs["friction"])
          attrs["friction"] = tuple(f + list(_GEOM_DEFAULTS_FRICTION[len(f):]))
        add_geom(bid, prefix + g.name if g.name else "", attrs, xml)
      for s in xb.sites:
        pos = np.asarray(s.attrs["pos"], float)
        from .mjcf import _orientation
        sites.append(dict(body=bid, name=prefix + s.name, pos=pos,
                          quat=_orientation(s.attrs, xml.angle_deg, xml.eulerseq)))
      for c in xb.children:
        walk(c, bid)

    for c in xml.world.children:
      walk(c, 0)
    for g in xml.world.geoms:
      add_geom(0, prefix + g.name if g.name else "", dict(g.attrs), xml)
    for (b1, b2) in xml.excludes:
      excludes.append((prefix + b1, prefix + b2))
    for tag, attrs in xml.sensors:
      xml_sensors.append((tag, {k: (prefix + v if k in ("site", "body", "joint", "objname")
                                    else v) for k, v in attrs.items()},
                          prefix + attrs.get("name", "")))
    # actuators (cfg order, joints in natural order)
    for grp in ent.actuators:
      if isinstance(grp, ActuatorSpec):
        if grp.joint not in joint_name_order:
          raise ValueError(f"actuator '{grp.name}': no joint '{grp.joint}'")
        actuators.append(dict(name=prefix + grp.name, joint=prefix + grp.joint, gear=grp.gear,
                              gain=grp.gain, bias=tuple(grp.bias), ctrllim=bool(grp.ctrllimited),
                              crange=tuple(grp.ctrlrange), forcelim=bool(grp.forcelimited),
                              frange=tuple(grp.forcerange), inherit=grp.inheritrange))
        continue
      names = _find_names(grp.joint_names_expr, joint_name_order)
      if not names:
        raise ValueError(f"no joints for actuator {grp.joint_names_expr}")
      for n in names:
        for j in joints:
          if j["name"] == prefix + n:
            j["attrs"] = dict(j["attrs"], armature=grp.armature, frictionloss=grp.frictionloss)
        actuators.append(_group_actuator(grp, prefix + n))
    keyframe_parts.append((ent, joint_name_order))

  # ---------------------------------------------------------------- flatten
  m = Model()
  nbody = len(B.bodies)
  m.nbody, m.njnt, m.ngeom, m.nsite = nbody, len(joints), len(geoms), len(sites)
  A = m.arrays
  A["body_parentid"] = np.array([max(b["parent"], 0) for b in B.bodies], np.int32)
  A["body_parentid"][0] = 0
  A["body_pos"] = np.array([b["pos"] for b in B.bodies])
  A["body_quat"] = np.array([b["quat"] for b in B.bodies])
  inr = [b["inertial"] or _inertial(XBody("", np.zeros(3), np.zeros(4), None)) for b in B.bodies]
  A["body_mass"] = np.array([i["mass"] for i in inr])
  A["body_ipos"] = np.array([i["ipos"] for i in inr])
  A["body_iquat"] = np.array([i["iquat"] for i in inr])
  A["body_inertia"] = np.array([i["inertia"] for i in inr])
  A["body_mocapid"] = np.full(nbody, -1, np.int32)
  nmocap = 0
  for i, b in enumerate(B.bodies):
    if b["mocap"]:
      A["body_mocapid"][i] = nmocap
      nmocap += 1
  m.names["body"] = [b["name"] for b in B.bodies]

  # joints / dofs
  jtype = np.array([JOINT_TYPES[j["attrs"]["type"]] for j in joints], np.int32)
  nqj = {0: 7, 1: 4, 2: 1, 3: 1}
  nvj = {0: 6, 1: 3, 2: 1, 3: 1}
  A["jnt_type"] = jtype
  A["jnt_bodyid"] = np.array([j["body"] for j in joints], np.int32)
  A["jnt_qposadr"] = np.zeros(m.njnt, np.int32)
  A["jnt_dofadr"] = np.zeros(m.njnt, np.int32)
  qa = da = 0
  for k in range(m.njnt):
    A["jnt_qposadr"][k], A["jnt_dofadr"][k] = qa, da
    qa += nqj[int(jtype[k])]
    da += nvj[int(jtype[k])]
  m.nq, m.nv = qa, da
  A["jnt_pos"] = np.array([j["attrs"]["pos"] for j in joints], float).reshape(-1, 3)
  ax = np.array([j["attrs"]["axis"] for j in joints], float).reshape(-1, 3)
  A["jnt_axis"] = ax / np.maximum(np.linalg.norm(ax, axis=1, keepdims=True), MINVAL)
  rng = np.array([j["attrs"]["range"] for j in joints], float).reshape(-1, 2)
  lim = []
  for j, r in zip(joints, rng):
    l = j["attrs"]["limited"]
    lim.append(1 if (l == "true" or (l == "auto" and r[0] < r[1])) and j["attrs"]["type"] != "free" else 0)
  A["jnt_limited"] = np.array(lim, np.int32)
  A["jnt_range"] = rng
  A["jnt_solref"] = np.array([j["attrs"]["solreflimit"] for j in joints], float).reshape(-1, 2)
  A["jnt_solimp"] = np.array([j["attrs"]["solimplimit"] for j in joints], float).reshape(-1, 5)
  A["jnt_margin"] = np.array([j["attrs"]["margin"] for j in joints], float)
  A["jnt_stiffness"] = np.array([j["attrs"]["stiffness"] for j in joints], float)
  m.names["joint"] = [j["name"] for j in joints]

  body_jntadr = np.full(nbody, -1, np.int32)
  body_jntnum = np.zeros(nbody, np.int32)
  for k, j in enumerate(joints):
    b = j["body"]
    if body_jntadr[b] < 0:
      body_jntadr[b] = k
    body_jntnum[b] += 1
  A["body_jntadr"], A["body_jntnum"] = body_jntadr, body_jntnum
  dof_bodyid = np.zeros(m.nv, np.int32)
  dof_jntid = np.zeros(m.nv, np.int32)
  dof_armature = np.zeros(m.nv)
  dof_damping = np.zeros(m.nv)
  dof_frictionloss = np.zeros(m.nv)
  for k, j in enumerate(joints):
    for d in range(nvj[int(jtype[k])]):
      i = A["jnt_dofadr"][k] + d
      dof_bodyid[i], dof_jntid[i] = j["body"], k
      dof_armature[i] = j["attrs"]["armature"]
      dof_damping[i] = j["attrs"]["damping"]
      dof_frictionloss[i] = j["attrs"]["frictionloss"]
  body_dofadr = np.full(nbody, -1, np.int32)
  body_dofnum = np.zeros(nbody, np.int32)
  for i in range(m.nv):
    b = dof_bodyid[i]
    if body_dofadr[b] < 0:
      body_dofadr[b] = i
    body_dofnum[b] += 1
  A["body_dofadr"], A["body_dofnum"] = body_dofadr, body_dofnum
  # dof_parentid: previous dof in same body, else last dof of nearest ancestor with dofs
  dof_parentid = np.full(m.nv, -1, np.int32)
  for i in range(m.nv):
    b = dof_bodyid[i]
    if i > body_dofadr[b]:
      dof_parentid[i] = i - 1
    else:
      p = A["body_parentid"][b]
      while p > 0 and body_dofnum[p] == 0:
        p = A["body_parentid"][p]
      dof_parentid[i] = body_dofadr[p] + body_dofnum[p] - 1 if p > 0 else -1
  A["dof_bodyid"], A["dof_jntid"], A["dof_parentid"] = dof_bodyid, dof_jntid, dof_parentid
  A["dof_armature"], A["dof_damping"], A["dof_frictionloss"] = dof_armature, dof_damping, dof_frictionloss
  if (dof_frictionloss > 0).any():  # MuJoCo adds a friction-loss constraint row per such dof
    raise NotImplementedError(
      "dof frictionloss > 0: the engine has no friction-loss constraint rows "
      f"(dofs {np.nonzero(dof_frictionloss > 0)[0].tolist()})")

  # root / weld ids, tree levels
  rootid = np.zeros(nbody, np.int32)
  weldid = np.zeros(nbody, np.int32)
  level = np.zeros(nbody, np.int32)
  for b in range(1, nbody):
    p = A["body_parentid"][b]
    rootid[b] = b if p == 0 else rootid[p]
    weldid[b] = b if body_jntnum[b] > 0 else weldid[p]
    level[b] = level[p] + 1
  A["body_rootid"], A["body_weldid"], A["body_level"] = rootid, weldid, level

  # qpos0 (MuJoCo: free joint = body pose, hinge/slide = ref) and springref
  qpos0 = np.zeros(m.nq)
  for k, j in enumerate(joints):
    a = A["jnt_qposadr"][k]
    if jtype[k] == 0:
      qpos0[a:a + 3] = A["body_pos"][j["body"]]
      qpos0[a + 3:a + 7] = A["body_quat"][j["body"]]
    elif jtype[k] == 1:
      qpos0[a:a + 4] = (1, 0, 0, 0)
    else:
      qpos0[a] = j["attrs"]["ref"]
  A["qpos0"] = qpos0
  A["qpos_spring"] = qpos0.copy()

  # geoms
  m.names["geom"] = [g["name"] for g in geoms]
  A["geom_type"] = np.array([g["type"] for g in geoms], np.int32)
  A["geom_bodyid"] = np.array([g["body"] for g in geoms], np.int32)
  for k in ("contype", "conaffinity", "condim", "priority"):
    A["geom_" + k] = np.array([g[k] for g in geoms], np.int32)
  for k in ("size", "pos", "quat", "friction", "solref", "solimp"):
    A["geom_" + k] = np.array([g[k] for g in geoms], float)
  for k in ("solmix", "margin", "gap"):
    A["geom_" + k] = np.array([g[k] for g in geoms], float)
  A["geom_dataid"] = np.array([g["hfield"] for g in geoms], np.int32)
  rb = np.zeros(m.ngeom)
  for i, g in enumerate(geoms):
    t, s = g["type"], g["size"]
    if t == GEOM_TYPES["sphere"]:
      rb[i] = s[0]
    elif t == GEOM_TYPES["capsule"]:
      rb[i] = s[0] + s[1]
    elif t == GEOM_TYPES["box"]:
      rb[i] = float(np.linalg.norm(s[:3]))
    elif t == GEOM_TYPES["cylinder"]:
      rb[i] = float(np.hypot(s[0], s[1]))
    elif t == GEOM_TYPES["ellipsoid"]:
      rb[i] = float(np.max(s[:3]))
    elif t == GEOM_TYPES["hfield"]:
      rb[i] = float(np.linalg.norm(s[:3]))
    else:
      rb[i] = 0.0
  A["geom_rbound"] = rb

  # sites
  m.names["site"] = [s["name"] for s in sites]
  A["site_bodyid"] = np.array([s["body"] for s in sites], np.int32)
  A["site_pos"] = np.array([s["pos"] for s in sites], float).reshape(-1, 3)
  A["site_quat"] = np.array([s["quat"] for s in sites], float).reshape(-1, 4)

  # actuators
  m.nu = len(actuators)
  m.names["actuator"] = [a["name"] for a in actuators]
  jname = m.names["joint"]
  A["actuator_trnid"] = np.array([jname.index(a["joint"]) for a in actuators], np.int32)
  A["actuator_gear"] = np.ones(m.nu)
  A["actuator_gainprm"] = np.zeros((m.nu, 3))
  A["actuator_biasprm"] = np.zeros((m.nu, 3))
  A["actuator_forcelimited"] = np.zeros(m.nu, np.int32)
  A["actuator_forcerange"] = np.zeros((m.nu, 2))
  A["actuator_ctrllimited"] = np.zeros(m.nu, np.int32)
  A["actuator_ctrlrange"] = np.zeros((m.nu, 2))
  for i, a in enumerate(actuators):
    A["actuator_gear"][i] = a["gear"]
    A["actuator_gainprm"][i, 0] = a["gain"]
    A["actuator_biasprm"][i] = a["bias"]
    if a["forcelim"]:
      A["actuator_forcelimited"][i] = 1
      A["actuator_forcerange"][i] = a["frange"]
    if a["ctrllim"]:
      A["actuator_ctrllimited"][i] = 1
      A["actuator_ctrlrange"][i] = a["crange"]
    if a["inherit"] > 0:  # MuJoCo: ctrlrange = range midpoint +- inheritrange * half range
      k = int(A["actuator_trnid"][i])
      lo, hi = (float(x) for x in A["jnt_range"][k])
      if not A["jnt_limited"][k] or not lo < hi:
        raise ValueError(f"actuator '{a['name']}': inheritrange needs a limited joint")
      mid, half = 0.5 * (lo + hi), 0.5 * (hi - lo) * a["inherit"]
      A["actuator_ctrllimited"][i] = 1
      A["actuator_ctrlrange"][i] = (mid - half, mid + half)

  # collision candidate pairs (static broadphase filter, MuJoCo filterBodyPair rules),
  # vectorised over the geom pairs i < j (a generated terrain has thousands of geoms)
  body_names = m.names["body"]
  excl = set()
  for b1, b2 in excludes:
    i1, i2 = body_names.index(b1), body_names.index(b2)
    excl.add((min(i1, i2), max(i1, i2)))
  gtype = A["geom_type"]
  ct, ca = A["geom_contype"], A["geom_conaffinity"]
  wg = weldid[A["geom_bodyid"]]
  pwg = weldid[A["body_parentid"][wg]]
  ok = ((ct[:, None] & ca[None, :]) | (ct[None, :] & ca[:, None])) != 0
  ok &= wg[:, None] != wg[None, :]
  ok &= ~((wg[:, None] != 0) & (wg[None, :] != 0) & ((wg[:, None] == pwg[None, :]) | (wg[None, :] == pwg[:, None])))
  pl, hfT = GEOM_TYPES["plane"], GEOM_TYPES["hfield"]
  flat = (gtype == pl) | (gtype == hfT)
  ok &= ~(flat[:, None] & flat[None, :])  # plane-plane, hfield-plane, hfield-hfield
  ii, jj = np.nonzero(np.triu(ok, 1))
  pairs = []
  for i, j in zip(ii.tolist(), jj.tolist()):
    bi, bj = int(A["geom_bodyid"][i]), int(A["geom_bodyid"][j])
    if excl and (min(bi, bj), max(bi, bj)) in excl:
      continue
    pairs.append((i, j) if gtype[i] <= gtype[j] else (j, i))
  # static terrain pairs last, grouped by their static geom (a heightfield, or a box welded
  # to the world): the engine's terrain broadphase walks them as per-geom blocks behind
  # chunk / geom bounding-box culls; capi.cpp checks the layout
  static = (gtype == hfT) | ((gtype == GEOM_TYPES["box"]) & (wg == 0))
  def tail_key(pr):
    a, b = pr
    sg = a if static[a] else (b if static[b] else -1)
    return (sg >= 0, sg)
  pairs.sort(key=tail_key)
  m.npair = len(pairs)
  A["pair_geom1"] = np.array([p[0] for p in pairs], np.int32)
  A["pair_geom2"] = np.array([p[1] for p in pairs], np.int32)

  # heightfields
  hfields = hfields or []
  m.nhfield = len(hfields)
  A["hfield_nrow"] = np.array([h.data.shape[0] for h in hfields], np.int32)
  A["hfield_ncol"] = np.array([h.data.shape[1] for h in hfields], np.int32)
  A["hfield_size"] = np.array([h.size for h in hfields], float).reshape(-1, 4)
  adr, acc = [], 0
  for h in hfields:
    adr.append(acc)
    acc += h.data.size
  A["hfield_adr"] = np.array(adr, np.int32)
  # float32 like the reference's hfield userdata (heightfield_terrains.py:220)
  A["hfield_data"] = (np.concatenate([np.asarray(h.data, np.float32).reshape(-1) for h in hfields])
                      if hfields else np.zeros(0, np.float32))
  m.nhfielddata = acc

  # sensors
  stype, sobjtype, sobjid, sreftype, srefid, sadr, sdim, sint = [], [], [], [], [], [], [], []
  snames = []
  smask1, smask2 = [], []
  adr = 0
  nmw = max(1, (m.ngeom + 31) // 32)  # mask words per sensor (mjxModelDesc.nmaskword)

  def push(t, ot, oi, rt, ri, dim, intprm=(0, 0, 0), name="", mk1=None, mk2=None):
    nonlocal adr
    stype.append(t); sobjtype.append(ot); sobjid.append(oi); sreftype.append(rt)
    srefid.append(ri); sadr.append(adr); sdim.append(dim); sint.append(intprm)
    snames.append(name)
    smask1.append(mk1 if mk1 is not None else np.zeros(nmw, np.uint32))
    smask2.append(mk2 if mk2 is not None else np.zeros(nmw, np.uint32))
    adr += dim

  def push_builtin(tag, attrs, name):
    if tag not in _SENSOR_TAGS:
      raise NotImplementedError(f"sensor '{name}': type {tag!r} (supported: {sorted(_SENSOR_TAGS)})")
    t = _SENSOR_TAGS[tag]
    if "site" in attrs:
      ot, oi = OBJ_SITE, m.names["site"].index(attrs["site"])
    elif "body" in attrs:
      ot, oi = OBJ_BODY, body_names.index(attrs["body"])
    elif "joint" in attrs:
      ot, oi = OBJ_JOINT, jname.index(attrs["joint"])
    else:
      raise ValueError(f"unsupported sensor attrs {attrs}")
    push(t, ot, oi, OBJ_NONE, -1, _SENSOR_DIM[t], name=name)

  for tag, attrs, name in xml_sensors:
    push_builtin(tag, attrs, name)

  children = [[] for _ in range(nbody)]
  for b in range(1, nbody):
    children[A["body_parentid"][b]].append(b)

  def subtree(b):
    out = [b]
    for c in children[b]:
      out += subtree(c)
    return out

  def geom_mask(mode, name):
    mk = np.zeros(nmw, np.uint32)
    if name is None:
      mk[:] = 0xFFFFFFFF
      return mk
    if mode == "geom":
      gs = [m.names["geom"].index(name)]
    elif mode == "body":
      b = body_names.index(name)
      gs = [g for g in range(m.ngeom) if A["geom_bodyid"][g] == b]
    elif mode == "subtree":
      bs = set(subtree(body_names.index(name)))
      gs = [g for g in range(m.ngeom) if A["geom_bodyid"][g] in bs]
    else:
      raise ValueError(mode)
    for g in gs:
      mk[g // 32] |= np.uint32(1 << (g % 32))
    return mk

  objmode = {"geom": OBJ_GEOM, "body": OBJ_BODY, "subtree": OBJ_XBODY}
  for cs in contact_sensors:
    if isinstance(cs, BuiltinSensorSpec):  # scene-config sensors keep the config's order
      push_builtin(cs.tag, cs.attrs, cs.name)
      continue
    for prim in cs.primary_names:
      for fld in cs.fields:
        m1 = geom_mask(cs.primary_mode, prim)
        m2 = geom_mask(cs.secondary_mode, cs.secondary_name)
        intprm = (1 << CONTACT_FIELD_BIT[fld], CONTACT_REDUCE[cs.reduce], cs.num_slots)
        push(SENS_CONTACT, objmode[cs.primary_mode], 0,
             objmode[cs.secondary_mode] if cs.secondary_mode else OBJ_NONE, 0,
             CONTACT_FIELD_DIM[fld] * cs.num_slots, intprm,
             name=f"{cs.name}_{prim.split('/')[-1]}_{fld}", mk1=m1, mk2=m2)
  m.nsensor = len(stype)
  m.nsensordata = adr
  A["sensor_type"] = np.array(stype, np.int32)
  A["sensor_objtype"] = np.array(sobjtype, np.int32)
  A["sensor_objid"] = np.array(sobjid, np.int32)
  A["sensor_reftype"] = np.array(sreftype, np.int32)
  A["sensor_refid"] = np.array(srefid, np.int32)
  A["sensor_adr"] = np.array(sadr, np.int32)
  A["sensor_dim"] = np.array(sdim, np.int32)
  A["sensor_intprm"] = np.array(sint, np.int32).reshape(-1, 3)
  A["sensor_geommask1"] = np.array(smask1, np.uint32).reshape(-1, nmw)
  A["sensor_geommask2"] = np.array(smask2, np.uint32).reshape(-1, nmw)
  m.names["sensor"] = snames

  # keyframe "init_state" (src/mjlab/entity/entity.py:170-207)
  key = qpos0.copy()
  for ent, jorder in keyframe_parts:
    prefix = f"{ent.name}/" if ent.name else ""
    if ent.key_qpos is not None:
      # the entity's own keyframe (entity.py:171-182), in its joint order
      own = [k for k, j in enumerate(joints) if j["name"].startswith(prefix)]
      width = sum(nqj[int(jtype[k])] for k in own)
      if np.asarray(ent.key_qpos).size != width:
        raise ValueError(f"entity '{ent.name}': keyframe qpos size {np.asarray(ent.key_qpos).size} != {width}")
      off = 0
      for k in own:
        a, w = A["jnt_qposadr"][k], nqj[int(jtype[k])]
        key[a:a + w] = np.asarray(ent.key_qpos, float)[off:off + w]
        off += w
      continue
    for k, j in enumerate(joints):
      if not j["name"].startswith(prefix):
        continue
      a = A["jnt_qposadr"][k]
      if jtype[k] == 0:
        key[a:a + 3] = ent.init_pos
        key[a + 3:a + 7] = ent.init_rot
      elif ent.init_joint_pos is not None:
        short = j["name"][len(prefix):]
        for pat, val in ent.init_joint_pos.items():  # resolve_expr: re.match semantics
          if re.match(pat, short):
            key[a] = val
            break
  A["key_qpos"] = key

  # options
  m.timestep, m.iterations, m.ls_iterations = timestep, iterations, ls_iterations
  m.tolerance, m.ls_tolerance, m.impratio = tolerance, ls_tolerance, impratio
  m.integrator = {"euler": 0, "implicitfast": 1}[integrator]
  m.gravity = np.asarray(gravity, float)

  # tree helpers for the HIP engine (level lists, children lists, dof->body masks)
  nlev = int(level.max()) + 1
  order = np.argsort(level, kind="stable").astype(np.int32)
  A["level_start"] = np.searchsorted(level[order], np.arange(nlev + 1)).astype(np.int32)
  A["level_body"] = order
  cadr, clist = [], []
  for b in range(nbody):
    cadr.append(len(clist))
    clist += children[b]
  cadr.append(len(clist))
  A["body_childadr"] = np.array(cadr, np.int32)
  A["body_child"] = np.array(clist if clist else [0], np.int32)
  if nbody > 64:
    raise ValueError("engine supports at most 64 bodies per world")
  dmask = np.zeros(m.nv, np.uint64)
  for i in range(m.nv):
    for b in subtree(int(dof_bodyid[i])):
      dmask[i] |= np.uint64(1) << np.uint64(b)
  A["dof_bodymask"] = dmask

  _set_const(m)
  return m


_GEOM_DEFAULTS_FRICTION = (1.0, 0.005, 0.0001)


# ---------------------------------------------------------------------------- setConst
def _kinematics_at(m: Model, qpos):
  """fp64 kinematics + com + cdof + CRB mass matrix at `qpos` (setup only)."""
  A = m.arrays
  nb = m.nbody
  xpos = np.zeros((nb, 3))
  xmat = np.zeros((nb, 3, 3))
  xmat[0] = np.eye(3)
  xquat = np.zeros((nb, 4))
  xquat[0] = (1, 0, 0, 0)
  xanchor = np.zeros((m.njnt, 3))
  xaxis = np.zeros((m.njnt, 3))
  for b in range(1, nb):
    p = A["body_parentid"][b]
    pos = xpos[p] + xmat[p] @ A["body_pos"][b]
    q = quat_mul(xquat[p], A["body_quat"][b])
    for k in range(A["body_jntadr"][b], A["body_jntadr"][b] + A["body_jntnum"][b]):
      t = A["jnt_type"][k]
      a = A["jnt_qposadr"][k]
      if t == 0:
        pos = qpos[a:a + 3].copy()
        q = quat_normalize(qpos[a + 3:a + 7])
        xanchor[k] = pos
        xaxis[k] = quat_to_mat(q) @ A["jnt_axis"][k]
        continue
      R = quat_to_mat(q)
      xanchor[k] = R @ A["jnt_pos"][k] + pos
      xaxis[k] = R @ A["jnt_axis"][k]
      if t == 3:
        from .mjcf import axisangle_to_quat
        q = quat_mul(q, axisangle_to_quat(A["jnt_axis"][k], qpos[a] - A["qpos0"][a]))
        pos = xanchor[k] - quat_to_mat(q) @ A["jnt_pos"][k]
      elif t == 2:
        pos = pos + xaxis[k] * (qpos[a] - A["qpos0"][a])
      else:
        raise NotImplementedError("ball joints")
    q = quat_normalize(q)
    xpos[b], xquat[b], xmat[b] = pos, q, quat_to_mat(q)
  xipos = np.array([xpos[b] + xmat[b] @ A["body_ipos"][b] for b in range(nb)])
  ximat = np.array([xmat[b] @ quat_to_mat(A["body_iquat"][b]) for b in range(nb)])
  mass = A["body_mass"]
  # subtree com
  stm = mass.copy()
  stc = mass[:, None] * xipos
  for b in range(nb - 1, 0, -1):
    p = A["body_parentid"][b]
    stm[p] += stm[b]
    stc[p] += stc[b]
  subtree_com = np.where(stm[:, None] > MINVAL, stc / np.maximum(stm[:, None], MINVAL), xipos)
  # cdof
  cdof = np.zeros((m.nv, 6))
  for k in range(m.njnt):
    b = A["jnt_bodyid"][k]
    off = subtree_com[A["body_rootid"][b]]
    d = A["jnt_dofadr"][k]
    t = A["jnt_type"][k]
    if t == 0:
      for i in range(3):
        cdof[d + i, 3 + i] = 1.0
      for i in range(3):
        ax = xmat[b][:, i]
        cdof[d + 3 + i, :3] = ax
        cdof[d + 3 + i, 3:] = np.cross(ax, off - xanchor[k])
    elif t == 3:
      cdof[d, :3] = xaxis[k]
      cdof[d, 3:] = np.cross(xaxis[k], off - xanchor[k])
    elif t == 2:
      cdof[d, 3:] = xaxis[k]
  # spatial inertias (6x6) at offset
  crb = np.zeros((nb, 6, 6))
  for b in range(1, nb):
    off = subtree_com[A["body_rootid"][b]]
    I = ximat[b] @ np.diag(A["body_inertia"][b]) @ ximat[b].T
    dvec = xipos[b] - off
    Ic = I + mass[b] * (np.dot(dvec, dvec) * np.eye(3) - np.outer(dvec, dvec))
    S = np.zeros((6, 6))
    S[:3, :3] = Ic
    h = mass[b] * dvec
    hx = np.array([[0, -h[2], h[1]], [h[2], 0, -h[0]], [-h[1], h[0], 0]])
    S[:3, 3:] = hx
    S[3:, :3] = -hx
    S[3:, 3:] = mass[b] * np.eye(3)
    crb[b] = S
  for b in range(nb - 1, 0, -1):
    p = A["body_parentid"][b]
    if p > 0:
      crb[p] += crb[b]
  M = np.zeros((m.nv, m.nv))
  for i in range(m.nv):
    f = crb[A["dof_bodyid"][i]] @ cdof[i]
    j = i
    while j >= 0:
      M[i, j] = M[j, i] = cdof[j] @ f
      j = A["dof_parentid"][j]
  M[np.diag_indices(m.nv)] += A["dof_armature"]
  return dict(xpos=xpos, xmat=xmat, xipos=xipos, subtree_com=subtree_com, cdof=cdof, M=M,
              stm=stm)


def _set_const(m: Model):
  A = m.arrays
  k = _kinematics_at(m, A["qpos0"])
  A["body_subtreemass"] = k["stm"]
  M = k["M"]
  if m.nv:
    if np.min(np.diag(M)) < MINVAL or np.linalg.cond(M) > 1e14:
      # MuJoCo's compiler error for the same model (mj_setConst)
      raise ValueError("mass and inertia of moving bodies must be larger than mjMINVAL")
    Minv = np.linalg.inv(M)
    m.meaninertia = float(np.trace(M) / m.nv)
  else:
    Minv = np.zeros((0, 0))
    m.meaninertia = 1.0
  dinv = np.zeros(m.nv)
  for j in range(m.njnt):
    d = A["jnt_dofadr"][j]
    t = A["jnt_type"][j]
    if t == 0:
      dinv[d:d + 3] = np.mean(np.diag(Minv)[d:d + 3])
      dinv[d + 3:d + 6] = np.mean(np.diag(Minv)[d + 3:d + 6])
    elif t == 1:
      dinv[d:d + 3] = np.mean(np.diag(Minv)[d:d + 3])
    else:
      dinv[d] = Minv[d, d]
  A["dof_invweight0"] = dinv
  binv = np.zeros((m.nbody, 2))
  for b in range(1, m.nbody):
    if A["body_weldid"][b] == 0:
      continue
    off = k["subtree_com"][A["body_rootid"][b]]
    p = k["xipos"][b]
    J = np.zeros((6, m.nv))
    for i in range(m.nv):
      if (int(A["dof_bodymask"][i]) >> b) & 1:
        J[:3, i] = k["cdof"][i, 3:] + np.cross(k["cdof"][i, :3], p - off)
        J[3:, i] = k["cdof"][i, :3]
    Amat = J @ Minv @ J.T
    binv[b, 0] = max(np.trace(Amat[:3, :3]) / 3, MINVAL)
    binv[b, 1] = max(np.trace(Amat[3:, 3:]) / 3, MINVAL)
  A["body_invweight0"] = binv
