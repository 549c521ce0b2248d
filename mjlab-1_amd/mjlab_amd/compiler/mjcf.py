"""MJCF-subset parser: XML -> a tree of plain Python bodies with resolved defaults.

This is the setup path that the reference delegates to MuJoCo's `MjSpec.from_file`
(`src/mjlab/asset_zoo/robots/unitree_g1/g1_constants.py:33-36`,
`src/mjlab/scene/scene.py:38-48`).  Only the subset the mjlab robots use is
supported: nested `<default>` classes and `childclass`, bodies with
`<inertial>`, free/hinge/slide/ball joints, primitive geoms (plane, sphere,
capsule, box, hfield placeholder) with `fromto`, sites, `<contact><exclude>` and
the sensors gyro / velocimeter / accelerometer / subtreeangmom.

Visual mesh geoms are kept as frames (they have no physics effect) and their
mesh files are never opened, so a missing STL (the Go1 `trunk.stl`,
SURVEY.md section 0) is tolerated.  Mesh geoms are NOT re-centred at the mesh
inertial frame as MuJoCo does; their `geom_xpos` is the frame as written.
"""

from __future__ import annotations

import copy
import math
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

GEOM_TYPES = {"plane": 0, "hfield": 1, "sphere": 2, "capsule": 3, "ellipsoid": 4,
              "cylinder": 5, "box": 6, "mesh": 7}
JOINT_TYPES = {"free": 0, "ball": 1, "slide": 2, "hinge": 3}

_GEOM_DEFAULTS = dict(
  type="sphere", size=(0.0, 0.0, 0.0), contype=1, conaffinity=1, condim=3, priority=0,
  friction=(1.0, 0.005, 0.0001), solmix=1.0, solref=(0.02, 1.0),
  solimp=(0.9, 0.95, 0.001, 0.5, 2.0), margin=0.0, gap=0.0, group=0, density=1000.0,
  pos=(0.0, 0.0, 0.0), quat=(1.0, 0.0, 0.0, 0.0), mesh=None, rgba=(0.5, 0.5, 0.5, 1.0),
)
_JOINT_DEFAULTS = dict(
  type="hinge", axis=(0.0, 0.0, 1.0), pos=(0.0, 0.0, 0.0), range=(0.0, 0.0), limited="auto",
  solreflimit=(0.02, 1.0), solimplimit=(0.9, 0.95, 0.001, 0.5, 2.0), margin=0.0,
  stiffness=0.0, damping=0.0, armature=0.0, frictionloss=0.0, springref=0.0, ref=0.0,
)
_SITE_DEFAULTS = dict(pos=(0.0, 0.0, 0.0), quat=(1.0, 0.0, 0.0, 0.0), type="sphere",
                      size=(0.005, 0.005, 0.005))

_FLOAT_VEC = {"size", "friction", "solref", "solimp", "pos", "quat", "axis", "range",
              "solreflimit", "solimplimit", "fromto", "rgba", "diaginertia", "fullinertia",
              "euler", "axisangle", "zaxis", "xyaxes"}
_FLOAT = {"solmix", "margin", "gap", "density", "stiffness", "damping", "armature",
          "frictionloss", "springref", "ref", "mass"}
_INT = {"contype", "conaffinity", "condim", "priority", "group"}


def _parse_attr(name: str, value: str):
  if name in _FLOAT_VEC:
    return tuple(float(x) for x in value.split())
  if name in _FLOAT:
    return float(value)
  if name in _INT:
    return int(value)
  return value


# --------------------------------------------------------------------------- quaternions
def quat_mul(a, b):
  aw, ax, ay, az = a
  bw, bx, by, bz = b
  return np.array([aw * bw - ax * bx - ay * by - az * bz,
                   aw * bx + ax * bw + ay * bz - az * by,
                   aw * by - ax * bz + ay * bw + az * bx,
                   aw * bz + ax * by - ay * bx + az * bw])


def quat_normalize(q):
  q = np.asarray(q, dtype=np.float64)
  n = np.linalg.norm(q)
  return q / n if n > 1e-15 else np.array([1.0, 0.0, 0.0, 0.0])


def quat_to_mat(q):
  w, x, y, z = quat_normalize(q)
  return np.array([
    [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
    [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
    [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def mat_to_quat(m):
  m = np.asarray(m, dtype=np.float64)
  tr = m[0, 0] + m[1, 1] + m[2, 2]
  if tr > 0:
    s = math.sqrt(tr + 1.0) * 2
    q = [0.25 * s, (m[2, 1] - m[1, 2]) / s, (m[0, 2] - m[2, 0]) / s, (m[1, 0] - m[0, 1]) / s]
  elif m[0, 0] > m[1, 1] and m[0, 0] > m[2, 2]:
    s = math.sqrt(1.0 + m[0, 0] - m[1, 1] - m[2, 2]) * 2
    q = [(m[2, 1] - m[1, 2]) / s, 0.25 * s, (m[0, 1] + m[1, 0]) / s, (m[0, 2] + m[2, 0]) / s]
  elif m[1, 1] > m[2, 2]:
    s = math.sqrt(1.0 + m[1, 1] - m[0, 0] - m[2, 2]) * 2
    q = [(m[0, 2] - m[2, 0]) / s, (m[0, 1] + m[1, 0]) / s, 0.25 * s, (m[1, 2] + m[2, 1]) / s]
  else:
    s = math.sqrt(1.0 + m[2, 2] - m[0, 0] - m[1, 1]) * 2
    q = [(m[1, 0] - m[0, 1]) / s, (m[0, 2] + m[2, 0]) / s, (m[1, 2] + m[2, 1]) / s, 0.25 * s]
  q = quat_normalize(q)
  return q if q[0] >= 0 else -q


def axisangle_to_quat(axis, ang):
  axis = np.asarray(axis, dtype=np.float64)
  axis = axis / np.linalg.norm(axis)
  s = math.sin(0.5 * ang)
  return np.array([math.cos(0.5 * ang), axis[0] * s, axis[1] * s, axis[2] * s])


def quat_z2vec(vec):
  """Minimal rotation taking +z onto `vec` (MuJoCo's fromto convention)."""
  v = np.asarray(vec, dtype=np.float64)
  v = v / np.linalg.norm(v)
  axis = np.cross([0.0, 0.0, 1.0], v)
  s = np.linalg.norm(axis)
  if s < 1e-12:
    return np.array([1.0, 0, 0, 0]) if v[2] >= 0 else np.array([0.0, 1.0, 0, 0])
  return axisangle_to_quat(axis / s, math.atan2(s, v[2]))


def euler_to_quat(euler, seq="xyz"):
  q = np.array([1.0, 0, 0, 0])
  for ang, ax in zip(euler, seq):
    axis = {"x": (1, 0, 0), "y": (0, 1, 0), "z": (0, 0, 1)}[ax.lower()]
    r = axisangle_to_quat(axis, ang)
    # lower-case = intrinsic (post-multiply), upper-case = extrinsic (pre-multiply)
    q = quat_mul(q, r) if ax.islower() else quat_mul(r, q)
  return q


# --------------------------------------------------------------------------- tree
@dataclass
class XJoint:
  name: str
  attrs: dict


@dataclass
class XGeom:
  name: str
  attrs: dict


@dataclass
class XSite:
  name: str
  attrs: dict


@dataclass
class XBody:
  name: str
  pos: np.ndarray
  quat: np.ndarray
  inertial: dict | None
  joints: list = field(default_factory=list)
  geoms: list = field(default_factory=list)
  sites: list = field(default_factory=list)
  children: list = field(default_factory=list)
  mocap: bool = False


@dataclass
class XModel:
  """Parsed MJCF: world body tree plus global sections."""
  name: str
  world: XBody
  excludes: list
  sensors: list
  angle_deg: bool
  eulerseq: str
  inertiafromgeom: str = "auto"  # <compiler inertiafromgeom>: "auto" | "true" | "false"


class _Defaults:
  def __init__(self):
    self.classes: dict[str, dict[str, dict]] = {}

  def build(self, elem, parent_cls: dict[str, dict] | None, name: str):
    cls = copy.deepcopy(parent_cls) if parent_cls else {"geom": {}, "joint": {}, "site": {}}
    for child in elem:
      if child.tag in ("geom", "joint", "site"):
        cls[child.tag].update({k: _parse_attr(k, v) for k, v in child.attrib.items()})
    self.classes[name] = cls
    for child in elem:
      if child.tag == "default":
        self.build(child, cls, child.attrib.get("class", name))


def _orientation(attrs: dict, angle_deg: bool, eulerseq: str):
  # Alternative orientation specs win over `quat` (which is always present via defaults).
  if "axisangle" in attrs:
    a = attrs["axisangle"]
    ang = math.radians(a[3]) if angle_deg else a[3]
    return axisangle_to_quat(a[:3], ang)
  if "euler" in attrs:
    e = [math.radians(x) if angle_deg else x for x in attrs["euler"]]
    return euler_to_quat(e, eulerseq)
  if "zaxis" in attrs:
    return quat_z2vec(attrs["zaxis"])
  if "xyaxes" in attrs:
    a = np.asarray(attrs["xyaxes"])
    x = a[:3] / np.linalg.norm(a[:3])
    y = a[3:] - x * np.dot(x, a[3:])
    y /= np.linalg.norm(y)
    return mat_to_quat(np.stack([x, y, np.cross(x, y)], axis=1))
  if "quat" in attrs:
    return quat_normalize(attrs["quat"])
  return np.array([1.0, 0.0, 0.0, 0.0])


def parse_mjcf(path: str) -> XModel:
  return parse_mjcf_string(open(path).read())


def parse_mjcf_string(text: str) -> XModel:
  root = ET.fromstring(text)
  comp = root.find("compiler")
  angle_deg = True
  eulerseq = "xyz"
  inertiafromgeom = "auto"
  if comp is not None:
    angle_deg = comp.attrib.get("angle", "degree") != "radian"
    eulerseq = comp.attrib.get("eulerseq", "xyz")
    inertiafromgeom = comp.attrib.get("inertiafromgeom", "auto")
  defaults = _Defaults()
  dflt = root.find("default")
  if dflt is not None:
    defaults.build(dflt, None, dflt.attrib.get("class", "main"))
  if "main" not in defaults.classes:
    defaults.classes["main"] = {"geom": {}, "joint": {}, "site": {}}

  def resolve(tag, elem, childclass):
    cls_name = elem.attrib.get("class", childclass)
    base = {"geom": _GEOM_DEFAULTS, "joint": _JOINT_DEFAULTS, "site": _SITE_DEFAULTS}[tag]
    attrs = dict(base)
    attrs.update(defaults.classes.get("main", {}).get(tag, {}))
    if cls_name:
      attrs.update(defaults.classes[cls_name][tag])
    attrs.update({k: _parse_attr(k, v) for k, v in elem.attrib.items() if k != "class"})
    return attrs

  def parse_body(elem, childclass):
    childclass = elem.attrib.get("childclass", childclass)
    b = XBody(
      name=elem.attrib.get("name", ""),
      pos=np.array(_parse_attr("pos", elem.attrib.get("pos", "0 0 0"))),
      quat=_orientation({k: _parse_attr(k, v) for k, v in elem.attrib.items()
                         if k in ("quat", "euler", "axisangle", "zaxis", "xyaxes")},
                        angle_deg, eulerseq),
      inertial=None,
      mocap=elem.attrib.get("mocap", "false") == "true",
    )
    for child in elem:
      if child.tag == "inertial":
        b.inertial = {k: _parse_attr(k, v) for k, v in child.attrib.items()}
      elif child.tag == "freejoint":
        b.joints.append(XJoint(child.attrib.get("name", ""), dict(_JOINT_DEFAULTS, type="free")))
      elif child.tag == "joint":
        b.joints.append(XJoint(child.attrib.get("name", ""), resolve("joint", child, childclass)))
      elif child.tag == "geom":
        b.geoms.append(XGeom(child.attrib.get("name", ""), resolve("geom", child, childclass)))
      elif child.tag == "site":
        b.sites.append(XSite(child.attrib.get("name", ""), resolve("site", child, childclass)))
      elif child.tag == "body":
        b.children.append(parse_body(child, childclass))
    return b

  wb = root.find("worldbody")
  world = XBody("world", np.zeros(3), np.array([1.0, 0, 0, 0]), None)
  if wb is not None:
    world_children = parse_body(wb, None)
    world.geoms, world.sites, world.children = (world_children.geoms, world_children.sites,
                                                world_children.children)
  excludes = []
  contact = root.find("contact")
  if contact is not None:
    for ex in contact.findall("exclude"):
      excludes.append((ex.attrib["body1"], ex.attrib["body2"]))
  sensors = []
  sens = root.find("sensor")
  if sens is not None:
    for s in sens:
      sensors.append((s.tag, dict(s.attrib)))
  return XModel(root.attrib.get("model", ""), world, excludes, sensors, angle_deg, eulerseq,
                inertiafromgeom)


def geom_frame(attrs: dict, angle_deg: bool, eulerseq: str):
  """Return (pos, quat, size) of a geom, resolving `fromto` for capsules/cylinders/boxes."""
  size = list(attrs["size"]) + [0.0] * (3 - len(attrs["size"]))
  if "fromto" in attrs:
    ft = np.asarray(attrs["fromto"], dtype=np.float64)
    a, b = ft[:3], ft[3:]
    pos = 0.5 * (a + b)
    quat = quat_z2vec(b - a)
    half = 0.5 * float(np.linalg.norm(b - a))
    if attrs["type"] in ("capsule", "cylinder"):
      size[1] = half
    elif attrs["type"] == "box":
      size[2] = half
    return pos, quat, np.array(size[:3])
  pos = np.asarray(attrs["pos"], dtype=np.float64)
  quat = _orientation(attrs, angle_deg, eulerseq)
  return pos, quat, np.array(size[:3], dtype=np.float64)


# --------------------------------------------------------------------------- serialisation
def _attrs_out(a: dict) -> dict:
  return {k: (list(v) if isinstance(v, (tuple, np.ndarray)) else v) for k, v in a.items()}


def _attrs_in(a: dict) -> dict:
  return {k: (tuple(v) if isinstance(v, list) else v) for k, v in a.items()}


def xmodel_to_dict(xm: XModel) -> dict:
  """The parsed MJCF tree as plain JSON-able data (defaults already resolved), so a robot
  description travels as data: `xmodel_from_dict` rebuilds the identical tree."""
  def body(b: XBody) -> dict:
    return dict(name=b.name, pos=[float(x) for x in b.pos], quat=[float(x) for x in b.quat],
                inertial=_attrs_out(b.inertial) if b.inertial is not None else None,
                mocap=bool(b.mocap),
                joints=[dict(name=j.name, attrs=_attrs_out(j.attrs)) for j in b.joints],
                geoms=[dict(name=g.name, attrs=_attrs_out(g.attrs)) for g in b.geoms],
                sites=[dict(name=s.name, attrs=_attrs_out(s.attrs)) for s in b.sites],
                children=[body(c) for c in b.children])
  return dict(name=xm.name, world=body(xm.world), excludes=[list(e) for e in xm.excludes],
              sensors=[[t, dict(a)] for t, a in xm.sensors], angle_deg=xm.angle_deg,
              eulerseq=xm.eulerseq, inertiafromgeom=xm.inertiafromgeom)


def xmodel_from_dict(d: dict) -> XModel:
  def body(b: dict) -> XBody:
    return XBody(name=b["name"], pos=np.array(b["pos"], float), quat=np.array(b["quat"], float),
                 inertial=_attrs_in(b["inertial"]) if b["inertial"] is not None else None,
                 joints=[XJoint(j["name"], _attrs_in(j["attrs"])) for j in b["joints"]],
                 geoms=[XGeom(g["name"], _attrs_in(g["attrs"])) for g in b["geoms"]],
                 sites=[XSite(s["name"], _attrs_in(s["attrs"])) for s in b["sites"]],
                 children=[body(c) for c in b["children"]], mocap=bool(b["mocap"]))
  return XModel(d["name"], body(d["world"]), [tuple(e) for e in d["excludes"]],
                [(t, dict(a)) for t, a in d["sensors"]], bool(d["angle_deg"]), d["eulerseq"],
                d.get("inertiafromgeom", "auto"))
