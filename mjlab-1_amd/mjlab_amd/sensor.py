"""Contact sensor configuration (`src/mjlab/sensor/contact_sensor.py:47-97,159-197,367-533`).

A `ContactSensorCfg` names a primary match (geoms, bodies or subtrees, by regex within an
entity, with excludes) and an optional secondary; at scene construction it expands into one
mjSENS_CONTACT sensor per primary x field, named `<name>_<primary>_<field>`, which the
compiler turns into the engine's per-sensor geom masks.  The runtime view over those
sensors (`ContactData`, air time) is `scene.ContactSensor`.
"""

from __future__ import annotations

import re
from dataclasses import dataclass
from typing import Literal

from .compiler.model import BuiltinSensorSpec, ContactSensorSpec


@dataclass
class ContactMatch:
  """`contact_sensor.py:47-60`: mode "geom" | "body" | "subtree"; pattern a regex or tuple of
  regexes expanded within `entity` (None: a literal MuJoCo name); exclude: exact names or
  regexes removed from the matches."""
  mode: Literal["geom", "body", "subtree"]
  pattern: str | tuple[str, ...]
  entity: str | None = None
  exclude: tuple[str, ...] = ()


@dataclass
class ContactSensorCfg:
  """`contact_sensor.py:63-96`."""
  name: str
  primary: ContactMatch
  secondary: ContactMatch | None = None
  fields: tuple[str, ...] = ("found", "force")
  reduce: Literal["none", "mindist", "maxforce", "netforce"] = "maxforce"
  num_slots: int = 1
  secondary_policy: Literal["first", "any", "error"] = "first"
  track_air_time: bool = False
  global_frame: bool = False
  debug: bool = False

  def expand(self, entities: dict) -> ContactSensorSpec:
    """Pattern expansion (`contact_sensor.py:159-197,367-440`) against the scene's
    `EntityBuild`s; names come out entity-prefixed."""
    if self.global_frame and self.reduce != "netforce":
      if "normal" not in self.fields or "tangent" not in self.fields:
        raise ValueError(f"Sensor '{self.name}': global_frame=True requires 'normal' and 'tangent' "
                         "in fields (needed to build rotation matrix)")
      raise NotImplementedError(f"Sensor '{self.name}': global_frame with reduce={self.reduce!r}")
    prim = self._primary_names(entities, self.primary)
    pref = f"{self.primary.entity}/" if self.primary.entity else ""
    sec_name, sec_mode = None, None
    if self.secondary is not None and self.secondary_policy != "any":
      sec = self._secondary_name(entities, self.secondary)
      sref = f"{self.secondary.entity}/" if self.secondary.entity else ""
      sec_name, sec_mode = sref + sec, self.secondary.mode
    return ContactSensorSpec(name=self.name, primary_mode=self.primary.mode,
                             primary_names=[pref + n for n in prim], secondary_mode=sec_mode,
                             secondary_name=sec_name, fields=tuple(self.fields),
                             reduce=self.reduce, num_slots=int(self.num_slots))

  @staticmethod
  def _primary_names(entities: dict, match: ContactMatch) -> list[str]:
    if match.entity in (None, ""):
      return [match.pattern] if isinstance(match.pattern, str) else list(match.pattern)
    if match.entity not in entities:
      raise ValueError(f"Primary entity '{match.entity}' not found. Available: {list(entities.keys())}")
    ent = entities[match.entity]
    patterns = [match.pattern] if isinstance(match.pattern, str) else list(match.pattern)
    if match.mode == "geom":
      _, names = ent.find_geoms(patterns)
    elif match.mode in ("body", "subtree"):
      _, names = ent.find_bodies(patterns)
      if not names and match.mode == "subtree":
        raise ValueError(f"Primary subtree pattern '{match.pattern}' matched no bodies in '{match.entity}'")
    else:
      raise ValueError("Primary mode must be one of {'geom','body','subtree'}")
    exact = {e for e in match.exclude if not any(c in e for c in r".*+?[]{}()\|^$")}
    regex = [re.compile(e) for e in match.exclude if e not in exact]
    names = [n for n in names if n not in exact and not any(rx.search(n) for rx in regex)]
    if not names:
      raise ValueError(f"Primary pattern '{match.pattern}' (after excludes) matched no names in "
                       f"'{match.entity}'")
    return names

  def _secondary_name(self, entities: dict, match: ContactMatch) -> str:
    if isinstance(match.pattern, tuple):
      raise ValueError("Secondary must specify a single name (string).")
    if match.entity in (None, ""):
      if match.mode not in {"geom", "body", "subtree"}:
        raise ValueError("Secondary mode must be one of {'geom','body','subtree'}")
      return match.pattern
    if match.entity not in entities:
      raise ValueError(f"Secondary entity '{match.entity}' not found. Available: {list(entities.keys())}")
    if match.mode == "subtree":
      return match.pattern
    ent = entities[match.entity]
    if match.mode == "geom":
      _, names = ent.find_geoms([match.pattern])
    elif match.mode == "body":
      _, names = ent.find_bodies([match.pattern])
    else:
      raise ValueError("Secondary mode must be one of {'geom','body','subtree'}")
    if not names:  # contact_sensor.py:459-462
      raise ValueError(f"Secondary pattern '{match.pattern}' matched nothing in '{match.entity}'")
    if len(names) == 1 or self.secondary_policy == "first":
      return names[0]
    raise ValueError(f"Secondary pattern '{match.pattern}' matched multiple: {names}. "
                     "Be explicit or set secondary_policy='first' or 'any'.")


# ----------------------------------------------------------------------------- builtin sensors
_REQUIRES_SITE = {"accelerometer", "velocimeter", "gyro", "force", "torque", "magnetometer",
                  "rangefinder"}
_REQUIRES_FRAME = {"framepos", "framequat", "framexaxis", "frameyaxis", "framezaxis",
                   "framelinvel", "frameangvel", "framelinacc", "frameangacc"}
_REQUIRES_BODY = {"subtreecom", "subtreelinvel", "subtreeangmom"}
_REQUIRES_OBJ = {"jointpos": "joint", "jointvel": "joint", "jointlimitpos": "joint",
                 "jointlimitvel": "joint", "jointlimitfrc": "joint", "jointactuatorfrc": "joint",
                 "tendonpos": "tendon", "tendonvel": "tendon", "tendonactuatorfrc": "tendon",
                 "actuatorpos": "actuator", "actuatorvel": "actuator", "actuatorfrc": "actuator"}
_FRAME_TYPES = {"body", "xbody", "geom", "site", "camera"}
# what the engine evaluates: sensor type -> the object types it takes
_ENGINE = {"accelerometer": {"site"}, "velocimeter": {"site"}, "gyro": {"site"},
           "framepos": {"site", "xbody"}, "framequat": {"site", "xbody"},
           "jointpos": {"joint"}, "jointvel": {"joint"}, "subtreeangmom": {"body"}}


@dataclass
class ObjRef:
  """`builtin_sensor.py:171-189`."""
  type: Literal["body", "xbody", "joint", "geom", "site", "actuator", "tendon", "camera"]
  name: str
  entity: str | None = None

  def prefixed_name(self) -> str:
    return f"{self.entity}/{self.name}" if self.entity else self.name


@dataclass
class BuiltinSensorCfg:
  """`builtin_sensor.py:195-250`: a MuJoCo builtin sensor added by the scene config; the
  name is entity-prefixed when `obj` names an entity.  The object-type rules are checked at
  construction as the reference does; types the engine does not evaluate raise at scene
  construction (`expand`)."""
  name: str
  sensor_type: str
  obj: ObjRef | None = None
  ref: ObjRef | None = None
  cutoff: float = 0.0

  def __post_init__(self) -> None:
    if self.obj is not None and self.obj.entity is not None:
      self.name = f"{self.obj.entity}/{self.name}"
    st = self.sensor_type
    if st in _REQUIRES_SITE:
      if self.obj is None:
        raise ValueError(f"Sensor type '{st}' requires obj with type='site'")
      if self.obj.type != "site":
        raise ValueError(f"Sensor type '{st}' requires obj.type='site', got '{self.obj.type}'")
    elif st in _REQUIRES_FRAME:
      if self.obj is None:
        raise ValueError(f"Sensor type '{st}' requires obj with spatial frame")
      if self.obj.type not in _FRAME_TYPES:
        raise ValueError(f"Sensor type '{st}' requires obj.type in {_FRAME_TYPES}, got '{self.obj.type}'")
    elif st in _REQUIRES_BODY:
      if self.obj is None:
        raise ValueError(f"Sensor type '{st}' requires obj with type='body'")
      if self.obj.type != "body":
        raise ValueError(f"Sensor type '{st}' requires obj.type='body', got '{self.obj.type}'")
    elif st in _REQUIRES_OBJ:
      req = _REQUIRES_OBJ[st]
      if self.obj is None:
        raise ValueError(f"Sensor type '{st}' requires obj with type='{req}'")
      if self.obj.type != req:
        raise ValueError(f"Sensor type '{st}' requires obj.type='{req}', got '{self.obj.type}'")
    if self.ref is not None and st not in _REQUIRES_FRAME:
      raise ValueError(f"Sensor type '{st}' does not support ref specification")

  def expand(self, entities: dict) -> BuiltinSensorSpec:
    del entities
    st, obj = self.sensor_type, self.obj
    if st not in _ENGINE or obj is None or obj.type not in _ENGINE[st]:
      raise NotImplementedError(f"sensor '{self.name}': {st} on a {obj.type if obj else None} "
                                f"(the engine evaluates {_ENGINE})")
    if self.ref is not None or self.cutoff > 0:
      raise NotImplementedError(f"sensor '{self.name}': ref frames and cutoff")
    key = {"site": "site", "xbody": "body", "body": "body", "joint": "joint"}[obj.type]
    return BuiltinSensorSpec(st, {key: obj.prefixed_name()}, self.name)
