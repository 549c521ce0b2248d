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

from .compiler.model import ContactSensorSpec


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
    if len(names) == 1 or self.secondary_policy == "first":
      return names[0]
    raise ValueError(f"Secondary pattern '{match.pattern}' matched multiple: {names}. "
                     "Be explicit or set secondary_policy='first' or 'any'.")
