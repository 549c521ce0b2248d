"""Entity configuration: what one robot or object contributes to a scene.

Restates `src/mjlab/entity/entity.py:52-207`: an `EntityCfg` holds a spec factory
(`spec_fn`, here returning this build's `mjlab_amd.spec.Spec`), the initial state that
becomes the entity's part of the scene keyframe, the articulation (builtin actuator groups,
soft joint-limit factor) and the collision edits.  `EntityBuild` is the construction-time
half of the reference's `Entity.__init__` (spec built, fixed base wrapped in a mocap body,
names resolved); the runtime half (index tensors, `EntityData`) is `scene.Entity`, bound
after the scene is compiled.
"""

from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Callable

import numpy as np

from .compiler.model import (ActuatorSpec, CollisionEdit, EntitySpec, MotorActuatorGroup,
                             PositionActuatorGroup, VelocityActuatorGroup)
from .spec import Spec, auto_wrap_fixed_base_mocap, mjtJoint

# the reference's builtin actuator cfgs (`actuator/builtin_actuator.py:27-147`) and
# CollisionCfg (`utils/spec_config.py:137-238`): same fields
BuiltinPositionActuatorCfg = PositionActuatorGroup
BuiltinMotorActuatorCfg = MotorActuatorGroup
BuiltinVelocityActuatorCfg = VelocityActuatorGroup
CollisionCfg = CollisionEdit


@dataclass
class InitialStateCfg:
  """`entity.py:55-65`: root pose / velocity and joint positions by regex (first match)."""
  pos: tuple = (0.0, 0.0, 0.0)
  rot: tuple = (1.0, 0.0, 0.0, 0.0)
  lin_vel: tuple = (0.0, 0.0, 0.0)
  ang_vel: tuple = (0.0, 0.0, 0.0)
  joint_pos: dict | None = field(default_factory=lambda: {".*": 0.0})
  joint_vel: dict = field(default_factory=lambda: {".*": 0.0})


@dataclass
class EntityArticulationInfoCfg:
  """`entity.py:91-94`."""
  actuators: tuple = ()
  soft_joint_pos_limit_factor: float = 1.0


@dataclass
class EntityCfg:
  """`entity.py:52-88` (lights / cameras / textures / materials are visual: not modelled)."""
  InitialStateCfg = InitialStateCfg
  init_state: InitialStateCfg = field(default_factory=InitialStateCfg)
  spec_fn: Callable[[], Spec] = field(default_factory=lambda: Spec)
  articulation: EntityArticulationInfoCfg | None = None
  collisions: tuple = ()
  debug_vis: bool = False


def resolve_expr(exprs: dict, names, default: float = 0.0) -> list[float]:
  """`utils/string.py:5-38` (resolve_expr): per name the first pattern that re.match-es."""
  out = []
  for n in names:
    v = default
    for pat, val in exprs.items():
      if re.match(pat, n):
        v = val
        break
    out.append(float(v))
  return out


class EntityBuild:
  """One entity at scene construction (`entity.py:127-207`): the spec (fixed-base entities
  wrapped in a mocap body, `utils/spec.py:9-51`), its element names in MuJoCo order, and the
  `EntitySpec` the scene compiler takes."""

  def __init__(self, name: str, cfg: EntityCfg):
    self.name = name
    self.cfg = cfg
    self.spec = auto_wrap_fixed_base_mocap(cfg.spec_fn)()
    joints = self.spec.joints
    self.free_joint = joints[0] if joints and joints[0].type == mjtJoint.mjJNT_FREE else None
    self.is_fixed_base = self.free_joint is None
    self.body_names = tuple(b.name for b in self.spec.bodies[1:])
    self.geom_names = tuple(g.name for g in self.spec.geoms)
    self.site_names = tuple(s.name for s in self.spec.sites)
    self.joint_names = tuple(j.name for j in joints if j.type != mjtJoint.mjJNT_FREE)

  # name resolution within the entity (`lab_api/string.py:227` resolve_matching_names)
  def _find(self, keys, names):
    from .managers import resolve_matching_names
    return resolve_matching_names(keys, names, False)

  def find_bodies(self, keys):
    return self._find(keys, self.body_names)

  def find_geoms(self, keys):
    return self._find(keys, self.geom_names)

  def find_sites(self, keys):
    return self._find(keys, self.site_names)

  def find_joints(self, keys):
    return self._find(keys, self.joint_names)

  def entity_spec(self) -> EntitySpec:
    """The compiler's view: the XML tree, collision edits, actuators (the spec's own, then
    the articulation's groups in cfg order, `entity.py:155-168`) and the initial state."""
    cfg, init = self.cfg, self.cfg.init_state
    acts = [a.to_actuator_spec() for a in self.spec.actuators]
    if cfg.articulation is not None:
      for grp in cfg.articulation.actuators:
        if not isinstance(grp, (PositionActuatorGroup, MotorActuatorGroup, VelocityActuatorGroup,
                                ActuatorSpec)):
          raise TypeError(f"entity '{self.name}': unsupported actuator cfg {type(grp).__name__}")
        acts.append(grp)
    key_qpos = None
    if init.joint_pos is None:
      # `entity.py:171-182`: keep the model's own keyframe
      if not self.spec.keys:
        raise ValueError("joint_pos=None requires the model to have a keyframe, but none exists.")
      key_qpos = np.asarray(self.spec.keys[0].qpos, float)
    xml = self.spec._xml
    if self.is_fixed_base:
      # `entity.py:205-207`: a fixed base is placed by moving its root body
      roots = xml.world.children
      if roots:
        roots[0].pos = np.asarray(init.pos, float)
        roots[0].quat = np.asarray(init.rot, float)
    return EntitySpec(self.name, xml, collisions=tuple(cfg.collisions), actuators=tuple(acts),
                      init_pos=tuple(init.pos), init_rot=tuple(init.rot),
                      init_joint_pos=dict(init.joint_pos) if init.joint_pos is not None else None,
                      key_qpos=key_qpos)
