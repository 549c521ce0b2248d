"""Robot constants for the Unitree G1 (29-DoF) and Go1 scenes.

Mirrors the actuator/collision/keyframe constants of
`src/mjlab/asset_zoo/robots/unitree_g1/g1_constants.py:41-295` and
`src/mjlab/asset_zoo/robots/unitree_go1/go1_constants.py:41-165`: armature is the
two-stage planetary reflected inertia, stiffness = armature * (2*pi*10Hz)^2,
damping = 2 * 2.0 * armature * (2*pi*10Hz), effort limits from the motor specs.
"""

from __future__ import annotations

import json
import os

from .compiler.model import CollisionEdit, PositionActuatorGroup

ROBOT_DIR = os.path.join(os.path.dirname(__file__), "assets", "robots")

_NATURAL_FREQ = 10 * 2.0 * 3.1415926535
_DAMPING_RATIO = 2.0


def two_stage_planetary(rotor, gear):
  """Reflected inertia of a two-stage planetary gearbox (`utils/actuator.py:25-34`)."""
  assert gear[0] == 1
  return rotor[0] * (gear[1] * gear[2]) ** 2 + rotor[1] * gear[2] ** 2 + rotor[2]


def _pd(armature):
  return (armature * _NATURAL_FREQ ** 2,
          2.0 * _DAMPING_RATIO * armature * _NATURAL_FREQ)


ARMATURE_5020 = two_stage_planetary((0.139e-4, 0.017e-4, 0.169e-4), (1, 1 + 46 / 18, 1 + 56 / 16))
ARMATURE_7520_14 = two_stage_planetary((0.489e-4, 0.098e-4, 0.533e-4), (1, 4.5, 1 + 48 / 22))
ARMATURE_7520_22 = two_stage_planetary((0.489e-4, 0.109e-4, 0.738e-4), (1, 4.5, 5))
ARMATURE_4010 = two_stage_planetary((0.068e-4, 0.0, 0.0), (1, 5, 5))


def g1_actuators() -> tuple[PositionActuatorGroup, ...]:
  k5020, d5020 = _pd(ARMATURE_5020)
  k14, d14 = _pd(ARMATURE_7520_14)
  k22, d22 = _pd(ARMATURE_7520_22)
  k4010, d4010 = _pd(ARMATURE_4010)
  return (
    PositionActuatorGroup((".*_elbow_joint", ".*_shoulder_pitch_joint", ".*_shoulder_roll_joint",
                           ".*_shoulder_yaw_joint", ".*_wrist_roll_joint"),
                          k5020, d5020, 25.0, ARMATURE_5020),
    PositionActuatorGroup((".*_hip_pitch_joint", ".*_hip_yaw_joint", "waist_yaw_joint"),
                          k14, d14, 88.0, ARMATURE_7520_14),
    PositionActuatorGroup((".*_hip_roll_joint", ".*_knee_joint"), k22, d22, 139.0,
                          ARMATURE_7520_22),
    PositionActuatorGroup((".*_wrist_pitch_joint", ".*_wrist_yaw_joint"), k4010, d4010, 5.0,
                          ARMATURE_4010),
    PositionActuatorGroup(("waist_pitch_joint", "waist_roll_joint"), 2 * k5020, 2 * d5020, 50.0,
                          2 * ARMATURE_5020),
    PositionActuatorGroup((".*_ankle_pitch_joint", ".*_ankle_roll_joint"), 2 * k5020, 2 * d5020,
                          50.0, 2 * ARMATURE_5020),
  )


G1_FULL_COLLISION = CollisionEdit(
  geom_names_expr=(".*_collision",),
  condim={r"^(left|right)_foot[1-7]_collision$": 3, ".*_collision": 1},
  priority={r"^(left|right)_foot[1-7]_collision$": 1},
  friction={r"^(left|right)_foot[1-7]_collision$": (0.6,)},
)

G1_KNEES_BENT = dict(
  pos=(0.0, 0.0, 0.76),
  joint_pos={
    ".*_hip_pitch_joint": -0.312, ".*_knee_joint": 0.669, ".*_ankle_pitch_joint": -0.363,
    ".*_elbow_joint": 0.6, "left_shoulder_roll_joint": 0.2, "left_shoulder_pitch_joint": 0.2,
    "right_shoulder_roll_joint": -0.2, "right_shoulder_pitch_joint": 0.2,
  },
)

G1_HOME = dict(
  pos=(0.0, 0.0, 0.783675),
  joint_pos={
    ".*_hip_pitch_joint": -0.1, ".*_knee_joint": 0.3, ".*_ankle_pitch_joint": -0.2,
    ".*_shoulder_pitch_joint": 0.2, ".*_elbow_joint": 1.28, "left_shoulder_roll_joint": 0.2,
    "right_shoulder_roll_joint": -0.2,
  },
)

# `tasks/jump/config/g1/env_cfgs.py:19-46` (first-match pattern resolution, so the
# ".*_shoulder_roll_joint" entry wins over the later left/right ones, as resolve_expr does)
G1_JUMP_CROUCH = dict(
  pos=(0.0, 0.0, 0.55),
  joint_pos={
    ".*_hip_pitch_joint": -0.6, ".*_knee_joint": 1.2, ".*_ankle_pitch_joint": -0.6,
    ".*_hip_roll_joint": 0.0, ".*_hip_yaw_joint": 0.0, ".*_ankle_roll_joint": 0.0,
    "waist_yaw_joint": 0.0, "waist_roll_joint": 0.0, "waist_pitch_joint": 0.15,
    ".*_shoulder_pitch_joint": -0.5, ".*_shoulder_roll_joint": 0.0,
    "left_shoulder_roll_joint": 0.3, "right_shoulder_roll_joint": -0.3,
    ".*_shoulder_yaw_joint": 0.0, ".*_elbow_joint": 0.8, ".*_wrist_pitch_joint": 0.0,
    ".*_wrist_roll_joint": 0.0, ".*_wrist_yaw_joint": 0.0,
  },
)

GO1_ROTOR_INERTIA = 0.000111842
GO1_HIP_ARMATURE = GO1_ROTOR_INERTIA * 6 ** 2
GO1_KNEE_ARMATURE = GO1_ROTOR_INERTIA * 9 ** 2


def go1_actuators() -> tuple[PositionActuatorGroup, ...]:
  kh, dh = _pd(GO1_HIP_ARMATURE)
  kk, dk = _pd(GO1_KNEE_ARMATURE)
  return (
    PositionActuatorGroup((".*_hip_joint", ".*_thigh_joint"), kh, dh, 23.7, GO1_HIP_ARMATURE),
    PositionActuatorGroup((".*_calf_joint",), kk, dk, 35.55, GO1_KNEE_ARMATURE),
  )


_GO1_FOOT = "^[FR][LR]_foot_collision$"
GO1_FULL_COLLISION = CollisionEdit(
  geom_names_expr=(".*_collision",),
  condim={_GO1_FOOT: 3, ".*_collision": 1},
  priority={_GO1_FOOT: 1},
  friction={_GO1_FOOT: (0.6,)},
  solimp={_GO1_FOOT: (0.9, 0.95, 0.023)},
  contype=1,
  conaffinity=0,
)

GO1_INIT = dict(
  pos=(0.0, 0.0, 0.278),
  joint_pos={".*thigh_joint": 0.9, ".*calf_joint": -1.8, ".*R_hip_joint": 0.1,
             ".*L_hip_joint": -0.1},
)


def action_scale(groups) -> dict[str, float]:
  """`G1_ACTION_SCALE` / `GO1_ACTION_SCALE`: 0.25 * effort / stiffness per pattern."""
  out = {}
  for g in groups:
    for n in g.joint_names_expr:
      out[n] = 0.25 * g.effort_limit / g.stiffness
  return out


# --------------------------------------------------------------------------- robot entities
def robot_spec(name: str):
  """The robot's MJCF as parsed data (`assets/robots/<name>.json`, written by
  scripts/build_assets.py from the reference's `asset_zoo/robots/*/xmls/*.xml`; visual meshes
  are frames only) as a fresh `Spec` -- the `spec_fn` of the robot's EntityCfg
  (`g1_constants.py:33-36` `get_spec`)."""
  from .compiler.mjcf import xmodel_from_dict
  from .spec import Spec
  path = os.path.join(ROBOT_DIR, f"{name}.json")
  if not os.path.exists(path):
    raise FileNotFoundError(f"robot description {path} missing; run scripts/build_assets.py")
  with open(path) as fh:
    return Spec(xmodel_from_dict(json.load(fh)))


def get_g1_spec():
  return robot_spec("unitree_g1")


def get_go1_spec():
  return robot_spec("unitree_go1")


def _init_state(d):
  from .entity import InitialStateCfg
  return InitialStateCfg(pos=tuple(d["pos"]), joint_pos=dict(d["joint_pos"]),
                         joint_vel={".*": 0.0})


def get_g1_robot_cfg(init: dict | None = None):
  """`g1_constants.py:260-285` (`get_g1_robot_cfg`): knees-bent init, full collision, the six
  builtin position-actuator groups, soft joint limits at 90 %."""
  from .entity import EntityArticulationInfoCfg, EntityCfg
  return EntityCfg(init_state=_init_state(init or G1_KNEES_BENT), spec_fn=get_g1_spec,
                   collisions=(G1_FULL_COLLISION,),
                   articulation=EntityArticulationInfoCfg(actuators=g1_actuators(),
                                                          soft_joint_pos_limit_factor=0.9))


def get_go1_robot_cfg():
  """`go1_constants.py:140-160` (`get_go1_robot_cfg`)."""
  from .entity import EntityArticulationInfoCfg, EntityCfg
  return EntityCfg(init_state=_init_state(GO1_INIT), spec_fn=get_go1_spec,
                   collisions=(GO1_FULL_COLLISION,),
                   articulation=EntityArticulationInfoCfg(actuators=go1_actuators(),
                                                          soft_joint_pos_limit_factor=0.9))
