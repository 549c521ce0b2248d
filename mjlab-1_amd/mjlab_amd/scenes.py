"""Compiled task scenes for the hot path: velocity G1 / Go1, tracking G1, jump G1.

Each builder reproduces the reference scene assembly for one task id
(`src/mjlab/tasks/velocity/config/g1/env_cfgs.py:20-56`,
`src/mjlab/tasks/velocity/config/go1/env_cfgs.py:15-49`,
`src/mjlab/tasks/tracking/config/g1/env_cfgs.py`, `src/mjlab/tasks/jump/config/g1/env_cfgs.py`)
from the robot MJCF.  Because the reference's MJCF files do not travel to the GPU
box, `scripts/build_assets.py` compiles each scene here and stores the numeric
model as `mjlab_amd/assets/<scene>.npz`; `load_scene()` reads that file.
"""

from __future__ import annotations

import json
import os
import re

import numpy as np

from . import asset_zoo as az
from .compiler.mjcf import parse_mjcf
from .compiler.model import ContactSensorSpec, EntitySpec, Model, compile_scene

ASSET_DIR = os.path.join(os.path.dirname(__file__), "assets")

# Simulation options of the velocity task (`tasks/velocity/velocity_env_cfg.py:343-351`).
VELOCITY_SIM = dict(timestep=0.005, iterations=10, ls_iterations=20)
# Jump task: dt 0.002 (`tasks/jump/jump_env_cfg.py:324-352`).
JUMP_SIM = dict(timestep=0.002, iterations=10, ls_iterations=20)


def _g1_entity(xml_path, init=az.G1_KNEES_BENT):
  return EntitySpec("robot", parse_mjcf(xml_path), collisions=(az.G1_FULL_COLLISION,),
                    actuators=az.g1_actuators(), init_pos=init["pos"],
                    init_joint_pos=init["joint_pos"])


def _g1_contact_sensors(self_collision=True):
  out = [ContactSensorSpec(
    name="feet_ground_contact", primary_mode="subtree",
    primary_names=["robot/left_ankle_roll_link", "robot/right_ankle_roll_link"],
    secondary_mode="body", secondary_name="terrain", fields=("found", "force"),
    reduce="netforce", num_slots=1)]
  if self_collision:
    out.append(ContactSensorSpec(
      name="self_collision", primary_mode="subtree", primary_names=["robot/pelvis"],
      secondary_mode="subtree", secondary_name="robot/pelvis", fields=("found",),
      reduce="none", num_slots=1))
  return out


def build_g1_velocity(xml_path: str) -> Model:
  return compile_scene([_g1_entity(xml_path)], contact_sensors=_g1_contact_sensors(),
                       **VELOCITY_SIM)


def build_go1_velocity(xml_path: str, terrain: str = "plane", terrain_geoms=None) -> Model:
  ent = EntitySpec("robot", parse_mjcf(xml_path), collisions=(az.GO1_FULL_COLLISION,),
                   actuators=az.go1_actuators(), init_pos=az.GO1_INIT["pos"],
                   init_joint_pos=az.GO1_INIT["joint_pos"])
  feet = [f"robot/{n}_foot_collision" for n in ("FR", "FL", "RR", "RL")]
  tmp = compile_scene([ent], **VELOCITY_SIM)
  nonfoot = [n for n in tmp.names["geom"]
             if n.startswith("robot/") and re.fullmatch(r".*_collision\d*$", n[6:])
             and n not in feet]
  sensors = [
    ContactSensorSpec("feet_ground_contact", "geom", feet, "body", "terrain",
                      ("found", "force"), "netforce", 1),
    ContactSensorSpec("nonfoot_ground_touch", "geom", nonfoot, "body", "terrain",
                      ("found",), "none", 1),
  ]
  return compile_scene([ent], terrain=terrain, terrain_geoms=terrain_geoms, contact_sensors=sensors,
                       **VELOCITY_SIM)


def build_go1_velocity_rough(xml_path: str) -> Model:
  """`Mjlab-Velocity-Rough-Unitree-Go1` (`tasks/velocity/config/go1/env_cfgs.py:15-112`): the
  Go1 velocity scene on the curriculum box-stair grid (as build_g1_velocity_rough); the
  trunk box meets the terrain boxes through the box-box narrowphase."""
  from .terrains import TerrainGenerator, rough_terrains_cfg
  cfg = rough_terrains_cfg(seed=0, curriculum=True)
  geoms, origins = TerrainGenerator(cfg).generate()
  m = build_go1_velocity(xml_path, terrain="generator", terrain_geoms=geoms)
  m.arrays["terrain_origins"] = np.asarray(origins, np.float64)
  m.arrays["terrain_size"] = np.asarray(cfg.size, np.float64)
  return m


def build_g1_tracking(xml_path: str) -> Model:
  """`tasks/tracking/config/g1/env_cfgs.py:22-33`: G1 (knees-bent init) on a plane with
  the self-collision sensor only; sim options of `tracking_env_cfg.py:303-316`."""
  sensors = [s for s in _g1_contact_sensors() if s.name == "self_collision"]
  return compile_scene([_g1_entity(xml_path)], contact_sensors=sensors, **VELOCITY_SIM)


def _g1_jump_sensors():
  """`tasks/jump/config/g1/env_cfgs.py:66-79`: feet vs terrain only."""
  return [s for s in _g1_contact_sensors(self_collision=False)]


def build_g1_jump(xml_path: str) -> Model:
  """`Mjlab-Jump-Flat-Unitree-G1`: crouch keyframe, plane, dt 0.002."""
  return compile_scene([_g1_entity(xml_path, init=az.G1_JUMP_CROUCH)],
                       contact_sensors=_g1_jump_sensors(), **JUMP_SIM)


def build_g1_jump_hfield(xml_path: str) -> Model:
  """Config 5: the jump scene re-terrained onto the seeded 10 x 20 grid of
  heightfield sub-terrains (terrains.hf_rough_terrains_cfg); spawn origins are stored
  with the model (`terrain_origins`, [rows, cols, 3])."""
  from .terrains import TerrainGenerator, hf_rough_terrains_cfg
  cfg = hf_rough_terrains_cfg(seed=0)
  hfields, origins = TerrainGenerator(cfg).generate()
  m = compile_scene([_g1_entity(xml_path, init=az.G1_JUMP_CROUCH)], terrain="hfield",
                    hfields=hfields, contact_sensors=_g1_jump_sensors(), **JUMP_SIM)
  m.arrays["terrain_origins"] = np.asarray(origins, np.float64)
  m.arrays["terrain_size"] = np.asarray(cfg.size, np.float64)
  return m


def build_g1_velocity_rough(xml_path: str) -> Model:
  """`Mjlab-Velocity-Rough-Unitree-G1` (`tasks/velocity/config/g1/env_cfgs.py:20-56`,
  `velocity_env_cfg.py:318-324`): the G1 velocity scene on ROUGH_TERRAINS_CFG in curriculum
  layout -- 80 flat box patches, 120 pyramid / inverted-pyramid stair patches of 25 boxes,
  the 20 m border; 3084 static boxes.  The reference draws the generator seed at random;
  the compiled asset fixes it (seed 0)."""
  from .terrains import TerrainGenerator, rough_terrains_cfg
  cfg = rough_terrains_cfg(seed=0, curriculum=True)
  geoms, origins = TerrainGenerator(cfg).generate()
  m = compile_scene([_g1_entity(xml_path)], terrain="generator", terrain_geoms=geoms,
                    contact_sensors=_g1_contact_sensors(), **VELOCITY_SIM)
  m.arrays["terrain_origins"] = np.asarray(origins, np.float64)
  m.arrays["terrain_size"] = np.asarray(cfg.size, np.float64)
  return m


def _rough_play_cfg():
  """The play-mode terrain of the rough velocity tasks (`tasks/velocity/config/g1/env_cfgs.py:
  131-148`, go1 likewise): curriculum off (random sub-terrain per patch), 5 x 5 patches, 10 m
  border.  The reference draws the generator seed at random; the compiled asset fixes it."""
  from .terrains import rough_terrains_cfg
  return rough_terrains_cfg(seed=0, curriculum=False, num_rows=5, num_cols=5, border_width=10.0)


def build_g1_velocity_rough_play(xml_path: str) -> Model:
  from .terrains import TerrainGenerator
  cfg = _rough_play_cfg()
  geoms, origins = TerrainGenerator(cfg).generate()
  m = compile_scene([_g1_entity(xml_path)], terrain="generator", terrain_geoms=geoms,
                    contact_sensors=_g1_contact_sensors(), **VELOCITY_SIM)
  m.arrays["terrain_origins"] = np.asarray(origins, np.float64)
  m.arrays["terrain_size"] = np.asarray(cfg.size, np.float64)
  return m


def build_go1_velocity_rough_play(xml_path: str) -> Model:
  from .terrains import TerrainGenerator
  cfg = _rough_play_cfg()
  geoms, origins = TerrainGenerator(cfg).generate()
  m = build_go1_velocity(xml_path, terrain="generator", terrain_geoms=geoms)
  m.arrays["terrain_origins"] = np.asarray(origins, np.float64)
  m.arrays["terrain_size"] = np.asarray(cfg.size, np.float64)
  return m


SCENE_BUILDERS = {
  "g1_velocity": ("unitree_g1/xmls/g1.xml", build_g1_velocity),
  "g1_tracking": ("unitree_g1/xmls/g1.xml", build_g1_tracking),
  "g1_jump": ("unitree_g1/xmls/g1.xml", build_g1_jump),
  "g1_jump_hfield": ("unitree_g1/xmls/g1.xml", build_g1_jump_hfield),
  "go1_velocity": ("unitree_go1/xmls/go1.xml", build_go1_velocity),
  "g1_velocity_rough": ("unitree_g1/xmls/g1.xml", build_g1_velocity_rough),
  "go1_velocity_rough": ("unitree_go1/xmls/go1.xml", build_go1_velocity_rough),
  "g1_velocity_rough_play": ("unitree_g1/xmls/g1.xml", build_g1_velocity_rough_play),
  "go1_velocity_rough_play": ("unitree_go1/xmls/go1.xml", build_go1_velocity_rough_play),
}


# ----------------------------------------------------------------------------- npz io
_SCALARS = ("nq", "nv", "nu", "nbody", "njnt", "ngeom", "nsite", "nsensor", "nsensordata",
            "npair", "nhfield", "nhfielddata", "timestep", "iterations", "ls_iterations",
            "tolerance", "ls_tolerance", "impratio", "integrator", "cone", "solver",
            "meaninertia")


def save_model(m: Model, path: str) -> None:
  payload = {f"a_{k}": v for k, v in m.arrays.items()}
  meta = {k: getattr(m, k) for k in _SCALARS}
  meta["gravity"] = list(map(float, m.gravity))
  meta["names"] = m.names
  payload["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
  if os.path.exists(path):  # keep the file (and its zip timestamps) when nothing changed
    with np.load(path, allow_pickle=False) as z:
      if set(z.files) == set(payload) and all(
          z[k].shape == np.asarray(v).shape and np.array_equal(z[k], v) for k, v in payload.items()):
        return
  np.savez_compressed(path, **payload)


def load_model(path: str) -> Model:
  with np.load(path, allow_pickle=False) as z:
    meta = json.loads(bytes(z["meta"]).decode())
    m = Model()
    for k in _SCALARS:
      setattr(m, k, meta[k])
    m.gravity = np.array(meta["gravity"])
    m.names = meta["names"]
    m.arrays = {k[2:]: z[k].copy() for k in z.files if k.startswith("a_")}
  return m


def load_scene(name: str) -> Model:
  path = os.path.join(ASSET_DIR, f"{name}.npz")
  if not os.path.exists(path):
    raise FileNotFoundError(f"compiled scene {path} missing; run scripts/build_assets.py")
  return load_model(path)
