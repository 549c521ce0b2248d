"""The edited G1 velocity scene of tests/test_gpu_scene_cfg.py (a cfg.scene edit: a heavier
torso, the foot geoms' friction, a hands contact sensor), shared with __graft_entry__.build(),
which compiles its run-time specialised kernels (mjlab_amd.jit) into the in-tree cache."""

from __future__ import annotations


def edited_g1_cfg(num_envs: int = 16):
  from mjlab_amd.envs import load_env_cfg
  from mjlab_amd.sensor import ContactMatch, ContactSensorCfg
  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = num_envs
  cfg.seed = 3
  robot = cfg.scene.entities["robot"]
  base_fn = robot.spec_fn

  def heavier_torso():
    spec = base_fn()
    spec.body("torso_link").mass = spec.body("torso_link").mass + 2.5
    return spec

  robot.spec_fn = heavier_torso
  robot.collisions[0].friction[r"^(left|right)_foot[1-7]_collision$"] = (0.9,)
  cfg.scene.sensors = cfg.scene.sensors + (ContactSensorCfg(
    name="hands", primary=ContactMatch(mode="body", entity="robot",
                                       pattern=r"^(left|right)_wrist_yaw_link$"),
    secondary=ContactMatch(mode="body", pattern="terrain"), fields=("found", "force"),
    reduce="netforce"),)
  cfg.events.pop("foot_friction")  # keep the edited friction (no startup randomisation)
  return cfg


def sensor_only_g1_cfg(num_envs: int = 16):
  """The shipped G1 velocity scene plus the hands contact sensor only: no physics change (the
  same dynamics, resets and randomisation as the shipped task), but the model dimensions no
  longer match any compiled specs.inc entry -- the run-time specialisation's cost alone."""
  from mjlab_amd.envs import load_env_cfg
  from mjlab_amd.sensor import ContactMatch, ContactSensorCfg
  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.scene.num_envs = num_envs
  cfg.scene.sensors = cfg.scene.sensors + (ContactSensorCfg(
    name="hands", primary=ContactMatch(mode="body", entity="robot",
                                       pattern=r"^(left|right)_wrist_yaw_link$"),
    secondary=ContactMatch(mode="body", pattern="terrain"), fields=("found", "force"),
    reduce="netforce"),)
  return cfg


def jit_targets(cfg):
  """(model, nconmax, njmax, role) of the run-time specialisations a Simulation of `cfg` loads."""
  from mjlab_amd.scene import Scene
  from mjlab_amd.sim.sim import max_capacity, world_capacity
  model = Scene(cfg.scene, "cpu").compile()
  cfg.sim.mujoco.apply(model)
  fast, big = world_capacity(cfg.sim, model), max_capacity(cfg.sim, model)
  out = [(model, fast[0], fast[1], 1)]
  if big != fast:
    out.append((model, big[0], big[1], 2))
  return out
