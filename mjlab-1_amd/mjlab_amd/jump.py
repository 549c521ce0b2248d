"""Jump task (`Mjlab-Jump-Flat-Unitree-G1`) on the MI355X engine, and
its heightfield variant (config 5, row a30).

Restates `src/mjlab/tasks/jump/mdp/{commands,rewards,observations,terminations,
curriculums}.py` and `tasks/jump/{jump_env_cfg.py,config/g1/env_cfgs.py}`: same names,
parameters and math, including the reference's behaviours that look accidental but are
what it computes:
  - `jump_height_reward` / `landing_balance` keep state but define `reset_idx`, not
    `reset`, so the reward manager never resets them (`managers/reward_manager.py:113`);
  - `explosive_takeoff` multiplies actuator forces (actuator order) by joint velocities
    (joint order) element-wise;
  - `synchronized_extension` is the variance of all joint velocities.
Each term also runs inside the sync-free graph-captured env step (no host reads).
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from . import mdp
from .managers import (CommandTerm, CommandTermCfg, CurriculumTermCfg, EventTermCfg,
                       ObservationGroupCfg, ObservationTermCfg, RewardTermCfg, SceneEntityCfg,
                       TerminationTermCfg, UniformNoiseCfg)

_ROBOT = SceneEntityCfg("robot")


# =========================================================================== command
class JumpCommand(CommandTerm):
  """`commands.py:17-62`: target height [B, 1], set on resample, never time-resampled."""

  def __init__(self, cfg, env):
    super().__init__(cfg, env)
    self.height_command = torch.full((self.num_envs, 1), cfg.target_height, device=self.device)
    self.metrics["target_height"] = torch.zeros(self.num_envs, device=self.device)
    self.metrics["peak_height"] = torch.zeros(self.num_envs, device=self.device)

  @property
  def command(self):
    return self.height_command

  def _resample_command(self, env_ids):
    self.height_command[env_ids] = self.cfg.target_height

  def _resample_command_masked(self, mask):
    # cfg.target_height changes only at curriculum time, which re-records the step graph
    self.height_command.masked_fill_(mask.unsqueeze(1), self.cfg.target_height)

  def _update_command(self):
    pass

  def _update_metrics(self):
    self.metrics["target_height"].fill_(self.cfg.target_height)


@dataclass(kw_only=True)
class JumpCommandCfg(CommandTermCfg):
  """`commands.py:65-76`."""
  class_type: type | None = None
  resampling_time_range: tuple[float, float] = (1e9, 1e9)
  target_height: float = 0.25
  height_tolerance: float = 0.05

  def __post_init__(self):
    if self.class_type is None:
      self.class_type = JumpCommand


# =========================================================================== observations
def height_above_ground(env, asset_cfg=_ROBOT):
  """`observations.py:19-41`: root z minus a flat terrain height of 0 (the reference
  does not query the terrain)."""
  return env.scene[asset_cfg.name].data.root_link_pos_w[:, 2].unsqueeze(-1)


def vertical_velocity(env, asset_cfg=_ROBOT):
  return env.scene[asset_cfg.name].data.root_link_lin_vel_w[:, 2:3]


def foot_height(env, asset_cfg=_ROBOT):
  return env.scene[asset_cfg.name].data.site_pos_w[:, asset_cfg.site_ids, 2]


def foot_air_time(env, sensor_name: str):
  return env.scene[sensor_name].data.current_air_time


def foot_contact(env, sensor_name: str):
  return (env.scene[sensor_name].data.found > 0).float()


def foot_contact_forces(env, sensor_name: str):
  f = env.scene[sensor_name].data.force.flatten(start_dim=1)
  return torch.sign(f) * torch.log1p(torch.abs(f))


# =========================================================================== rewards
class jump_height_reward:
  """`rewards.py:20-70`."""

  def __init__(self, cfg, env):
    self.peak_heights = torch.zeros(env.num_envs, device=env.device)
    self.initial_heights = torch.zeros(env.num_envs, device=env.device)
    self.initialized = torch.zeros(env.num_envs, dtype=torch.bool, device=env.device)

  def __call__(self, env, target_height: float, std: float, asset_cfg=_ROBOT):
    h = env.scene[asset_cfg.name].data.root_link_pos_w[:, 2]
    self.initial_heights.copy_(torch.where(~self.initialized, h, self.initial_heights))
    self.initialized.fill_(True)
    torch.maximum(self.peak_heights, h, out=self.peak_heights)
    jump = self.peak_heights - self.initial_heights
    env.extras["log"]["Metrics/peak_jump_height"] = torch.mean(self.peak_heights)
    env.extras["log"]["Metrics/jump_height"] = torch.mean(jump)
    return torch.exp(-((jump - target_height) ** 2) / (std ** 2))

  def reset_idx(self, env_ids):
    self.peak_heights[env_ids] = 0.0
    self.initial_heights[env_ids] = 0.0
    self.initialized[env_ids] = False


def explosive_takeoff(env, sensor_name: str, power_threshold: float = 500.0, asset_cfg=_ROBOT):
  """`rewards.py:73-108`."""
  a = env.scene[asset_cfg.name]
  in_contact = (env.scene[sensor_name].data.found > 0).any(dim=1)
  power = torch.abs(a.data.actuator_force * a.data.joint_vel)
  leg = asset_cfg.joint_ids if asset_cfg.joint_ids is not None else slice(None)
  total = torch.sum(power[:, leg], dim=1)
  return torch.clamp(total - power_threshold, min=0.0) * in_contact.float() / 1000.0


def synchronized_extension(env, asset_cfg=_ROBOT):
  """`rewards.py:111-139`."""
  jv = env.scene[asset_cfg.name].data.joint_vel
  return torch.mean((jv - torch.mean(jv, dim=1, keepdim=True)) ** 2, dim=1)


def vertical_impulse(env, sensor_name: str):
  """`rewards.py:142-167`."""
  f = env.scene[sensor_name].data.force
  return torch.sum(torch.clamp(f[:, :, 2], min=0.0), dim=1) / 500.0


def air_time_bonus(env, sensor_name: str, min_air_time: float = 0.2):
  """`rewards.py:170-204`."""
  at = env.scene[sensor_name].data.current_air_time
  r = torch.clamp(torch.exp((torch.min(at, dim=1)[0] - min_air_time) / min_air_time) - 1.0, min=0.0)
  in_air = (at > 0).float()
  env.extras["log"]["Metrics/air_time_mean"] = torch.sum(at * in_air) / torch.clamp(in_air.sum(), min=1)
  return r


class landing_balance:
  """`rewards.py:207-270`."""

  def __init__(self, cfg, env):
    self.stability_timer = torch.zeros(env.num_envs, device=env.device)
    self.was_in_air = torch.zeros(env.num_envs, dtype=torch.bool, device=env.device)
    self.step_dt = env.step_dt

  def __call__(self, env, sensor_name: str, stability_time: float = 0.5, asset_cfg=_ROBOT):
    a = env.scene[asset_cfg.name]
    in_contact = (env.scene[sensor_name].data.found > 0).any(dim=1)
    just_landed = self.was_in_air & in_contact
    self.was_in_air.copy_(~in_contact)
    upright = torch.abs(a.data.projected_gravity_b[:, 2] + 1.0) < 0.2
    low_vel = (torch.norm(a.data.root_link_lin_vel_w, dim=1) < 0.5) & \
              (torch.norm(a.data.root_link_ang_vel_w, dim=1) < 0.5)
    stable = upright & low_vel & in_contact
    t = torch.where(just_landed, torch.zeros_like(self.stability_timer), self.stability_timer)
    self.stability_timer.copy_(torch.where(stable, t + self.step_dt, torch.zeros_like(t)))
    env.extras["log"]["Metrics/landing_success_rate"] = torch.mean(
      (self.stability_timer > stability_time).float())
    return torch.exp(self.stability_timer / stability_time) - 1.0

  def reset_idx(self, env_ids):
    self.stability_timer[env_ids] = 0.0
    self.was_in_air[env_ids] = False


def symmetric_landing(env, sensor_name: str, time_tolerance: float = 0.05):
  """`rewards.py:273-316`."""
  first = env.scene[sensor_name].compute_first_contact(dt=env.step_dt)
  if first.shape[1] < 2:
    return torch.zeros(env.num_envs, device=env.device)
  return (first[:, 0] & first[:, 1]).float()


# =========================================================================== terminations
def excessive_landing_force(env, sensor_name: str, force_threshold: float = 2500.0):
  """`terminations.py:15-45`."""
  f = env.scene[sensor_name].data.force
  return torch.max(torch.norm(f, dim=-1), dim=1)[0] > force_threshold


# =========================================================================== curricula
def progressive_jump_height(env, env_ids, command_name: str, height_stages: list):
  """`curriculums.py:37-70` (global, by common_step_counter)."""
  cfg = env.command_manager.get_term(command_name).cfg
  for st in height_stages:
    if env.common_step_counter > st["step"]:
      cfg.target_height = st["target_height"]
      cfg.height_tolerance = st["tolerance"]
  return {"target_height": torch.tensor(cfg.target_height),
          "height_tolerance": torch.tensor(cfg.height_tolerance)}


def progressive_stability_requirement(env, env_ids, reward_name: str, weight_stages: list):
  """`curriculums.py:73-97`."""
  c = env.reward_manager.get_term_cfg(reward_name)
  for st in weight_stages:
    if env.common_step_counter > st["step"]:
      c.weight = st["weight"]
  return torch.tensor([c.weight])


# =========================================================================== task config
def make_jump_env_cfg(scene_name: str = "g1_jump"):
  """`tasks/jump/jump_env_cfg.py:36-354`."""
  from .envs import ManagerBasedRlEnvCfg, SceneCfg
  from .sim import MujocoCfg, SimulationCfg
  U = UniformNoiseCfg
  policy = {
    "base_lin_vel": ObservationTermCfg(func=mdp.builtin_sensor, params={"sensor_name": "robot/imu_lin_vel"},
                                       noise=U(n_min=-0.5, n_max=0.5)),
    "base_ang_vel": ObservationTermCfg(func=mdp.builtin_sensor, params={"sensor_name": "robot/imu_ang_vel"},
                                       noise=U(n_min=-0.2, n_max=0.2)),
    "projected_gravity": ObservationTermCfg(func=mdp.projected_gravity, noise=U(n_min=-0.05, n_max=0.05)),
    "joint_pos": ObservationTermCfg(func=mdp.joint_pos_rel, noise=U(n_min=-0.01, n_max=0.01)),
    "joint_vel": ObservationTermCfg(func=mdp.joint_vel_rel, noise=U(n_min=-1.5, n_max=1.5)),
    "actions": ObservationTermCfg(func=mdp.last_action),
    "height_above_ground": ObservationTermCfg(func=height_above_ground),
    "vertical_velocity": ObservationTermCfg(func=vertical_velocity),
    "contact_state": ObservationTermCfg(func=foot_contact, params={"sensor_name": "feet_ground_contact"}),
    "time_in_air": ObservationTermCfg(func=foot_air_time, params={"sensor_name": "feet_ground_contact"}),
    "command": ObservationTermCfg(func=mdp.generated_commands, params={"command_name": "jump"}),
  }
  import copy
  critic = {k: copy.deepcopy(v) for k, v in policy.items()}
  critic.update({
    "foot_height": ObservationTermCfg(func=foot_height,
                                      params={"asset_cfg": SceneEntityCfg("robot", site_names=())}),
    "foot_contact_forces": ObservationTermCfg(func=foot_contact_forces,
                                              params={"sensor_name": "feet_ground_contact"}),
  })
  observations = {
    "policy": ObservationGroupCfg(terms=policy, concatenate_terms=True, enable_corruption=True),
    "critic": ObservationGroupCfg(terms=critic, concatenate_terms=True, enable_corruption=False),
  }
  actions = {"joint_pos": mdp.JointPositionActionCfg(asset_name="robot", actuator_names=(".*",),
                                                    scale=0.5, use_default_offset=True)}
  commands = {"jump": JumpCommandCfg(target_height=0.25, height_tolerance=0.05)}
  events = {
    "reset_base": EventTermCfg(func=mdp.reset_root_state_uniform, mode="reset", params={
      "pose_range": {"x": (-0.1, 0.1), "y": (-0.1, 0.1), "yaw": (-0.1, 0.1)}, "velocity_range": {}}),
    "reset_robot_joints": EventTermCfg(func=mdp.reset_joints_by_offset, mode="reset", params={
      "position_range": (-0.1, 0.1), "velocity_range": (0.0, 0.0),
      "asset_cfg": SceneEntityCfg("robot", joint_names=(".*",))}),
  }
  fs = {"sensor_name": "feet_ground_contact"}
  rewards = {
    "jump_height": RewardTermCfg(func=jump_height_reward, weight=10.0,
                                 params={"target_height": 0.25, "std": 0.15}),
    "explosive_takeoff": RewardTermCfg(func=explosive_takeoff, weight=3.0,
                                       params={**fs, "power_threshold": 500.0}),
    "synchronized_extension": RewardTermCfg(func=synchronized_extension, weight=-2.0),
    "vertical_impulse": RewardTermCfg(func=vertical_impulse, weight=2.0, params=dict(fs)),
    "air_time_bonus": RewardTermCfg(func=air_time_bonus, weight=1.5, params={**fs, "min_air_time": 0.2}),
    "upright_in_flight": RewardTermCfg(func=mdp.flat_orientation, weight=3.0, params={
      "std": math.sqrt(0.3), "asset_cfg": SceneEntityCfg("robot", body_names=())}),
    "angular_momentum_control": RewardTermCfg(func=mdp.angular_momentum_penalty, weight=-0.5,
                                              params={"sensor_name": "robot/root_angmom"}),
    "soft_landing": RewardTermCfg(func=mdp.soft_landing, weight=-2.0, params={**fs, "command_name": None}),
    "landing_stability": RewardTermCfg(func=landing_balance, weight=4.0,
                                       params={**fs, "stability_time": 0.5}),
    "symmetric_landing": RewardTermCfg(func=symmetric_landing, weight=1.0,
                                       params={**fs, "time_tolerance": 0.05}),
    "action_rate_l2": RewardTermCfg(func=mdp.action_rate_l2, weight=-0.05),
    "action_smoothness": RewardTermCfg(func=mdp.action_acc_l2, weight=-0.01),
    "joint_torques_l2": RewardTermCfg(func=mdp.joint_torques_l2, weight=-1e-5,
                                      params={"asset_cfg": SceneEntityCfg("robot", joint_names=(".*",))}),
    "dof_pos_limits": RewardTermCfg(func=mdp.joint_pos_limits, weight=-5.0),
    "alive": RewardTermCfg(func=mdp.is_alive, weight=0.5),
  }
  terminations = {
    "time_out": TerminationTermCfg(func=mdp.time_out, time_out=True),
    "fell_over": TerminationTermCfg(func=mdp.bad_orientation, params={"limit_angle": math.radians(60.0)}),
    "height_too_low": TerminationTermCfg(func=mdp.root_height_below_minimum, params={
      "minimum_height": 0.35, "asset_cfg": SceneEntityCfg("robot")}),
    "excessive_impact": TerminationTermCfg(func=excessive_landing_force,
                                           params={**fs, "force_threshold": 2500.0}),
  }
  curriculum = {
    "jump_height_progression": CurriculumTermCfg(func=progressive_jump_height, params={
      "command_name": "jump", "height_stages": [
        {"step": 0, "target_height": 0.10, "tolerance": 0.05},
        {"step": 10000 * 24, "target_height": 0.15, "tolerance": 0.05},
        {"step": 20000 * 24, "target_height": 0.20, "tolerance": 0.05},
        {"step": 35000 * 24, "target_height": 0.25, "tolerance": 0.08}]}),
    "landing_stability_progression": CurriculumTermCfg(func=progressive_stability_requirement, params={
      "reward_name": "landing_stability", "weight_stages": [
        {"step": 0, "weight": 1.0}, {"step": 15000 * 24, "weight": 2.5},
        {"step": 30000 * 24, "weight": 4.0}]}),
  }
  from .terrains import TerrainImporterCfg, hf_rough_terrains_cfg
  if scene_name == "g1_jump_hfield":
    # config 5: the jump cfg re-terrained onto the seeded heightfield grid
    terrain = TerrainImporterCfg(terrain_type="generator", terrain_generator=hf_rough_terrains_cfg(seed=0))
  else:
    terrain = TerrainImporterCfg(terrain_type="plane")
  return ManagerBasedRlEnvCfg(
    scene=SceneCfg(num_envs=4096, terrain=terrain), observations=observations,
    actions=actions, commands=commands, events=events, rewards=rewards,
    terminations=terminations, curriculum=curriculum,
    sim=SimulationCfg(nconmax=35, njmax=300, mujoco=MujocoCfg(timestep=0.002, iterations=10,
                                                               ls_iterations=20)),
    decimation=2, episode_length_s=5.0)


def unitree_g1_jump_env_cfg(play: bool = False, scene_name: str = "g1_jump"):
  """`tasks/jump/config/g1/env_cfgs.py:49-112`."""
  from . import asset_zoo as az
  from .sensor import ContactMatch, ContactSensorCfg
  cfg = make_jump_env_cfg(scene_name)
  cfg.scene.entities = {"robot": az.get_g1_robot_cfg(az.G1_JUMP_CROUCH)}
  cfg.scene.sensors = (ContactSensorCfg(
    name="feet_ground_contact",
    primary=ContactMatch(mode="subtree", entity="robot",
                         pattern=r"^(left_ankle_roll_link|right_ankle_roll_link)$"),
    secondary=ContactMatch(mode="body", pattern="terrain"),
    fields=("found", "force"), reduce="netforce", num_slots=1, track_air_time=True),)
  cfg.actions["joint_pos"].scale = az.action_scale(az.g1_actuators())
  cfg.observations["critic"].terms["foot_height"].params["asset_cfg"].site_names = (
    "left_foot", "right_foot")
  cfg.rewards["upright_in_flight"].params["asset_cfg"].body_names = ("torso_link",)
  if play:
    cfg.episode_length_s = int(1e9)
    cfg.observations["policy"].enable_corruption = False
    cfg.events.clear()
  return cfg
