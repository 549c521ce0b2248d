"""ManagerBasedRlEnv, task configs and the task registry.

`ManagerBasedRlEnv.step()` / `reset()` follow `src/mjlab/envs/manager_based_rl_env.py:
254-416` step for step (decimation loop, counters, terminations, rewards, resets with
write_data_to_sim + forward, commands, interval events, observations).  Task factories
restate `tasks/velocity/velocity_env_cfg.py:33-354` and
`tasks/velocity/config/{g1,go1}/env_cfgs.py`.
"""

from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Any

import numpy as np
import torch

from . import asset_zoo as az
from . import mdp
from .managers import (ActionManager, CommandManager, CurriculumManager, CurriculumTermCfg,
                       EventManager, EventTermCfg, NullCommandManager, NullCurriculumManager,
                       ObservationGroupCfg, ObservationManager, ObservationTermCfg,
                       RewardManager, RewardTermCfg, SceneEntityCfg, TerminationManager,
                       TerminationTermCfg, UniformNoiseCfg)
from .entity import EntityCfg  # noqa: F401  (re-exported: the reference's mjlab.entity)
from .scene import Scene, SceneCfg
from .sensor import ContactMatch, ContactSensorCfg
from .sim import MujocoCfg, Simulation, SimulationCfg
from .terrains import TerrainImporterCfg, rough_terrains_cfg


@dataclass(kw_only=True)
class ManagerBasedRlEnvCfg:
  decimation: int
  scene: SceneCfg
  observations: dict[str, ObservationGroupCfg] = field(default_factory=dict)
  actions: dict = field(default_factory=dict)
  events: dict = field(default_factory=dict)
  seed: int | None = None
  sim: SimulationCfg = field(default_factory=SimulationCfg)
  rewards: dict = field(default_factory=dict)
  terminations: dict = field(default_factory=dict)
  commands: dict | None = None
  curriculum: dict | None = None
  episode_length_s: float = 0.0
  is_finite_horizon: bool = False


def _cfg_fingerprint(v, depth: int = 0):
  """Hashable snapshot of the plain values in a cfg (dataclass / dict / sequence of
  scalars); callables, tensors and other objects are skipped (curricula change numbers,
  not functions)."""
  if isinstance(v, (bool, int, float, str)) or v is None:
    return v
  if depth > 4:
    return None
  if isinstance(v, (tuple, list)):
    return tuple(_cfg_fingerprint(x, depth + 1) for x in v)
  if isinstance(v, dict):
    return tuple((k, _cfg_fingerprint(x, depth + 1)) for k, x in v.items())
  fields = getattr(v, "__dataclass_fields__", None)
  if fields is not None:
    return tuple((k, _cfg_fingerprint(getattr(v, k, None), depth + 1)) for k in fields)
  return None


def seed_rng(seed: int) -> None:
  import random
  random.seed(seed)
  np.random.seed(seed)
  torch.manual_seed(seed)


class ManagerBasedRlEnv:
  """Manager-based RL environment on the MI355X engine."""

  is_vector_env = True

  def __init__(self, cfg: ManagerBasedRlEnvCfg, device: str, render_mode: str | None = None,
               **kwargs):
    self.cfg = cfg
    if cfg.seed is not None:
      self.cfg.seed = self.seed(cfg.seed)
    self._sim_step_counter = 0
    self.extras: dict[str, Any] = {}
    self.obs_buf = {}
    self._fused = None
    # the scene is assembled from cfg.scene (entities, terrain, sensors) and compiled here
    # (`envs/manager_based_rl_env.py:115-122`)
    self.scene = Scene(cfg.scene, device)
    model = self.scene.compile()
    self.sim = self._make_sim(model, device)
    self.scene.initialize(self.sim.mj_model, self.sim.model, self.sim.data)
    self.common_step_counter = 0
    self.episode_length_buf = torch.zeros(cfg.scene.num_envs, device=device, dtype=torch.long)
    self.render_mode = render_mode
    self.sync_free = False
    self._use_graph = False
    self.load_managers()

  def _make_sim(self, model, device: str):
    """The physics boundary (`envs/manager_based_rl_env.py:117-122`): the HIP engine.  There
    is no CPU fallback; `Simulation` refuses a non-ROCm device."""
    return Simulation(num_envs=self.cfg.scene.num_envs, cfg=self.cfg.sim, model=model, device=device)

  @property
  def num_envs(self) -> int:
    return self.scene.num_envs

  @property
  def physics_dt(self) -> float:
    return self.cfg.sim.mujoco.timestep

  @property
  def step_dt(self) -> float:
    return self.cfg.sim.mujoco.timestep * self.cfg.decimation

  @property
  def device(self) -> str:
    return self.sim.device

  @property
  def max_episode_length_s(self) -> float:
    return self.cfg.episode_length_s

  @property
  def max_episode_length(self) -> int:
    return math.ceil(self.max_episode_length_s / self.step_dt)

  @property
  def unwrapped(self):
    return self

  def load_managers(self) -> None:
    self.extras["log"] = {}
    self.event_manager = EventManager(self.cfg.events, self)
    self.sim.expand_model_fields(self.event_manager.domain_randomization_fields)
    self.command_manager = (CommandManager(self.cfg.commands, self) if self.cfg.commands
                            else NullCommandManager())
    self.action_manager = ActionManager(self.cfg.actions, self)
    self.observation_manager = ObservationManager(self.cfg.observations, self)
    self.termination_manager = TerminationManager(self.cfg.terminations, self)
    self.reward_manager = RewardManager(self.cfg.rewards, self)
    self.curriculum_manager = (CurriculumManager(self.cfg.curriculum, self) if self.cfg.curriculum
                               else NullCurriculumManager())
    self._configure_spaces()
    if "startup" in self.event_manager.available_modes:
      self.event_manager.apply(mode="startup")

  def _configure_spaces(self):
    self.single_action_dim = sum(self.action_manager.action_term_dim)
    self.observation_dims = dict(self.observation_manager.group_obs_dim)

  @staticmethod
  def seed(seed: int = -1) -> int:
    if seed == -1:
      seed = np.random.randint(0, 10_000)
    seed_rng(seed)
    return seed

  def reset(self, *, seed: int | None = None, env_ids: torch.Tensor | None = None,
            options: dict | None = None):
    if env_ids is None:
      env_ids = torch.arange(self.num_envs, dtype=torch.int64, device=self.device)
    if seed is not None:
      self.seed(seed)
    self._reset_idx(env_ids)
    self.scene.write_data_to_sim()
    self.sim.forward()
    self.obs_buf = self.observation_manager.compute(update_history=True)
    return self.obs_buf, self.extras

  # ------------------------------------------------------------------ sync-free + graph
  def _step_sync_free(self, action: torch.Tensor):
    """Same stages as step(), with every data-dependent branch turned into masks so the
    whole env step is host-sync-free and can be captured in one HIP graph.  Velocity-task
    configs run the fused HIP managers instead (mjlab_amd/fused.py)."""
    if self._fused is not None:
      self.obs_buf, rew, term, trunc = self._fused.step(action)
      self.reward_buf, self.reset_terminated, self.reset_time_outs = rew, term, trunc
      self.reset_buf = self._fused.reset_buf
      self._log_sim_counters(self.extras.setdefault("log", {}))
      return self.obs_buf, rew, term, trunc
    self.action_manager.process_action(action)
    for _ in range(self.cfg.decimation):
      self.action_manager.apply_action()
      self.scene.write_data_to_sim()
      self.sim.step()
      self.scene.update(dt=self.physics_dt)
    self.episode_length_buf += 1
    self.reset_buf = self.termination_manager.compute()
    self.reset_terminated = self.termination_manager.terminated
    self.reset_time_outs = self.termination_manager.time_outs
    self.reward_buf = self.reward_manager.compute(dt=self.step_dt)
    self._reset_masked(self.reset_buf)
    self.scene.write_data_to_sim()
    self.sim.forward(mask=self.reset_buf)
    self.command_manager.compute(dt=self.step_dt)
    if "interval" in self.event_manager.available_modes:
      self.event_manager.apply_masked(mode="interval", dt=self.step_dt)
    self.obs_buf = self.observation_manager.compute(update_history=True)
    return self.obs_buf, self.reward_buf, self.reset_terminated, self.reset_time_outs

  def _reset_masked(self, mask: torch.Tensor) -> None:
    self.curriculum_manager.compute_masked(mask)
    self.sim.reset_masked(mask)
    self.scene.reset_masked(mask)
    if "reset" in self.event_manager.available_modes:
      self.event_manager.apply_masked(mode="reset", mask=mask)
    log = self.extras.setdefault("log", {})
    for mgr in (self.action_manager, self.reward_manager, self.command_manager,
                self.event_manager, self.termination_manager):
      log.update(mgr.reset_masked(mask))
    self._log_sim_counters(log)
    self.observation_manager.reset(None)
    self.episode_length_buf.masked_fill_(mask, 0)

  def _graph_key(self):
    """Everything a curriculum may mutate that the captured step bakes in as a host
    constant: every field of each command cfg (ranges, and e.g. the jump task's
    target_height / height_tolerance, `tasks/jump/mdp/curriculums.py:37-70`), and each
    reward term's weight and scalar params (`curriculums.py:73-97` sets a weight; a
    zero weight is skipped at capture time).  A change re-records the graph."""
    cmds = tuple(_cfg_fingerprint(t.cfg) for t in self.command_manager._terms.values()) \
        if self.cfg.commands else ()
    rm = self.reward_manager
    rews = tuple((c.weight, _cfg_fingerprint(c.params)) for c in rm._term_cfgs)
    return cmds, rews

  def enable_graph(self, capture: bool = True, fused: bool = True) -> None:
    """Switch to the sync-free step; with capture=True record it into a HIP graph
    (replayed per step; re-recorded when a curriculum changes command ranges)."""
    if self.sim.nan_guard.enabled:
      import warnings
      warnings.warn("NanGuard is enabled: the env step stays eager (the guard reads a NaN "
                    "flag back to the host after every physics step)")
      return
    self.sync_free = True
    self._use_graph = capture
    if self._fused is not None and hasattr(self._fused, "release"):
      self._fused.release()  # the engine stops owning the contact air-time buffers
    self._fused = None
    if fused and os.environ.get("MJX355_FUSED", "1") != "0":
      from .fused import FusedJumpStep, FusedVelocityStep
      from .fused_tracking import FusedTrackingStep
      why = []
      for kind, cls in (("velocity", FusedVelocityStep), ("jump", FusedJumpStep),
                        ("tracking", FusedTrackingStep)):
        self._fused = cls.build(self)
        if self._fused is not None:
          break
        why.append(f"{kind}: {getattr(self, '_fused_unsupported', '')}")
      if self._fused is None:
        self._fused_unsupported = "; ".join(why)
      if self._fused is not None:
        self.extras["log"] = self._fused.log()
    self._graph = None
    self._static_action = torch.zeros(self.num_envs, self.action_manager.total_action_dim,
                                      device=self.device)

  @torch.inference_mode(False)
  def _capture(self, action: torch.Tensor):
    """Run one real sync-free step (it also warms the allocator and lazy tensors), then
    record the step into a HIP graph.  Recording executes nothing, so the env advances
    exactly one step per call, as in eager mode.  Recorded outside inference mode (a
    runner steps the env inside it): tensors made here are updated in place by every
    later step, and the capture registers the CUDA generator's graph state."""
    if self._fused is not None:
      self._fused.upload()  # command ranges may have changed (curriculum)
    self._static_action.copy_(action)
    s = torch.cuda.Stream(device=self.device)
    s.wait_stream(torch.cuda.current_stream(self.device))
    with torch.cuda.stream(s):
      out = tuple(t.clone() for t in self._step_sync_free(self._static_action)[1:])
      obs = {k: v.clone() for k, v in self.obs_buf.items()}
    torch.cuda.current_stream(self.device).wait_stream(s)
    # fused managers: the action kernel stays outside the graph and runs before each replay,
    # on the caller's tensor (no copy into the static input buffer)
    fa = self._fused if self._fused is not None and hasattr(self._fused, "apply_action") else None
    if os.environ.get("MJX355_GRAPH_ACTION", "0") != "0":  # diagnostic: the action kernel in the graph
      fa = None
    g = torch.cuda.CUDAGraph()
    if fa is not None:
      fa.action_in_step = False
    try:
      with torch.cuda.graph(g):
        self._graph_out = self._step_sync_free(self._static_action)
    finally:
      if fa is not None:
        fa.action_in_step = True
    self._graph_action = fa
    self._graph = g
    self._graph_key_captured = self._graph_key()
    self.obs_buf = obs
    self.reward_buf, self.reset_terminated, self.reset_time_outs = out
    return (obs, *out)

  def step(self, action: torch.Tensor):
    if getattr(self, "sync_free", False):
      # per-env curriculum terms (terrain levels) run on the reset mask inside the step
      self.curriculum_manager.compute(env_ids=None, skip_masked=True)
      self._sim_step_counter += self.cfg.decimation
      self.common_step_counter += 1
      if not self._use_graph:
        if self._fused is not None and self._graph_key() != getattr(self, "_fused_key", None):
          self._fused.upload()
          self._fused_key = self._graph_key()
        out = self._step_sync_free(action.to(self.device).contiguous())
        return (*out, self.extras)
      if self._graph is None or self._graph_key() != self._graph_key_captured:
        return (*self._capture(action), self.extras)
      fa = getattr(self, "_graph_action", None)
      if fa is not None:
        a = action
        if not (a.is_cuda and a.dtype == torch.float32 and a.is_contiguous()
                and a.device == self._static_action.device and a.shape == self._static_action.shape):
          self._static_action.copy_(a)
          a = self._static_action
        fa.apply_action(a)
      else:
        self._static_action.copy_(action)
      self._graph.replay()
      self.obs_buf, self.reward_buf, self.reset_terminated, self.reset_time_outs = self._graph_out
      return (*self._graph_out, self.extras)
    return self._step_eager(action)

  def _step_eager(self, action: torch.Tensor):
    self.action_manager.process_action(action.to(self.device))
    for _ in range(self.cfg.decimation):
      self._sim_step_counter += 1
      self.action_manager.apply_action()
      self.scene.write_data_to_sim()
      self.sim.step()
      self.scene.update(dt=self.physics_dt)
    self.episode_length_buf += 1
    self.common_step_counter += 1
    self.reset_buf = self.termination_manager.compute()
    self.reset_terminated = self.termination_manager.terminated
    self.reset_time_outs = self.termination_manager.time_outs
    self.reward_buf = self.reward_manager.compute(dt=self.step_dt)
    reset_env_ids = self.reset_buf.nonzero(as_tuple=False).squeeze(-1)
    if len(reset_env_ids) > 0:
      self._reset_idx(reset_env_ids)
      self.scene.write_data_to_sim()
      self.sim.forward()
    self.command_manager.compute(dt=self.step_dt)
    if "interval" in self.event_manager.available_modes:
      self.event_manager.apply(mode="interval", dt=self.step_dt)
    self.obs_buf = self.observation_manager.compute(update_history=True)
    return self.obs_buf, self.reward_buf, self.reset_terminated, self.reset_time_outs, self.extras

  def _reset_idx(self, env_ids: torch.Tensor) -> None:
    self.curriculum_manager.compute(env_ids=env_ids)
    self.sim.reset(env_ids)
    self.scene.reset(env_ids)
    if "reset" in self.event_manager.available_modes:
      self.event_manager.apply(mode="reset", env_ids=env_ids,
                               global_env_step_count=self._sim_step_counter // self.cfg.decimation)
    self.extras["log"] = {}
    for mgr in (self.observation_manager, self.action_manager, self.reward_manager,
                self.curriculum_manager, self.command_manager, self.event_manager,
                self.termination_manager):
      self.extras["log"].update(mgr.reset(env_ids))
    self._log_sim_counters(self.extras["log"])
    self.episode_length_buf[env_ids] = 0

  def _log_sim_counters(self, log: dict) -> None:
    """Engine overflow counters (contacts dropped because a world's contacts or rows
    exceeded its max capacity, and unsupported geom pairs) and the world-substeps re-solved
    at the max capacity after overflowing the fast carve, cumulative over all worlds, as
    device scalars: no host sync."""
    ev = getattr(self, "_sim_events", None)
    if ev is None:
      ev = self._sim_events = self.sim.event_counts()
    log["Sim/contact_overflow"] = ev[0]
    log["Sim/row_overflow"] = ev[1]
    log["Sim/unsupported_pairs"] = ev[2]
    log["Sim/resolved_overflow"] = ev[3]

  def packed_episode_stats(self) -> torch.Tensor:
    """Episode statistics of the last reset, packed into one fp32 vector (for the
    cross-rank all-gather)."""
    vals = []
    for v in self.extras.get("log", {}).values():
      vals.append(torch.as_tensor(v, dtype=torch.float32, device=self.device).reshape(-1)[:1])
    if not vals:
      return torch.zeros(1, device=self.device)
    return torch.cat(vals)

  def close(self) -> None:
    pass


# =========================================================================== task configs
def make_velocity_env_cfg() -> ManagerBasedRlEnvCfg:
  """`tasks/velocity/velocity_env_cfg.py:33-354`: the rough-terrain scene (ROUGH_TERRAINS_CFG,
  `max_init_terrain_level` 5; the reference draws the generator seed at random, this build
  fixes it at 0) with no entity yet; the robot configs add the robot and its sensors."""
  policy = {
    "base_lin_vel": ObservationTermCfg(func=mdp.builtin_sensor, params={"sensor_name": "robot/imu_lin_vel"},
                                       noise=UniformNoiseCfg(n_min=-0.5, n_max=0.5)),
    "base_ang_vel": ObservationTermCfg(func=mdp.builtin_sensor, params={"sensor_name": "robot/imu_ang_vel"},
                                       noise=UniformNoiseCfg(n_min=-0.2, n_max=0.2)),
    "projected_gravity": ObservationTermCfg(func=mdp.projected_gravity,
                                            noise=UniformNoiseCfg(n_min=-0.05, n_max=0.05)),
    "joint_pos": ObservationTermCfg(func=mdp.joint_pos_rel, noise=UniformNoiseCfg(n_min=-0.01, n_max=0.01)),
    "joint_vel": ObservationTermCfg(func=mdp.joint_vel_rel, noise=UniformNoiseCfg(n_min=-1.5, n_max=1.5)),
    "actions": ObservationTermCfg(func=mdp.last_action),
    "command": ObservationTermCfg(func=mdp.generated_commands, params={"command_name": "twist"}),
  }
  import copy
  critic = {k: copy.deepcopy(v) for k, v in policy.items()}
  critic.update({
    "foot_height": ObservationTermCfg(func=mdp.foot_height, params={"asset_cfg": SceneEntityCfg("robot", site_names=())}),
    "foot_air_time": ObservationTermCfg(func=mdp.foot_air_time, params={"sensor_name": "feet_ground_contact"}),
    "foot_contact": ObservationTermCfg(func=mdp.foot_contact, params={"sensor_name": "feet_ground_contact"}),
    "foot_contact_forces": ObservationTermCfg(func=mdp.foot_contact_forces, params={"sensor_name": "feet_ground_contact"}),
  })
  observations = {
    "policy": ObservationGroupCfg(terms=policy, concatenate_terms=True, enable_corruption=True),
    "critic": ObservationGroupCfg(terms=critic, concatenate_terms=True, enable_corruption=False),
  }
  actions = {"joint_pos": mdp.JointPositionActionCfg(asset_name="robot", actuator_names=(".*",),
                                                    scale=0.5, use_default_offset=True)}
  commands = {"twist": mdp.UniformVelocityCommandCfg(
    asset_name="robot", resampling_time_range=(3.0, 8.0), rel_standing_envs=0.1,
    rel_heading_envs=0.3, heading_command=True, heading_control_stiffness=0.5,
    ranges=mdp.UniformVelocityCommandCfg.Ranges(lin_vel_x=(-1.0, 1.0), lin_vel_y=(-1.0, 1.0),
                                                ang_vel_z=(-0.5, 0.5), heading=(-math.pi, math.pi)))}
  events = {
    "reset_base": EventTermCfg(func=mdp.reset_root_state_uniform, mode="reset", params={
      "pose_range": {"x": (-0.5, 0.5), "y": (-0.5, 0.5), "yaw": (-3.14, 3.14)}, "velocity_range": {}}),
    "reset_robot_joints": EventTermCfg(func=mdp.reset_joints_by_offset, mode="reset", params={
      "position_range": (0.0, 0.0), "velocity_range": (0.0, 0.0),
      "asset_cfg": SceneEntityCfg("robot", joint_names=(".*",))}),
    "push_robot": EventTermCfg(func=mdp.push_by_setting_velocity, mode="interval",
                               interval_range_s=(1.0, 3.0),
                               params={"velocity_range": {"x": (-0.5, 0.5), "y": (-0.5, 0.5)}}),
    "foot_friction": EventTermCfg(mode="startup", func=mdp.randomize_field, domain_randomization=True,
                                  params={"asset_cfg": SceneEntityCfg("robot", geom_names=()),
                                          "operation": "abs", "field": "geom_friction",
                                          "ranges": (0.3, 1.2)}),
  }
  rewards = {
    "track_linear_velocity": RewardTermCfg(func=mdp.track_linear_velocity, weight=2.0,
                                           params={"command_name": "twist", "std": math.sqrt(0.25)}),
    "track_angular_velocity": RewardTermCfg(func=mdp.track_angular_velocity, weight=2.0,
                                            params={"command_name": "twist", "std": math.sqrt(0.5)}),
    "upright": RewardTermCfg(func=mdp.flat_orientation, weight=1.0,
                             params={"std": math.sqrt(0.2), "asset_cfg": SceneEntityCfg("robot", body_names=())}),
    "pose": RewardTermCfg(func=mdp.variable_posture, weight=1.0, params={
      "asset_cfg": SceneEntityCfg("robot", joint_names=(".*",)), "command_name": "twist",
      "std_standing": {}, "std_walking": {}, "std_running": {}, "walking_threshold": 0.05,
      "running_threshold": 1.5}),
    "body_ang_vel": RewardTermCfg(func=mdp.body_angular_velocity_penalty, weight=0.0,
                                  params={"asset_cfg": SceneEntityCfg("robot", body_names=())}),
    "angular_momentum": RewardTermCfg(func=mdp.angular_momentum_penalty, weight=0.0,
                                      params={"sensor_name": "robot/root_angmom"}),
    "dof_pos_limits": RewardTermCfg(func=mdp.joint_pos_limits, weight=-1.0),
    "action_rate_l2": RewardTermCfg(func=mdp.action_rate_l2, weight=-0.1),
    "air_time": RewardTermCfg(func=mdp.feet_air_time, weight=0.0, params={
      "sensor_name": "feet_ground_contact", "threshold_min": 0.05, "threshold_max": 0.5,
      "command_name": "twist", "command_threshold": 0.5}),
    "foot_clearance": RewardTermCfg(func=mdp.feet_clearance, weight=-2.0, params={
      "target_height": 0.1, "command_name": "twist", "command_threshold": 0.05,
      "asset_cfg": SceneEntityCfg("robot", site_names=())}),
    "foot_swing_height": RewardTermCfg(func=mdp.feet_swing_height, weight=-0.25, params={
      "sensor_name": "feet_ground_contact", "target_height": 0.1, "command_name": "twist",
      "command_threshold": 0.05, "asset_cfg": SceneEntityCfg("robot", site_names=())}),
    "foot_slip": RewardTermCfg(func=mdp.feet_slip, weight=-0.1, params={
      "sensor_name": "feet_ground_contact", "command_name": "twist", "command_threshold": 0.05,
      "asset_cfg": SceneEntityCfg("robot", site_names=())}),
    "soft_landing": RewardTermCfg(func=mdp.soft_landing, weight=-1e-5, params={
      "sensor_name": "feet_ground_contact", "command_name": "twist", "command_threshold": 0.05}),
  }
  terminations = {
    "time_out": TerminationTermCfg(func=mdp.time_out, time_out=True),
    "fell_over": TerminationTermCfg(func=mdp.bad_orientation, params={"limit_angle": math.radians(70.0)}),
  }
  curriculum = {"command_vel": CurriculumTermCfg(func=mdp.commands_vel, params={
    "command_name": "twist", "velocity_stages": [
      {"step": 0, "lin_vel_x": (-1.0, 1.0), "ang_vel_z": (-0.5, 0.5)},
      {"step": 5000 * 24, "lin_vel_x": (-1.5, 2.0), "ang_vel_z": (-0.7, 0.7)},
      {"step": 10000 * 24, "lin_vel_x": (-2.0, 3.0)}]})}
  curriculum = {"terrain_levels": CurriculumTermCfg(func=mdp.terrain_levels_vel,
                                                    params={"command_name": "twist"}),
                **curriculum}
  scene = SceneCfg(num_envs=1, terrain=TerrainImporterCfg(
    terrain_type="generator", terrain_generator=rough_terrains_cfg(seed=0), max_init_terrain_level=5))
  return ManagerBasedRlEnvCfg(
    scene=scene, observations=observations,
    actions=actions, commands=commands, events=events, rewards=rewards,
    terminations=terminations, curriculum=curriculum,
    sim=SimulationCfg(nconmax=35, njmax=300, mujoco=MujocoCfg(timestep=0.005, iterations=10,
                                                               ls_iterations=20)),
    decimation=4, episode_length_s=20.0)


def _flat(cfg: ManagerBasedRlEnvCfg) -> ManagerBasedRlEnvCfg:
  """`tasks/velocity/config/g1/env_cfgs.py:153-175`: plane terrain, no terrain curriculum."""
  cfg.scene.terrain.terrain_type = "plane"
  cfg.scene.terrain.terrain_generator = None
  del cfg.curriculum["terrain_levels"]
  return cfg


def _rough(cfg: ManagerBasedRlEnvCfg, play: bool) -> ManagerBasedRlEnvCfg:
  """Rough terrain in curriculum layout (`env_cfgs.py:51-52`); play mode
  (`env_cfgs.py:131-148`): the random-layout 5 x 5 grid with a 10 m border and the
  randomize_terrain reset event."""
  if play:
    cfg.scene.terrain.terrain_generator = rough_terrains_cfg(
      seed=0, curriculum=False, num_rows=5, num_cols=5, border_width=10.0)
    _rough_play_events(cfg)
  else:
    cfg.scene.terrain.terrain_generator.curriculum = True
  return cfg


def unitree_g1_flat_env_cfg(play: bool = False) -> ManagerBasedRlEnvCfg:
  """`tasks/velocity/config/g1/env_cfgs.py:20-175` (flat)."""
  cfg = _g1_velocity_cfg(play)
  if play:
    t = cfg.commands["twist"]
    t.ranges.lin_vel_x = (-1.5, 2.0)
    t.ranges.ang_vel_z = (-0.7, 0.7)
  return _flat(cfg)


def unitree_g1_rough_env_cfg(play: bool = False) -> ManagerBasedRlEnvCfg:
  """`tasks/velocity/config/g1/env_cfgs.py:20-148` (rough): the G1 velocity task on the
  box-stair terrain grid with the terrain-level curriculum (`velocity_env_cfg.py:296-300`)."""
  return _rough(_g1_velocity_cfg(play), play)


def _rough_play_events(cfg) -> None:
  """Play mode of the rough tasks (`tasks/velocity/config/{g1,go1}/env_cfgs.py`, play
  overrides): every reset puts the env on a random sub-terrain (`randomize_terrain`)."""
  cfg.events["randomize_terrain"] = EventTermCfg(func=mdp.randomize_terrain, mode="reset", params={})


def _g1_velocity_cfg(play: bool) -> ManagerBasedRlEnvCfg:
  cfg = make_velocity_env_cfg()
  cfg.scene.entities = {"robot": az.get_g1_robot_cfg()}
  cfg.scene.sensors = (
    ContactSensorCfg(name="feet_ground_contact",
                     primary=ContactMatch(mode="subtree", entity="robot",
                                          pattern=r"^(left_ankle_roll_link|right_ankle_roll_link)$"),
                     secondary=ContactMatch(mode="body", pattern="terrain"),
                     fields=("found", "force"), reduce="netforce", num_slots=1, track_air_time=True),
    ContactSensorCfg(name="self_collision",
                     primary=ContactMatch(mode="subtree", pattern="pelvis", entity="robot"),
                     secondary=ContactMatch(mode="subtree", pattern="pelvis", entity="robot"),
                     fields=("found",), reduce="none", num_slots=1),
  )
  sites = ("left_foot", "right_foot")
  geoms = tuple(f"{s}_foot{i}_collision" for s in ("left", "right") for i in range(1, 8))
  cfg.actions["joint_pos"].scale = az.action_scale(az.g1_actuators())
  cfg.observations["critic"].terms["foot_height"].params["asset_cfg"].site_names = sites
  cfg.events["foot_friction"].params["asset_cfg"].geom_names = geoms
  p = cfg.rewards["pose"].params
  p["std_standing"] = {".*": 0.05}
  p["std_walking"] = {r".*hip_pitch.*": 0.3, r".*hip_roll.*": 0.15, r".*hip_yaw.*": 0.15,
                      r".*knee.*": 0.35, r".*ankle_pitch.*": 0.25, r".*ankle_roll.*": 0.1,
                      r".*waist_yaw.*": 0.2, r".*waist_roll.*": 0.08, r".*waist_pitch.*": 0.1,
                      r".*shoulder_pitch.*": 0.15, r".*shoulder_roll.*": 0.15,
                      r".*shoulder_yaw.*": 0.1, r".*elbow.*": 0.15, r".*wrist.*": 0.3}
  p["std_running"] = {r".*hip_pitch.*": 0.5, r".*hip_roll.*": 0.2, r".*hip_yaw.*": 0.2,
                      r".*knee.*": 0.6, r".*ankle_pitch.*": 0.35, r".*ankle_roll.*": 0.15,
                      r".*waist_yaw.*": 0.3, r".*waist_roll.*": 0.08, r".*waist_pitch.*": 0.2,
                      r".*shoulder_pitch.*": 0.5, r".*shoulder_roll.*": 0.2,
                      r".*shoulder_yaw.*": 0.15, r".*elbow.*": 0.35, r".*wrist.*": 0.3}
  cfg.rewards["upright"].params["asset_cfg"].body_names = ("torso_link",)
  cfg.rewards["body_ang_vel"].params["asset_cfg"].body_names = ("torso_link",)
  for r in ("foot_clearance", "foot_swing_height", "foot_slip"):
    cfg.rewards[r].params["asset_cfg"].site_names = sites
  cfg.rewards["body_ang_vel"].weight = -0.05
  cfg.rewards["angular_momentum"].weight = -0.02
  cfg.rewards["air_time"].weight = 0.0
  cfg.rewards["self_collisions"] = RewardTermCfg(func=mdp.self_collision_cost, weight=-1.0,
                                                 params={"sensor_name": "self_collision"})
  if play:
    cfg.episode_length_s = int(1e9)
    cfg.observations["policy"].enable_corruption = False
    cfg.events.pop("push_robot", None)
  return cfg


def unitree_go1_flat_env_cfg(play: bool = False) -> ManagerBasedRlEnvCfg:
  """`tasks/velocity/config/go1/env_cfgs.py:15-127` (flat).

  Engine carve (not a reference field): 16 contacts / 64 rows per world in the fast LDS
  carve (Go1 flat sees at most 6 / 24), so every phase's carve holds 16 worlds per CU (its
  phase B at 4 waves per SIMD: engine_impl.h kLean); a world past it is re-solved at the max
  capacity (njmax rows), nothing is dropped.  Measured Go1 8,192: 24 / 96 7.96 / 8.00 M,
  16 / 64 8.66 / 8.65 M env-steps/s (round 6)."""
  cfg = _flat(_go1_velocity_cfg(play))
  cfg.sim.engine_capacity = (16, 64)
  return cfg


def unitree_go1_rough_env_cfg(play: bool = False) -> ManagerBasedRlEnvCfg:
  """`tasks/velocity/config/go1/env_cfgs.py:15-112` (rough): the Go1 task on the curriculum
  box-stair grid with the terrain-level curriculum."""
  cfg = _rough(_go1_velocity_cfg(play), play)
  # engine carve: 24 / 96 (its chain inlines the box-box narrowphase; 16 / 64 with phase B at 4
  # waves per SIMD measured -20 %, round 6)
  cfg.sim.engine_capacity = (24, 96)
  return cfg


def _go1_velocity_cfg(play: bool) -> ManagerBasedRlEnvCfg:
  cfg = make_velocity_env_cfg()
  cfg.scene.entities = {"robot": az.get_go1_robot_cfg()}
  names = ("FR", "FL", "RR", "RL")
  geoms = tuple(f"{n}_foot_collision" for n in names)
  cfg.scene.sensors = (
    ContactSensorCfg(name="feet_ground_contact",
                     primary=ContactMatch(mode="geom", pattern=geoms, entity="robot"),
                     secondary=ContactMatch(mode="body", pattern="terrain"),
                     fields=("found", "force"), reduce="netforce", num_slots=1, track_air_time=True),
    ContactSensorCfg(name="nonfoot_ground_touch",
                     primary=ContactMatch(mode="geom", entity="robot", pattern=r".*_collision\d*$",
                                          exclude=geoms),
                     secondary=ContactMatch(mode="body", pattern="terrain"),
                     fields=("found",), reduce="none", num_slots=1),
  )
  cfg.actions["joint_pos"].scale = az.action_scale(az.go1_actuators())
  cfg.observations["critic"].terms["foot_height"].params["asset_cfg"].site_names = names
  cfg.events["foot_friction"].params["asset_cfg"].geom_names = geoms
  p = cfg.rewards["pose"].params
  p["std_standing"] = {r".*(FR|FL|RR|RL)_(hip|thigh)_joint.*": 0.05, r".*(FR|FL|RR|RL)_calf_joint.*": 0.1}
  p["std_walking"] = {r".*(FR|FL|RR|RL)_(hip|thigh)_joint.*": 0.3, r".*(FR|FL|RR|RL)_calf_joint.*": 0.6}
  p["std_running"] = {r".*(FR|FL|RR|RL)_(hip|thigh)_joint.*": 0.3, r".*(FR|FL|RR|RL)_calf_joint.*": 0.6}
  cfg.rewards["upright"].params["asset_cfg"].body_names = ("trunk",)
  cfg.rewards["body_ang_vel"].params["asset_cfg"].body_names = ("trunk",)
  for r in ("foot_clearance", "foot_swing_height", "foot_slip"):
    cfg.rewards[r].params["asset_cfg"].site_names = names
  cfg.rewards["body_ang_vel"].weight = 0.0
  cfg.rewards["angular_momentum"].weight = 0.0
  cfg.rewards["air_time"].weight = 0.0
  cfg.terminations["illegal_contact"] = TerminationTermCfg(
    func=mdp.illegal_contact, params={"sensor_name": "nonfoot_ground_touch"})
  if play:
    cfg.episode_length_s = int(1e9)
    cfg.observations["policy"].enable_corruption = False
    cfg.events.pop("push_robot", None)
  return cfg


def _tracking_g1(play: bool = False):
  from .tracking import unitree_g1_flat_tracking_env_cfg
  return unitree_g1_flat_tracking_env_cfg(play=play)


def _jump_g1(play: bool = False):
  from .jump import unitree_g1_jump_env_cfg
  return unitree_g1_jump_env_cfg(play=play)


def _jump_g1_hfield(play: bool = False):
  """Config 5: the jump cfg on the seeded heightfield terrain grid."""
  from .jump import unitree_g1_jump_env_cfg
  return unitree_g1_jump_env_cfg(play=play, scene_name="g1_jump_hfield")


TASKS = {
  "Mjlab-Velocity-Flat-Unitree-G1": unitree_g1_flat_env_cfg,
  "Mjlab-Velocity-Rough-Unitree-G1": unitree_g1_rough_env_cfg,
  "Mjlab-Velocity-Flat-Unitree-Go1": unitree_go1_flat_env_cfg,
  "Mjlab-Velocity-Rough-Unitree-Go1": unitree_go1_rough_env_cfg,
  "Mjlab-Tracking-Flat-Unitree-G1": _tracking_g1,
  "Mjlab-Jump-Flat-Unitree-G1": _jump_g1,
  "Mjlab-Jump-Hfield-Unitree-G1": _jump_g1_hfield,
}


def load_env_cfg(task: str, play: bool = False) -> ManagerBasedRlEnvCfg:
  if task not in TASKS:
    raise KeyError(f"unknown task {task}; available: {sorted(TASKS)}")
  return TASKS[task](play=play)


def make_env(task: str, num_envs: int, device: str, seed: int = 42, play: bool = False):
  cfg = load_env_cfg(task, play)
  cfg.scene.num_envs = num_envs
  cfg.seed = seed
  return ManagerBasedRlEnv(cfg, device=device)
