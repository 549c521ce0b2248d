"""RSL-RL runner configuration (`src/mjlab/rl/config.py:1-115`): same dataclasses, names,
fields and defaults, so the reference's per-task `rl_cfg.py` factories port unchanged."""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Literal, Tuple


@dataclass
class RslRlPpoActorCriticCfg:
  init_noise_std: float = 1.0
  noise_std_type: Literal["scalar", "log"] = "scalar"
  actor_obs_normalization: bool = False
  critic_obs_normalization: bool = False
  actor_hidden_dims: Tuple[int, ...] = (128, 128, 128)
  critic_hidden_dims: Tuple[int, ...] = (128, 128, 128)
  activation: str = "elu"
  class_name: str = "ActorCritic"


@dataclass
class RslRlPpoAlgorithmCfg:
  num_learning_epochs: int = 5
  num_mini_batches: int = 4
  learning_rate: float = 1e-3
  schedule: Literal["adaptive", "fixed"] = "adaptive"
  gamma: float = 0.99
  lam: float = 0.95
  entropy_coef: float = 0.005
  desired_kl: float = 0.01
  max_grad_norm: float = 1.0
  value_loss_coef: float = 1.0
  use_clipped_value_loss: bool = True
  clip_param: float = 0.2
  normalize_advantage_per_mini_batch: bool = False
  class_name: str = "PPO"


@dataclass
class RslRlBaseRunnerCfg:
  seed: int = 42
  num_steps_per_env: int = 24
  max_iterations: int = 300
  obs_groups: dict = field(default_factory=lambda: {"policy": ("policy",), "critic": ("critic",)})
  save_interval: int = 50
  experiment_name: str = "exp1"
  run_name: str = ""
  logger: Literal["wandb", "tensorboard"] = "wandb"
  wandb_project: str = "mjlab"
  wandb_tags: Tuple[str, ...] = ()
  resume: bool = False
  load_run: str = ".*"
  load_checkpoint: str = "model_.*.pt"
  clip_actions: float | None = None


@dataclass
class RslRlOnPolicyRunnerCfg(RslRlBaseRunnerCfg):
  class_name: str = "OnPolicyRunner"
  policy: RslRlPpoActorCriticCfg = field(default_factory=RslRlPpoActorCriticCfg)
  algorithm: RslRlPpoAlgorithmCfg = field(default_factory=RslRlPpoAlgorithmCfg)


# ---------------------------------------------------------------------------- task configs
def _ppo(actor=(512, 256, 128), critic=(512, 256, 128), norm=True, entropy=0.01, epochs=5,
         lr=1.0e-3, gamma=0.99, value_coef=1.0, name="exp", save=50, iters=30_000):
  return RslRlOnPolicyRunnerCfg(
    policy=RslRlPpoActorCriticCfg(init_noise_std=1.0, actor_obs_normalization=norm,
                                  critic_obs_normalization=norm, actor_hidden_dims=actor,
                                  critic_hidden_dims=critic, activation="elu"),
    algorithm=RslRlPpoAlgorithmCfg(value_loss_coef=value_coef, use_clipped_value_loss=True,
                                   clip_param=0.2, entropy_coef=entropy,
                                   num_learning_epochs=epochs, num_mini_batches=4,
                                   learning_rate=lr, schedule="adaptive", gamma=gamma, lam=0.95,
                                   desired_kl=0.01, max_grad_norm=1.0),
    experiment_name=name, save_interval=save, num_steps_per_env=24, max_iterations=iters)


def unitree_g1_ppo_runner_cfg():
  """`tasks/velocity/config/g1/rl_cfg.py:10-39`."""
  return _ppo(name="g1_velocity")


def unitree_go1_ppo_runner_cfg():
  """`tasks/velocity/config/go1/rl_cfg.py`: no observation normalisation, 10k iterations."""
  return _ppo(norm=False, name="go1_velocity", iters=10_000)


def unitree_g1_tracking_ppo_runner_cfg():
  """`tasks/tracking/config/g1/rl_cfg.py`: entropy 0.005, save every 500."""
  return _ppo(entropy=0.005, name="g1_tracking", save=500)


def unitree_g1_jump_ppo_cfg():
  """`tasks/jump/config/g1/rl_cfg.py`: smaller actor, 6 epochs, lr 3e-4, gamma 0.98,
  value coefficient 2, entropy 0.015, 1000 iterations as the reference currently ships."""
  return _ppo(actor=(256, 128, 64), entropy=0.015, epochs=6, lr=3e-4, gamma=0.98, value_coef=2.0,
              name="g1_jump", save=100, iters=1000)


RL_CFGS = {
  "Mjlab-Velocity-Flat-Unitree-G1": unitree_g1_ppo_runner_cfg,
  "Mjlab-Velocity-Flat-Unitree-Go1": unitree_go1_ppo_runner_cfg,
  "Mjlab-Tracking-Flat-Unitree-G1": unitree_g1_tracking_ppo_runner_cfg,
  "Mjlab-Jump-Flat-Unitree-G1": unitree_g1_jump_ppo_cfg,
  "Mjlab-Jump-Hfield-Unitree-G1": unitree_g1_jump_ppo_cfg,
}


def load_rl_cfg(task: str) -> RslRlOnPolicyRunnerCfg:
  if task not in RL_CFGS:
    raise KeyError(f"no RL config for {task}; available: {sorted(RL_CFGS)}")
  return RL_CFGS[task]()
