"""Learner side: the rsl_rl PPO stack the reference trains
with (`src/mjlab/rl/*`, rsl-rl-lib 3.1.0), restated on torch for the MI355X env step."""

from .config import (RL_CFGS, RslRlBaseRunnerCfg, RslRlOnPolicyRunnerCfg, RslRlPpoActorCriticCfg,
                     RslRlPpoAlgorithmCfg, load_rl_cfg)
from .ppo import PPO, ActorCritic, EmpiricalNormalization, RolloutStorage
from .runner import OnPolicyRunner
from .vecenv_wrapper import RslRlVecEnvWrapper

__all__ = ["RL_CFGS", "RslRlBaseRunnerCfg", "RslRlOnPolicyRunnerCfg", "RslRlPpoActorCriticCfg",
           "RslRlPpoAlgorithmCfg", "load_rl_cfg", "PPO", "ActorCritic", "EmpiricalNormalization",
           "RolloutStorage", "OnPolicyRunner", "RslRlVecEnvWrapper"]
