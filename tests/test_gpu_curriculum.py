"""Curricula under the graph-captured sync-free step.

The jump task's curricula (`tasks/jump/mdp/curriculums.py:37-97`) change the command's
target_height / height_tolerance and the landing_stability reward weight.  The captured
step bakes both in as host constants, so advancing past a stage must re-record the graph
and the next replay must use the new values.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _jump_env(gpu_device, n=64):
  from mjlab_amd.envs import make_env
  env = make_env("Mjlab-Jump-Flat-Unitree-G1", num_envs=n, device=gpu_device, seed=3)
  env.reset()
  env.enable_graph(capture=True)
  return env


def _step(env, g, n):
  nact = env.action_manager.total_action_dim
  a = 0.1 * (2 * torch.rand(n, nact, device=env.device, generator=g) - 1)
  return env.step(a)


def test_jump_curriculum_rerecords_graph(gpu_device):
  n = 64
  env = _jump_env(gpu_device, n)
  g = torch.Generator(device=gpu_device).manual_seed(0)
  for _ in range(3):
    _step(env, g, n)
  torch.cuda.synchronize()
  cmd = env.command_manager.get_term("jump")
  assert cmd.cfg.target_height == pytest.approx(0.10)
  assert torch.allclose(cmd.metrics["target_height"], torch.full_like(cmd.metrics["target_height"], 0.10))
  graph0 = env._graph
  # jump past height stage 2 (10000*24) and stability stage 2 (15000*24)
  env.common_step_counter = 16000 * 24
  # force a time-out reset of every env in the next step, so every env resamples
  env.episode_length_buf.fill_(env.max_episode_length)
  _step(env, g, n)
  torch.cuda.synchronize()
  assert env._graph is not graph0, "curriculum change must re-record the step graph"
  assert cmd.cfg.target_height == pytest.approx(0.15)
  assert env.reward_manager.get_term_cfg("landing_stability").weight == pytest.approx(2.5)
  assert torch.allclose(cmd.metrics["target_height"], torch.full_like(cmd.metrics["target_height"], 0.15))
  assert torch.allclose(cmd.height_command, torch.full_like(cmd.height_command, 0.15))
  # replays after the re-record keep the new stage
  graph1 = env._graph
  _step(env, g, n)
  torch.cuda.synchronize()
  assert env._graph is graph1
  assert torch.allclose(cmd.metrics["target_height"], torch.full_like(cmd.metrics["target_height"], 0.15))


def test_reward_weight_change_reaches_replay(gpu_device):
  """A weight changed between replays (as a curriculum does) is used by the next step:
  `alive` (is_alive, always 1 for live envs) reports exactly its new weight."""
  n = 64
  env = _jump_env(gpu_device, n)
  g = torch.Generator(device=gpu_device).manual_seed(1)
  for _ in range(2):
    _step(env, g, n)
  rm = env.reward_manager
  k = rm._term_names.index("alive")
  torch.cuda.synchronize()
  live = ~(env.reset_terminated | env.reset_time_outs)
  assert torch.allclose(rm._step_reward[live, k], torch.full_like(rm._step_reward[live, k], 0.5))
  rm.get_term_cfg("alive").weight = 1.75
  _step(env, g, n)
  torch.cuda.synchronize()
  live = ~(env.reset_terminated | env.reset_time_outs)
  assert live.any()
  assert torch.allclose(rm._step_reward[live, k], torch.full_like(rm._step_reward[live, k], 1.75))
