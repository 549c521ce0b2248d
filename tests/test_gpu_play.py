"""Play mode of the rough velocity tasks on the GPU (`tasks/velocity/config/g1/env_cfgs.py:
131-148`): the random-layout 5 x 5 terrain grid and the `randomize_terrain` reset event,
through the graph-captured sync-free env step.  Forced resets must put every resetting env
on the origin of a random sub-terrain (all 5 columns reached, not the curriculum's type per
env block); reset_base, which the reference cfg lists first, placed the root about the
origin the terrain-level curriculum had chosen."""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("task", ["Mjlab-Velocity-Rough-Unitree-G1", "Mjlab-Velocity-Rough-Unitree-Go1"])
def test_play_rough_randomizes_terrain(task, gpu_device):
  from mjlab_amd.envs import make_env
  n = 256
  env = make_env(task, num_envs=n, device=gpu_device, seed=5, play=True)
  env.reset()
  env.enable_graph(capture=True)
  t = env.scene.terrain
  types0 = t.terrain_types.clone()
  nact = env.action_manager.total_action_dim
  g = torch.Generator(device=gpu_device).manual_seed(0)
  for _ in range(3):
    env.step(0.1 * (2 * torch.rand(n, nact, device=gpu_device, generator=g) - 1))
  env.episode_length_buf.fill_(env.max_episode_length - 1)  # everyone resets next step
  env.step(torch.zeros(n, nact, device=gpu_device))
  torch.cuda.synchronize()
  assert (env.episode_length_buf == 0).all()
  lv, ty = t.terrain_levels, t.terrain_types
  assert len(torch.unique(ty)) == 5 and len(torch.unique(lv)) == 5
  assert not torch.equal(ty, types0)
  torch.testing.assert_close(t.env_origins, t.terrain_origins[lv, ty])
  # reset_base runs before randomize_terrain (event order of the reference cfg), so each
  # root sits within the reset pose range about a sub-terrain origin -- the one the
  # terrain-level curriculum chose -- while env_origins already holds the next one
  root = env.scene["robot"].data.root_link_pos_w[:, :2]
  grid = t.terrain_origins.reshape(-1, 3)[:, :2]
  d = (root[:, None, :] - grid[None, :, :]).abs().amax(dim=-1).amin(dim=1)
  assert float(d.max()) <= 0.5 + 1e-3
  assert torch.isfinite(env.sim.data.qpos).all()
