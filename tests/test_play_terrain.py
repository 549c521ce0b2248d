"""Play mode of the rough velocity tasks on CPU (`tasks/velocity/config/g1/env_cfgs.py:
131-148`, go1 likewise; `envs/mdp/events.py:26-37`; `terrains/terrain_importer.py:203-222`):
the random-layout 5 x 5 box-stair grid with a 10 m border, and the `randomize_terrain` reset
event that puts each resetting env on a random sub-terrain (level row and type column)."""

import numpy as np
import torch

from mjlab_amd import mdp
from mjlab_amd import terrains as T
from mjlab_amd.envs import load_env_cfg
from mjlab_amd.scene import Terrain
from mjlab_amd.scenes import load_scene


def test_play_configs():
  for task in ("Mjlab-Velocity-Rough-Unitree-G1", "Mjlab-Velocity-Rough-Unitree-Go1"):
    cfg = load_env_cfg(task, play=True)
    tg = cfg.scene.terrain.terrain_generator
    assert (tg.num_rows, tg.num_cols, tg.border_width, tg.curriculum) == (5, 5, 10.0, False)
    ev = cfg.events["randomize_terrain"]
    assert ev.func is mdp.randomize_terrain and ev.mode == "reset" and ev.params == {}
    assert "push_robot" not in cfg.events and not cfg.observations["policy"].enable_corruption
    assert cfg.episode_length_s == int(1e9)
    train = load_env_cfg(task, play=False)
    assert "randomize_terrain" not in train.events
    tg = train.scene.terrain.terrain_generator
    assert (tg.num_rows, tg.num_cols, tg.border_width, tg.curriculum) == (10, 20, 20.0, True)


def test_play_grid_is_random_layout():
  cfg = T.rough_terrains_cfg(seed=0, curriculum=False, num_rows=5, num_cols=5, border_width=10.0)
  assert not cfg.curriculum and (cfg.num_rows, cfg.num_cols, cfg.border_width) == (5, 5, 10.0)
  geoms, origins = T.TerrainGenerator(cfg).generate()
  assert origins.shape == (5, 5, 3)
  m = load_scene("g1_velocity_rough_play")
  np.testing.assert_allclose(m.arrays["terrain_origins"], origins)
  # curriculum layout: difficulty grows with the row; random layout: it does not have to --
  # the stair heights (spawn z of the stair patches) are not sorted by row
  cur_geoms, cur_origins = T.TerrainGenerator(T.rough_terrains_cfg(
    seed=0, curriculum=True, num_rows=5, num_cols=5, border_width=10.0)).generate()
  assert not np.array_equal(origins, cur_origins)


def _terrain(n=512, rows=5, cols=5):
  origins = np.zeros((rows, cols, 3))
  origins[..., 0] = np.arange(rows)[:, None] * 8.0
  origins[..., 1] = np.arange(cols)[None, :] * 8.0
  return Terrain(origins, (8.0, 8.0), n, "cpu", max_init_terrain_level=None)


def test_randomize_env_origins_eager_and_masked():
  torch.manual_seed(0)
  t = _terrain()
  ids = torch.arange(0, 512, 2)
  keep = t.env_origins[1::2].clone()
  t.randomize_env_origins(ids)
  lv, ty = t.terrain_levels[ids], t.terrain_types[ids]
  assert int(lv.min()) == 0 and int(lv.max()) == 4 and int(ty.min()) == 0 and int(ty.max()) == 4
  torch.testing.assert_close(t.env_origins[ids], t.terrain_origins[lv, ty])
  torch.testing.assert_close(t.env_origins[1::2], keep)
  # masked form: the unmasked envs keep level, type and origin
  t2 = _terrain()
  mask = torch.zeros(512, dtype=torch.bool)
  mask[::3] = True
  before = (t2.terrain_levels.clone(), t2.terrain_types.clone(), t2.env_origins.clone())
  t2.randomize_env_origins_masked(mask)
  for a, b in zip((t2.terrain_levels, t2.terrain_types, t2.env_origins), before):
    assert torch.equal(a[~mask], b[~mask])
  m_lv, m_ty = t2.terrain_levels[mask], t2.terrain_types[mask]
  torch.testing.assert_close(t2.env_origins[mask], t2.terrain_origins[m_lv, m_ty])
  # every column is reachable (the curriculum start puts type by env block; play does not)
  assert len(torch.unique(m_ty)) == 5 and len(torch.unique(m_lv)) == 5


def test_randomize_terrain_event_on_scene():
  class _Env:
    num_envs, device = 64, "cpu"

    class scene:  # noqa: N801
      terrain = _terrain(64)
  torch.manual_seed(1)
  env = _Env()
  mdp.randomize_terrain(env, torch.arange(10))
  t = env.scene.terrain
  torch.testing.assert_close(t.env_origins[:10], t.terrain_origins[t.terrain_levels[:10], t.terrain_types[:10]])
  mask = torch.zeros(64, dtype=torch.bool)
  mask[20:30] = True
  mdp.randomize_terrain.masked(env, mask)
  torch.testing.assert_close(t.env_origins[20:30],
                             t.terrain_origins[t.terrain_levels[20:30], t.terrain_types[20:30]])
