"""Per-world engine capacity (sim.world_capacity): the default 48-contact / 160-row carve,
the tracking task's 56 / 200 fast carve under the reference's njmax (250 rows,
`tasks/tracking/tracking_env_cfg.py:307-308`) as its max capacity, and the specialised kernels' table
(specs.inc) carrying the same capacities, so the bench configs never fall back to the
generic kernels."""
import os
import re

import pytest

from mjlab_amd.scenes import load_scene
from mjlab_amd.sim.sim import SimulationCfg, max_capacity, world_capacity

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_default_capacity_clamps_to_the_fast_carve():
  m = load_scene("g1_velocity")
  assert world_capacity(SimulationCfg(nconmax=35, njmax=300), m) == (48, 160)
  assert world_capacity(SimulationCfg(), m) == (48, 160)
  assert world_capacity(SimulationCfg(njmax=100), m) == (48, 100)


def test_tracking_holds_the_reference_njmax():
  from mjlab_amd.tracking import make_tracking_env_cfg
  cfg = make_tracking_env_cfg()
  assert cfg.sim.njmax == 250 and cfg.sim.engine_capacity == (56, 200)
  assert world_capacity(cfg.sim, load_scene("g1_tracking")) == (56, 200)


def test_engine_capacity_bounds():
  m = load_scene("g1_velocity")
  with pytest.raises(ValueError):
    world_capacity(SimulationCfg(engine_capacity=(65, 160)), m)
  with pytest.raises(ValueError):
    world_capacity(SimulationCfg(engine_capacity=(48, 300)), m)


def test_max_capacity_is_the_resolve_carve(monkeypatch):
  """An overflowing world is re-solved at njmax rows and as many contacts (every contact makes
  a row; the reference pools nconmax, sim/sim.py:82-93), at most MAX_CONTACTS; with njmax
  unset, the rows 64 pyramidal contacts and every joint limit make.  MJX355_RESOLVE=0 turns
  the re-solve off."""
  from mjlab_amd.sim.sim import MAX_CONTACTS
  g1, go1 = load_scene("g1_velocity"), load_scene("go1_velocity")
  cfg = SimulationCfg(nconmax=35, njmax=300)
  assert max_capacity(cfg, g1) == (300, 300)
  assert max_capacity(cfg, go1) == (300, 300)
  assert max_capacity(SimulationCfg(), g1) == (4 * 64 + 2 * 29, 4 * 64 + 2 * 29)
  assert max_capacity(SimulationCfg(njmax=100), g1) == (100, 100)
  assert max_capacity(SimulationCfg(njmax=2000), g1) == (MAX_CONTACTS, 2000)
  from mjlab_amd.tracking import make_tracking_env_cfg
  assert max_capacity(make_tracking_env_cfg().sim, load_scene("g1_tracking")) == (250, 250)
  monkeypatch.setenv("MJX355_RESOLVE", "0")
  assert max_capacity(cfg, g1) == (48, 160)


def test_specs_carry_the_task_capacities():
  text = open(os.path.join(ROOT, "mjlab-1_amd", "csrc", "specs.inc")).read()
  caps = {}
  for mm in re.finditer(r"^MJX_SPEC\(\d+, (\w+),.*, (\d+), (\d+)\)$", text, re.M):
    caps.setdefault(mm.group(1), []).append((int(mm.group(2)), int(mm.group(3))))
  assert caps["g1_tracking"] == [(56, 200), (48, 160), (250, 250)]
  for name in ("g1_velocity", "g1_jump", "g1_velocity_rough", "g1_jump_hfield"):
    assert caps[name] == [(48, 160), (300, 300)], name
  # Go1: its tasks' engine_capacity first (flat 16 / 64, rough 24 / 96), the default and the
  # max carve
  from mjlab_amd.envs import unitree_go1_flat_env_cfg, unitree_go1_rough_env_cfg
  for name, make, cap in (("go1_velocity", unitree_go1_flat_env_cfg, (16, 64)),
                          ("go1_velocity_rough", unitree_go1_rough_env_cfg, (24, 96))):
    assert caps[name] == [cap, (48, 160), (300, 300)], name
    sim, go1 = make().sim, load_scene(name)
    assert world_capacity(sim, go1) == cap
    assert max_capacity(sim, go1) == (300, 300)
