"""Per-world engine capacity (sim.world_capacity): the default 48-contact / 160-row carve,
the tracking task's engine_capacity holding the reference's njmax (250 rows,
`tasks/tracking/tracking_env_cfg.py:307-308`), and the specialised kernels' table
(specs.inc) carrying the same capacities, so the bench configs never fall back to the
generic kernels."""
import os
import re

import pytest

from mjlab_amd.scenes import load_scene
from mjlab_amd.sim.sim import SimulationCfg, world_capacity

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_default_capacity_clamps_to_the_fast_carve():
  m = load_scene("g1_velocity")
  assert world_capacity(SimulationCfg(nconmax=35, njmax=300), m) == (48, 160)
  assert world_capacity(SimulationCfg(), m) == (48, 160)
  assert world_capacity(SimulationCfg(njmax=100), m) == (48, 100)


def test_tracking_holds_the_reference_njmax():
  from mjlab_amd.tracking import make_tracking_env_cfg
  cfg = make_tracking_env_cfg()
  assert cfg.sim.njmax == 250 and cfg.sim.engine_capacity == (64, 256)
  assert world_capacity(cfg.sim, load_scene("g1_tracking")) == (64, 250)


def test_engine_capacity_bounds():
  m = load_scene("g1_velocity")
  with pytest.raises(ValueError):
    world_capacity(SimulationCfg(engine_capacity=(65, 160)), m)
  with pytest.raises(ValueError):
    world_capacity(SimulationCfg(engine_capacity=(48, 300)), m)


def test_specs_carry_the_task_capacities():
  text = open(os.path.join(ROOT, "mjlab-1_amd", "csrc", "specs.inc")).read()
  caps = {mm.group(1): (int(mm.group(2)), int(mm.group(3))) for mm in
          re.finditer(r"^MJX_SPEC\(\d+, (\w+),.*, (\d+), (\d+)\)$", text, re.M)}
  assert caps["g1_tracking"] == (64, 250)
  assert caps["g1_velocity"] == caps["go1_velocity"] == caps["g1_jump"] == (48, 160)
