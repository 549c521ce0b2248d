"""The fast LDS carve and the max-capacity carve compute the same substep, bit for bit, for a
world that fits both.

The engine runs every substep in the fast carve (48 contacts / 160 rows for G1) and re-solves a
world that overflows it in the max carve (the reference's njmax, DESIGN.md section 3 "Overflow
re-solve"); the masked forward (the reset worlds) runs in the max carve too.  A world's
arithmetic must not depend on which carve held it: the fused env step and single steps may
place a world differently (a re-solved world's later substeps), and the rollout parity tests
require them to agree bit for bit.  Here `forward()` over every world (fast carve, the Newton
row classes) is compared with `forward(mask=all)` (one max-carve A -> B -> C launch,
step_masked) from the same state, over every mjData output."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from parity_util import DATA_FIELDS, diff_detail, differing_outputs

pytestmark = pytest.mark.gpu

_STATE = ("qpos", "qvel", "qacc_warmstart", "ctrl", "time")


@pytest.mark.parametrize("task,n", [("Mjlab-Velocity-Flat-Unitree-G1", 1024),
                                    ("Mjlab-Velocity-Flat-Unitree-Go1", 1024),
                                    ("Mjlab-Tracking-Flat-Unitree-G1", 512)])
def test_fast_and_max_carve_agree(task, n, gpu_device):
  from mjlab_amd.envs import make_env
  env = make_env(task, num_envs=n, device=gpu_device, seed=3)
  gen = torch.Generator(device=gpu_device)
  gen.manual_seed(3)
  nact = env.action_manager.total_action_dim
  env.reset()
  env.enable_graph(capture=True)
  for _ in range(30):  # contact-rich states: feet landing, stumbles
    env.step(2.0 * torch.rand((n, nact), device=gpu_device, generator=gen) - 1.0)
  torch.cuda.synchronize()
  sim = env.sim
  assert sim.info()["resolve_list"] > 0, "no max carve wired"
  d = sim.data
  s0 = {k: getattr(d, k).clone() for k in _STATE}
  sim.forward()
  torch.cuda.synchronize()
  fast = {k: getattr(d, k).clone() for k in DATA_FIELDS}
  for k, v in s0.items():
    getattr(d, k).copy_(v)
  sim.forward(mask=torch.ones(n, dtype=torch.bool, device=d.qpos.device))
  torch.cuda.synchronize()
  big = {k: getattr(d, k).clone() for k in DATA_FIELDS}
  c, r = sim.fast_capacity
  over = ((fast["ncon"].reshape(-1) > c) | (fast["nefc"].reshape(-1) > r))
  assert not bool(over.any()), "a world overflowed the fast carve (it would be re-solved)"
  bad = differing_outputs(fast, big)
  assert not bad, f"fast carve != max carve in {bad}: {diff_detail(fast, big, bad)}"
  assert int(fast["nefc"].max()) > 0
