"""Batch split (engine.hip launch_step): models without Newton row
classes run large batches as concurrent world ranges on their own streams.  Worlds are
independent, so every split count must give results bit-identical to one launch set, eager
and under HIP graph capture, across fused substeps.

MJX355_SPLIT (read at Simulation creation) pins the split count; MJX355_ROW_CLASSES=""
turns the row classes off so the G1 scene can split too.
"""

import os

import numpy as np
import pytest
import torch

from parity_util import g1_states

pytestmark = pytest.mark.gpu

FIELDS = ("qpos", "qvel", "qacc", "qfrc_constraint", "nefc", "solver_niter", "sensordata")


def _make(env, n, device):
  from mjlab_amd.scenes import load_scene
  from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
  old = {k: os.environ.get(k) for k in env}
  os.environ.update(env)
  try:
    m = load_scene("g1_velocity")
    cfg = SimulationCfg(nconmax=48, njmax=160,
                        mujoco=MujocoCfg(timestep=m.timestep, iterations=10, ls_iterations=20))
    sim = Simulation(n, cfg, m, device)
  finally:
    for k, v in old.items():
      if v is None:
        os.environ.pop(k, None)
      else:
        os.environ[k] = v
  return sim


def _load(sim, q, qv, ctrl):
  d = sim.data
  d.qpos[:] = torch.as_tensor(q, dtype=torch.float32)
  d.qvel[:] = torch.as_tensor(qv, dtype=torch.float32)
  d.ctrl[:] = torch.as_tensor(ctrl, dtype=torch.float32)
  d.qacc_warmstart[:] = 0


def _snap(sim):
  torch.cuda.synchronize()
  return {k: getattr(sim.data, k).cpu().numpy().copy() for k in FIELDS}


def _run(split, q, qv, ctrl, device, graph=False):
  sim = _make({"MJX355_SPLIT": str(split), "MJX355_ROW_CLASSES": ""}, q.shape[0], device)
  _load(sim, q, qv, ctrl)
  out = []
  if graph:
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
      sim.step(nsubstep=3)
    _load(sim, q, qv, ctrl)  # capture does not run the step
    for _ in range(2):
      g.replay()
      out.append(_snap(sim))
  else:
    for _ in range(2):
      sim.step(nsubstep=3)
      out.append(_snap(sim))
  return out


def test_split_bit_identical(gpu_device):
  from mjlab_amd.scenes import load_scene
  n = 97  # ragged ranges
  q, qv, ctrl = g1_states(load_scene("g1_velocity"), n, seed=21)
  base = _run(1, q, qv, ctrl, gpu_device)
  for split, graph in ((2, False), (3, False), (4, False), (2, True), (1, True)):
    got = _run(split, q, qv, ctrl, gpu_device, graph=graph)
    for a, b in zip(base, got):
      for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=f"split={split} graph={graph} field {k}")


def _run_env(env, q, qv, ctrl, device, graph, nsub=3, reps=2):
  sim = _make(env, q.shape[0], device)
  _load(sim, q, qv, ctrl)
  out = []
  if graph:
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
      sim.step(nsubstep=nsub)
    _load(sim, q, qv, ctrl)
  for _ in range(reps):
    if graph:
      g.replay()
    else:
      sim.step(nsubstep=nsub)
    out.append(_snap(sim))
  return out


@pytest.mark.parametrize("classes", ["24", "24,60"])
def test_split_with_row_classes(classes, gpu_device):
  """Batch split x Newton row classes (each split forks its own class streams and joins
  them back, SideStream in engine.h): eager and HIP-graph-captured multi-substep steps,
  split 2 and 3, bit-identical to one split.  Worlds with rows above every class capacity
  must be present so the full-capacity class runs too."""
  from mjlab_amd.scenes import load_scene
  n = 131  # ragged ranges
  q, qv, ctrl = g1_states(load_scene("g1_velocity"), n, seed=22)
  base = _run_env({"MJX355_ROW_CLASSES": classes, "MJX355_SPLIT": "1"}, q, qv, ctrl, gpu_device, False)
  cap = max(int(c) for c in classes.split(","))
  assert (base[0]["nefc"] > cap).any() and (base[0]["nefc"] <= 24).any()
  for split, graph in ((2, False), (2, True), (3, True), (1, True)):
    got = _run_env({"MJX355_ROW_CLASSES": classes, "MJX355_SPLIT": str(split)}, q, qv, ctrl,
                   gpu_device, graph)
    for a, b in zip(base, got):
      for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=f"split={split} graph={graph} field {k}")
