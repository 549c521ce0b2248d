"""Config 1 of BASELINE.json through the product: `Mjlab-Velocity-Flat-Unitree-G1` at
num_envs = 1 with zero actions (the reference's `play.py --agent zero`,
`src/mjlab/scripts/play.py:161-178`), eager and HIP-graph captured, every physics substep
shadowed on the fp64 oracle with the rollout parity test's checks (`_check_step`).

A one-world sim is where the engine's single-world edge cases live: the Newton row classes
classify one world, the task kernels' cross-env reductions (`k_accum`) run one block over one
env, and no batch split applies.  Besides the per-substep oracle checks:
  - the captured env step's physics equals `decimation` single `Simulation.step` calls bit
    for bit (qpos, qacc_warmstart, time; qvel except the root's planar velocity an interval
    push wrote after the physics);
  - the env's episode logs stay finite and the engine drops no contact.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

import oracle_lib as ol
from parity_util import diff_detail, differing_outputs, output_snapshot
from parity_util import expanded_fields, world_model
from test_gpu_rollout_parity import _OUT, _STATE, _check_step, _snap, write_stats

pytestmark = pytest.mark.gpu

TASK = "Mjlab-Velocity-Flat-Unitree-G1"
NSTEPS = 200


def _stats():
  return dict(checked=0, ties=0, heavy_checked=0, max_nefc=0, qacc_ratio=0.0, qacc_abs=0.0,
              qacc_rel_world=0.0, qvel_ratio=0.0, sens_ratio=0.0, qacc_worst=[], niter_maxdiff=0,
              capped=0, qpos_ratio=0.0, qacc_energy_rel=0.0, cost_gap_fp32=-1.0,
              qacc_fp32_ratio=0.0, qacc_fp32_ratio_p99=[], in_model=0, out_of_model=[],
              per_dof_within=0, e2e_qvel_abs=0.0, e2e_qpos_abs=0.0, niter_equal=0)


def _shadow(sim, m, st0, st1, out, stats, where):
  """One substep (GPU state st0 -> st1, outputs `out`) against the oracle's step from st0."""
  ref = ol.forward(m, st0["qpos"][0], st0["qvel"][0], st0["qacc_warmstart"][0], st0["ctrl"][0],
                   float(st0["time"][0].reshape(-1)[0]), step=True, nconmax=sim.nconmax,
                   njmax=sim.njmax)
  assert not ref["overflow"]
  _check_step(m, ref, st0, st1, out, 0, stats, where, sim)


def _env(device):
  from mjlab_amd.envs import make_env
  env = make_env(TASK, num_envs=1, device=device, seed=42)
  assert env.num_envs == 1 and env.sim.num_envs == 1
  env.reset()
  return env


def _assert_clean(env, stats, name):
  write_stats(name, stats)
  ev = env.sim.overflow_events().cpu().tolist()
  assert ev == [0, 0, 0], f"contacts dropped / unsupported pairs in the one-world run: {ev}"
  for k, v in env.extras.get("log", {}).items():
    if isinstance(v, torch.Tensor):
      assert torch.isfinite(v).all(), f"extras['log'][{k!r}] not finite"
  assert stats["checked"] >= 0.95 * 4 * NSTEPS, stats
  assert stats["niter_equal"] >= 0.8 * stats["checked"]
  assert not stats["out_of_model"], stats["out_of_model"][:5]  # no world-step outside the fp32 model


def test_config1_eager_every_substep(gpu_device):
  """The reference-style eager env.step at one world: every `Simulation.step` of 200 env
  steps (800 substeps) shadowed on the oracle."""
  env = _env(gpu_device)
  sim = env.sim
  fields = expanded_fields(sim)
  assert "geom_friction" in fields  # startup friction randomisation reaches the one world
  sel = np.array([0])
  m = world_model(sim, 0, fields)
  stats = _stats()
  real_step = sim.step
  count = {"n": 0}

  def shadowed(nsubstep=1):
    assert nsubstep == 1
    torch.cuda.synchronize()
    st0 = _snap(sim, sel, _STATE)
    real_step()
    torch.cuda.synchronize()
    st1, out = _snap(sim, sel, _STATE), _snap(sim, sel, _OUT)
    _shadow(sim, m, st0, st1, out, stats, f"eager substep {count['n']}")
    count["n"] += 1

  sim.step = shadowed
  zero = torch.zeros(1, env.action_manager.total_action_dim, device=gpu_device)
  try:
    for _ in range(NSTEPS):
      env.step(zero)
  finally:
    sim.step = real_step
  assert count["n"] == 4 * NSTEPS
  _assert_clean(env, stats, "config1_eager")


def test_config1_captured_every_substep(gpu_device):
  """The HIP-graph-captured fused env step at one world.  Around every replay the pre-step
  state is restored and the same physics re-run as `decimation` single steps, each shadowed
  on the oracle; the single steps must reproduce the graph's physics bit for bit."""
  env = _env(gpu_device)
  env.enable_graph(capture=True)
  assert env._fused is not None, getattr(env, "_fused_unsupported", "")
  sim, d = env.sim, env.sim.data
  fields = expanded_fields(sim)
  sel = np.array([0])
  m = world_model(sim, 0, fields)
  dec = env.cfg.decimation
  air = env.scene["feet_ground_contact"]._air
  keys = ("qpos", "qvel", "qacc_warmstart", "time")
  stats = _stats()
  zero = torch.zeros(1, env.action_manager.total_action_dim, device=gpu_device)
  pushed = 0
  for k in range(NSTEPS):
    torch.cuda.synchronize()
    s0 = {n: getattr(d, n).clone() for n in keys}
    a0 = {n: t.clone() for n, t in air.items()}
    env.step(zero)
    torch.cuda.synchronize()
    s1 = {n: getattr(d, n).clone() for n in keys}
    a1 = {n: t.clone() for n, t in air.items()}
    o1 = output_snapshot(sim)
    reset = bool((env.episode_length_buf == 0).any())
    # re-run this env step's physics from the pre-step state as single steps (ctrl holds the
    # value the graph's action kernel wrote for all of its substeps)
    for n in keys:
      getattr(d, n).copy_(s0[n])
    for n, t in air.items():
      t.copy_(a0[n])
    for j in range(dec):
      torch.cuda.synchronize()
      st0 = _snap(sim, sel, _STATE)
      sim.step()
      torch.cuda.synchronize()
      _shadow(sim, m, st0, _snap(sim, sel, _STATE), _snap(sim, sel, _OUT), stats,
              f"captured step {k} substep {j}")
    if not reset:
      assert torch.equal(d.qpos, s1["qpos"]), f"step {k}: graph physics != single steps (qpos)"
      assert torch.equal(d.qacc_warmstart, s1["qacc_warmstart"]), f"step {k}: qacc_warmstart"
      assert torch.equal(d.time, s1["time"]), f"step {k}: time"
      same_xy = torch.equal(d.qvel[:, :2], s1["qvel"][:, :2])
      pushed += int(not same_xy)
      if same_xy:
        assert torch.equal(d.qvel[:, 2:], s1["qvel"][:, 2:]), f"step {k}: qvel"
      else:
        # a push (push_by_setting_velocity, events.py:209-223) rewrites the whole root twist
        # from root_link_vel_w -- read from cvel, i.e. the velocity before the last substep's
        # integration, as in the reference -- plus the kick: only the joints compare
        assert torch.equal(d.qvel[:, 6:], s1["qvel"][:, 6:]), f"step {k}: joint qvel after a push"
      for n in ("current_air_time", "last_air_time", "current_contact_time", "last_contact_time"):
        assert torch.equal(air[n], a1[n]), f"step {k}: engine air time {n}"
      # every other mjData output the graph's last substep wrote (frames, velocities,
      # subtree quantities, sites, geoms, forces, contacts, sensors, counters): the
      # post-physics managers write only qvel (a push), compared above
      bad = differing_outputs(o1, output_snapshot(sim))
      bad.pop("qvel", None)
      assert not bad, f"step {k}: graph step outputs != single steps in {bad}: {diff_detail(o1, output_snapshot(sim), bad)}"
    # continue the graph's trajectory (post-physics events and resets included)
    for n in keys:
      getattr(d, n).copy_(s1[n])
    for n, t in air.items():
      t.copy_(a1[n])
  # interval pushes every U(1, 3) s: several land in 200 env steps (4 s)
  assert pushed >= 1
  _assert_clean(env, stats, "config1_captured")
