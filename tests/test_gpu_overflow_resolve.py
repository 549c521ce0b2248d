"""Overflow re-solve: a world whose contacts or constraint rows overflow the fast LDS carve
(48 contacts / 160 rows) in a substep is re-solved inside the same step at the max capacity
(njmax 300 rows on G1 and as many contacts: every contact makes a row), instead of dropping
contacts.

The reference pools its contact budget over worlds (`sim/sim.py:82-91`: nconmax is a
per-world *average*, one world may hold more) and its njmax bounds a world's rows: at the
velocity task's njmax=300 a world with more than 48 contacts -- more than 64 too -- loses
nothing there, and loses nothing here.  Two set-ups:
  - parity: a small fast carve (20 / 80) and G1 worlds standing up to 25 mm into the floor
    (14-28 contacts), so about half the worlds overflow it in physical states; every world
    is shadowed on the oracle at 300 / 300 substep by substep (the rollout-parity checks of
    test_gpu_rollout_parity.py), the re-solve counter equals the worlds that overflowed,
    nothing is dropped;
  - the task's own 48 / 160 carve with worlds placed at pelvis heights that give 40..64
    contacts and 160..256 rows (`_HEIGHTS`, measured on the oracle): the fused and
    graph-captured multi-substep step (the re-solve chain behind the full-capacity Newton
    class, joined before the next substep's classify) equals single steps bit for bit, also
    at the bench batch (where worlds pass 64 contacts: the max carve's multi-round contact
    passes, engine_impl.h kCon1), and the masked forward matches the oracle's contact counts.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

import oracle_lib as ol
from parity_util import diff_detail, differing_outputs, output_snapshot
from test_gpu_rollout_parity import _OUT, _STATE, _check_step, _snap, write_stats

pytestmark = pytest.mark.gpu

# pelvis height -> (contacts, rows) at the G1 keyframe pose, oracle at (64, 300) (round 4)
_HEIGHTS = {0.3: (40, 160), 0.2: (42, 168), 0.1: (49, 196), 0.0: (53, 212), -0.1: (60, 240),
            -0.3: (63, 252)}
NWORLD = 48
K = 3


def _stats():
  return dict(checked=0, ties=0, heavy_checked=0, max_nefc=0, qacc_ratio=0.0, qacc_abs=0.0,
              qacc_rel_world=0.0, qvel_ratio=0.0, qpos_abs=0.0, sens_ratio=0.0, qacc_worst=[],
              niter_maxdiff=0, capped=0, qpos_ratio=0.0, qacc_energy_rel=0.0, cost_gap_fp32=-1.0,
              qacc_fp32_ratio=0.0, qacc_fp32_ratio_p99=[], in_model=0, out_of_model=[],
              per_dof_within=0, e2e_qvel_abs=0.0, e2e_qpos_abs=0.0, niter_equal=0)


def _sim(device, n=NWORLD, engine_capacity=None):
  from mjlab_amd.envs import load_env_cfg
  from mjlab_amd.scenes import load_scene
  from mjlab_amd.sim import Simulation
  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  cfg.sim.engine_capacity = engine_capacity
  m = load_scene("g1_velocity")
  sim = Simulation(n, cfg.sim, m, device)
  return sim, m


# a fast carve of 20 contacts / 80 rows: G1 worlds standing 0-25 mm into the floor hold
# 14-28 contacts (56-112 rows), so about half of them overflow it -- physical states the
# rollout-parity bounds were made for (the deep placements below launch the robot)
SMALL = (20, 80)


def _place_standing(sim, m, seed):
  rng = np.random.default_rng(seed)
  n = sim.num_envs
  q = np.tile(np.asarray(m.key_qpos, float), (n, 1))
  q[:, 2] -= 0.005 * (np.arange(n) % 6)
  q[:, 7:] += rng.uniform(-0.05, 0.05, (n, m.nq - 7))
  d = sim.data
  d.qpos[:] = torch.as_tensor(q, dtype=torch.float32)
  d.qvel[:] = torch.as_tensor(rng.normal(0.0, 0.05, (n, m.nv)), dtype=torch.float32)
  d.qacc_warmstart.zero_()
  d.ctrl[:] = torch.as_tensor(np.asarray(m.key_qpos, float)[7:][None] + rng.uniform(-0.1, 0.1, (n, m.nu)),
                              dtype=torch.float32)


def _place(sim, m, seed):
  """World w at pelvis height list(_HEIGHTS)[w % 6], or the keyframe every 7th world, with
  small joint jitter and velocities."""
  rng = np.random.default_rng(seed)
  n = sim.num_envs
  q = np.tile(np.asarray(m.key_qpos, float), (n, 1))
  hs = list(_HEIGHTS)
  for w in range(n):
    if w % 7 != 6:
      q[w, 2] = hs[w % len(hs)]
  q[:, 7:] += rng.uniform(-0.05, 0.05, (n, m.nq - 7))
  v = rng.normal(0.0, 0.1, (n, m.nv))
  d = sim.data
  d.qpos[:] = torch.as_tensor(q, dtype=torch.float32)
  d.qvel[:] = torch.as_tensor(v, dtype=torch.float32)
  d.qacc_warmstart.zero_()
  d.ctrl[:] = torch.as_tensor(rng.uniform(-0.3, 0.3, (n, m.nu)), dtype=torch.float32)


def test_capacities(gpu_device):
  sim, _ = _sim(gpu_device, 4)
  assert sim.fast_capacity == (48, 160)
  assert (sim.nconmax, sim.njmax) == (300, 300)
  info = sim.info()
  assert (info["nconmax"], info["njmax"], info["nconmax_max"], info["njmax_max"]) == (48, 160, 300, 300)
  assert info["resolve_list"] > 0
  # both carves run the G1 kernels specialised for them (specs.inc), not the generic ones
  assert info["spec"] > 0 and info["spec_max"] > 0


def test_overflow_resolved_matches_oracle(gpu_device):
  """Worlds past a small fast carve re-solved at 300 / 300, shadowed on the oracle at 300 / 300."""
  sim, m = _sim(gpu_device, engine_capacity=SMALL)
  assert sim.fast_capacity == SMALL and (sim.nconmax, sim.njmax) == (300, 300)
  _place_standing(sim, m, 0)
  ev0 = sim.event_counts().clone()
  sel = np.arange(sim.num_envs)
  states = [_snap(sim, sel, _STATE)]
  outs = []
  overflowing = 0
  for _ in range(K):
    sim.step()
    torch.cuda.synchronize()
    states.append(_snap(sim, sel, _STATE))
    outs.append(_snap(sim, sel, _OUT))
    nc, ne = outs[-1]["ncon"].reshape(-1), outs[-1]["nefc"].reshape(-1)
    overflowing += int(((nc > SMALL[0]) | (ne > SMALL[1])).sum())
  ev = (sim.event_counts() - ev0).cpu().tolist()
  assert ev[:3] == [0, 0, 0], f"contacts dropped: {ev}"
  # one re-solve per world-substep whose contacts or rows overflowed the fast carve
  assert ev[3] == overflowing > K * NWORLD // 4, (ev, overflowing)
  st = sim.stats()
  assert st["resolved"] >= ev[3] and st["max_ncon"] > SMALL[0] and st["max_nefc"] > SMALL[1]
  stats = _stats()
  over_checked = 0
  for t in range(K):
    st0, st1, out = states[t], states[t + 1], outs[t]
    for w in sel:
      ref = ol.forward(m, st0["qpos"][w], st0["qvel"][w], st0["qacc_warmstart"][w], st0["ctrl"][w],
                       float(st0["time"][w].reshape(-1)[0]), step=True, nconmax=300, njmax=300)
      assert not ref["overflow"], f"world {w} substep {t}: the oracle overflows 300/300"
      before = stats["checked"]
      _check_step(m, ref, st0, st1, out, int(w), stats, f"world {w} substep {t}", sim)
      if stats["checked"] > before and (ref["ncon"] > SMALL[0] or ref["nefc"] > SMALL[1]):
        over_checked += 1
  write_stats("overflow_resolve", stats)
  assert stats["checked"] >= 0.8 * K * NWORLD, stats
  assert over_checked >= K * NWORLD // 4, over_checked
  assert stats["niter_equal"] >= 0.8 * stats["checked"]
  assert not stats["out_of_model"], stats["out_of_model"]  # no world-step outside the fp32 model


def _fused_vs_single(sim, nsub, graph):
  """One fused `nsub`-substep step (eager or graph-replayed) against `nsub` single steps from
  the same state: every mjData output (parity_util.DATA_FIELDS: frames, velocities, subtree
  quantities, sites, geoms, forces, contacts, sensors), the per-world counters and the event
  counts bit for bit."""
  d = sim.data
  s0 = {k: getattr(d, k).clone() for k in _STATE}
  ev0 = sim.event_counts().clone()
  if graph:
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
      sim.step(nsubstep=nsub)  # warm the launch path outside capture
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    for k, v in s0.items():
      getattr(d, k).copy_(v)
    ev0 = sim.event_counts().clone()
    with torch.cuda.graph(g):
      sim.step(nsubstep=nsub)
    for k, v in s0.items():
      getattr(d, k).copy_(v)
    ev0 = sim.event_counts().clone()
    g.replay()
  else:
    sim.step(nsubstep=nsub)
  torch.cuda.synchronize()
  fused = output_snapshot(sim)
  ev_f = (sim.event_counts() - ev0).cpu().tolist()
  for k, v in s0.items():
    getattr(d, k).copy_(v)
  ev1 = sim.event_counts().clone()
  for _ in range(nsub):
    sim.step()
  torch.cuda.synchronize()
  ev_s = (sim.event_counts() - ev1).cpu().tolist()
  single = output_snapshot(sim)
  bad = differing_outputs(fused, single)
  if bad:
    c, r = sim.fast_capacity
    over = (((d.ncon > c) | (d.nefc > r)).nonzero().flatten().tolist())
    print(f"differing fields (worlds): {bad}; overflowing after the steps: {over[:24]}")
  assert not bad, (f"{'graph' if graph else 'fused'} {nsub}-substep != single steps in {bad}: "
                   f"{diff_detail(fused, single, bad)}")
  assert ev_f == ev_s and ev_f[3] > 0, (ev_f, ev_s)
  return ev_f


@pytest.mark.parametrize("graph", [False, True])
def test_fused_substeps_with_resolve_equal_single_steps(graph, gpu_device):
  sim, m = _sim(gpu_device)
  _place(sim, m, 1)
  ev = _fused_vs_single(sim, 4, graph)
  assert ev[:3] == [0, 0, 0], ev


def test_large_batch_resolve(gpu_device):
  """The bench batch (4096 G1 worlds: row-class pipelines, several thousand worlds listed
  per substep, more than the re-solve grid): nothing dropped, fused == single steps."""
  sim, m = _sim(gpu_device, 4096)
  _place(sim, m, 2)
  ev = _fused_vs_single(sim, 4, graph=False)
  # nearly every world is re-solved, some past 64 contacts (round 4 dropped those: 18 of
  # ~10,500 re-solved world-substeps); nothing is dropped below the reference's njmax
  assert ev[3] > 2 * sim.num_envs and ev[:3] == [0, 0, 0], ev
  assert sim.stats()["max_ncon"] > 64


def test_masked_forward_at_max_capacity(gpu_device):
  """forward(mask) (the reset path) re-solves its overflowing worlds at the max capacity:
  their contacts and rows match the oracle's forward."""
  sim, m = _sim(gpu_device)
  _place(sim, m, 3)
  mask = torch.zeros(sim.num_envs, dtype=torch.bool, device=sim.data.qpos.device)
  mask[::2] = True
  sim.forward(mask)
  torch.cuda.synchronize()
  sel = np.flatnonzero(mask.cpu().numpy())
  out = _snap(sim, sel, ("ncon", "nefc", "qacc", "qpos", "qvel", "qacc_warmstart", "ctrl", "time"))
  seen_over = 0
  for i, w in enumerate(sel):
    ref = ol.forward(m, out["qpos"][i], out["qvel"][i], out["qacc_warmstart"][i], out["ctrl"][i],
                     float(out["time"][i].reshape(-1)[0]), step=False, nconmax=300, njmax=300)
    assert int(out["ncon"][i].reshape(-1)[0]) == ref["ncon"], f"world {w}"
    assert int(out["nefc"][i].reshape(-1)[0]) == ref["nefc"], f"world {w}"
    seen_over += int(ref["ncon"] > 48 or ref["nefc"] > 160)
  assert seen_over > 0
  ev = sim.overflow_events().cpu().tolist()
  assert ev == [0, 0, 0]


def test_split_batch_resolve_in_line(gpu_device):
  """A batch split (Go1 at 2,048 worlds: two ranges on their own streams, no row classes)
  runs the re-solve chain in line behind each range's phase C: with a 2-contact / 8-row fast
  carve every standing Go1 world overflows and is re-solved, nothing is dropped, the fused
  and graph-captured steps equal single steps bit for bit, and the re-solved worlds' contact
  counts match the oracle's."""
  from mjlab_amd.envs import load_env_cfg
  from mjlab_amd.scenes import load_scene
  from mjlab_amd.sim import Simulation
  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-Go1")
  cfg.sim.engine_capacity = (2, 8)
  m = load_scene("go1_velocity")
  sim = Simulation(2048, cfg.sim, m, gpu_device)
  assert sim.fast_capacity == (2, 8) and sim.info()["resolve_list"] > 0
  rng = np.random.default_rng(5)
  n = sim.num_envs
  q = np.tile(np.asarray(m.key_qpos, float), (n, 1))
  q[:, 2] -= 0.01 * (np.arange(n) % 4)
  q[:, 7:] += rng.uniform(-0.05, 0.05, (n, m.nq - 7))
  d = sim.data
  d.qpos[:] = torch.as_tensor(q, dtype=torch.float32)
  d.qvel[:] = torch.as_tensor(rng.normal(0.0, 0.05, (n, m.nv)), dtype=torch.float32)
  d.qacc_warmstart.zero_()
  d.ctrl[:] = torch.as_tensor(np.asarray(m.key_qpos, float)[7:][None].repeat(n, 0), dtype=torch.float32)
  for graph in (False, True):
    ev = _fused_vs_single(sim, 4, graph)
    assert ev[:3] == [0, 0, 0] and ev[3] > n, ev
  sel = np.arange(0, n, 97)
  out = _snap(sim, sel, ("ncon", "nefc", "qpos", "qvel", "qacc_warmstart", "ctrl", "time"))
  over = 0
  for i, w in enumerate(sel):
    ref = ol.forward(m, out["qpos"][i], out["qvel"][i], out["qacc_warmstart"][i], out["ctrl"][i],
                     float(out["time"][i].reshape(-1)[0]), step=False, nconmax=300, njmax=300)
    over += int(ref["ncon"] > 2)
  assert over > 0


def test_unsplit_range_chain_resolve(gpu_device):
  """Go1 at 1,024 worlds: one batch range (no split), so the range chain (B -> C -> next A as
  one launch) runs and the re-solve chain runs in line behind it (on a stream of its
  own it raced the range chain's ovf_flag reads).  With a 2-contact / 8-row fast carve every
  standing world overflows each substep; the fused and graph-captured steps equal single steps
  bit for bit in every output, nothing is dropped."""
  from mjlab_amd.envs import load_env_cfg
  from mjlab_amd.scenes import load_scene
  from mjlab_amd.sim import Simulation
  cfg = load_env_cfg("Mjlab-Velocity-Flat-Unitree-Go1")
  cfg.sim.engine_capacity = (2, 8)
  m = load_scene("go1_velocity")
  sim = Simulation(1024, cfg.sim, m, gpu_device)
  assert sim.fast_capacity == (2, 8) and sim.info()["resolve_list"] > 0
  rng = np.random.default_rng(7)
  n = sim.num_envs
  q = np.tile(np.asarray(m.key_qpos, float), (n, 1))
  q[:, 2] -= 0.01 * (np.arange(n) % 4)
  q[:, 7:] += rng.uniform(-0.05, 0.05, (n, m.nq - 7))
  d = sim.data
  d.qpos[:] = torch.as_tensor(q, dtype=torch.float32)
  d.qvel[:] = torch.as_tensor(rng.normal(0.0, 0.05, (n, m.nv)), dtype=torch.float32)
  d.qacc_warmstart.zero_()
  d.ctrl[:] = torch.as_tensor(np.asarray(m.key_qpos, float)[7:][None].repeat(n, 0), dtype=torch.float32)
  for graph in (False, True):
    ev = _fused_vs_single(sim, 4, graph)
    assert ev[:3] == [0, 0, 0] and ev[3] > n, ev
