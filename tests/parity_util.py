"""Shared helpers for GPU-vs-oracle parity tests (test infrastructure)."""

from __future__ import annotations

import numpy as np

import oracle_lib as ol


def g1_states(model, n, seed=0, height_jitter=0.03, joint_jitter=0.15, vel_scale=0.5):
  """Seeded perturbations of the init keyframe: some worlds in contact, some airborne."""
  rng = np.random.default_rng(seed)
  q = np.tile(model.key_qpos, (n, 1))
  nq, nv = model.nq, model.nv
  q[:, 2] += rng.uniform(-height_jitter, height_jitter, n)
  # random small root rotation
  ang = rng.normal(0, 0.05, (n, 3))
  for i in range(n):
    th = np.linalg.norm(ang[i])
    if th > 1e-9:
      ax = ang[i] / th
      dq = np.array([np.cos(th / 2), *(ax * np.sin(th / 2))])
      w, x, y, z = q[i, 3:7]
      a = np.array([w, x, y, z])
      b = dq
      q[i, 3:7] = [a[0]*b[0]-a[1]*b[1]-a[2]*b[2]-a[3]*b[3], a[0]*b[1]+a[1]*b[0]+a[2]*b[3]-a[3]*b[2],
                   a[0]*b[2]-a[1]*b[3]+a[2]*b[0]+a[3]*b[1], a[0]*b[3]+a[1]*b[2]-a[2]*b[1]+a[3]*b[0]]
  q[:, 7:] += rng.uniform(-joint_jitter, joint_jitter, (n, nq - 7))
  qv = rng.normal(0, vel_scale, (n, nv))
  qv[:, :3] *= 0.3
  jnt_q = np.array([model.jnt_qposadr[j] for j in model.actuator_trnid])
  ctrl = q[:, jnt_q] + rng.uniform(-0.2, 0.2, (n, model.nu))
  return q, qv, ctrl


def oracle_step(model, q, qv, qws, ctrl, step=True, nconmax=64, njmax=160):
  outs = []
  for i in range(q.shape[0]):
    outs.append(ol.forward(model, q[i], qv[i], qws[i], ctrl[i], 0.0, step=step,
                           nconmax=nconmax, njmax=njmax))
  return outs


def expanded_fields(sim) -> list[str]:
  """Model fields the sim holds one copy of per world (Simulation.expand_model_fields)."""
  from mjlab_amd._lib import lib
  out = []
  for name in sim.mj_model.arrays:
    try:
      getattr(sim.model, name)
    except AttributeError:
      continue
    # the engine's own record (a one-world sim has no stride to tell an expanded field by)
    if lib().mjx_field_is_expanded(sim._sim, name.encode()):
      out.append(name)
  return out


def world_model(sim, w: int, fields=None):
  """The compiled model with world `w`'s copies of the expanded (domain-randomised) model
  fields, for the oracle: the engine reads `base + w * stride` (sim/sim.py:226-240)."""
  import dataclasses
  base = sim.mj_model
  fields = expanded_fields(sim) if fields is None else fields
  arrays = dict(base.arrays)
  for f in fields:
    shape = np.asarray(base.arrays[f]).shape
    arrays[f] = getattr(sim.model, f)[w].double().cpu().numpy().reshape(shape)
  return dataclasses.replace(base, arrays=arrays)


# mjData fields the caller writes (inputs of a step); every other data field the engine exposes
# is an output (csrc/fields.h MJX_DATA_*_FIELDS)
DATA_INPUTS = ("ctrl", "qfrc_applied", "xfrc_applied", "mocap_pos", "mocap_quat")
DATA_FIELDS = ("qpos", "qvel", "qacc", "qacc_warmstart", "qacc_smooth", "time", "xpos", "xquat",
               "xmat", "xipos", "ximat", "cvel", "cacc", "subtree_com", "subtree_linvel",
               "subtree_angmom", "geom_xpos", "geom_xmat", "site_xpos", "site_xmat", "sensordata",
               "actuator_force", "actuator_length", "actuator_velocity", "qfrc_actuator",
               "qfrc_bias", "qfrc_passive", "qfrc_constraint", "qfrc_smooth", "contact_dist",
               "contact_pos", "contact_frame", "contact_force", "ncon", "nefc", "solver_niter",
               "contact_geom")


def air_time_buffers(env) -> dict:
  """The contact air-time tensors the engine updates every substep for a fused env
  (mjx_sim_track_air_time), by name; {} when the env has none."""
  fused = getattr(env, "_fused", None)
  sensor = getattr(fused, "_feet_sensor", None) if fused is not None else None
  air = getattr(sensor, "_air", None) if sensor is not None else None
  if not air or not getattr(sensor, "engine_owned", False):
    return {}
  return {f"air_{k}": v for k, v in air.items() if isinstance(v, __import__("torch").Tensor)}


def output_snapshot(sim, extra: dict | None = None) -> dict:
  """Clones of every mjData output field of the sim (all of DATA_FIELDS), the engine's per-world
  counters that describe the last substep (contacts, rows, Newton iterations) and the extra
  tensors (e.g. air_time_buffers), for bit-for-bit comparisons of two step paths."""
  d = sim.data
  out = {k: getattr(d, k).clone() for k in DATA_FIELDS}
  out["engine_counters[0,1,5]"] = sim.engine_counters[:, [0, 1, 5]].clone()
  for k, v in (extra or {}).items():
    out[k] = v.clone()
  return out


def restore_state(sim, state: dict, extra: dict | None = None) -> None:
  for k, v in state.items():
    if k in (extra or {}):
      extra[k].copy_(v)
    else:
      getattr(sim.data, k).copy_(v)


def differing_outputs(a: dict, b: dict) -> dict:
  """{field: number of worlds whose entries differ} for the fields of two output snapshots that
  are not bit-identical (NaN never appears in a finite step; compared as raw values)."""
  bad = {}
  for k, v in a.items():
    w = b[k]
    if v.shape != w.shape:
      bad[k] = -1
      continue
    ne = v != w
    if bool(ne.any()):
      bad[k] = int(ne.reshape(ne.shape[0], -1).any(dim=1).sum()) if ne.dim() > 0 else 1
  return bad


def diff_detail(a: dict, b: dict, bad: dict, nmax: int = 3) -> str:
  """A readable account of the first differing worlds of each field in `bad`: world, its
  ncon / nefc in both snapshots, the first differing flat indices and their values."""
  import torch
  lines = []
  for k in bad:
    v, w = a[k], b[k]
    if v.shape != w.shape:
      lines.append(f"{k}: shapes {tuple(v.shape)} vs {tuple(w.shape)}")
      continue
    ne = (v != w).reshape(v.shape[0], -1)
    worlds = ne.any(dim=1).nonzero().flatten().tolist()[:nmax]
    for wd in worlds:
      idx = ne[wd].nonzero().flatten().tolist()[:6]
      va = v.reshape(v.shape[0], -1)[wd][idx].tolist()
      vb = w.reshape(w.shape[0], -1)[wd][idx].tolist()
      nc = (int(a["ncon"].reshape(-1)[wd]), int(b["ncon"].reshape(-1)[wd])) if "ncon" in a else None
      ne_ = (int(a["nefc"].reshape(-1)[wd]), int(b["nefc"].reshape(-1)[wd])) if "nefc" in a else None
      lines.append(f"{k} world {wd} ncon {nc} nefc {ne_}: idx {idx} {va} vs {vb}")
  del torch
  return "; ".join(lines)
