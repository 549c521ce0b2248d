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
