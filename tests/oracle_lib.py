"""ctypes loader for the CPU oracle (oracle/liboracle.so) — test infrastructure only.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
product path.
"""

from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mjlab-1_amd"))

from mjlab_amd._capi import ModelDesc, make_desc  # noqa: E402

_LIB = None
_D = ctypes.POINTER(ctypes.c_double)
_I = ctypes.POINTER(ctypes.c_int)


def build_oracle() -> str:
  path = os.path.join(ROOT, "oracle", "liboracle.so")
  src = os.path.join(ROOT, "oracle", "oracle.c")
  if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
  return path


def lib():
  global _LIB
  if _LIB is None:
    _LIB = ctypes.CDLL(build_oracle())
    _LIB.orc_model_desc_size.restype = ctypes.c_size_t
    assert _LIB.orc_model_desc_size() == ctypes.sizeof(ModelDesc), "oracle ABI mismatch"
    _LIB.orc_forward_dump.restype = ctypes.c_int
    _LIB.orc_rollout.restype = ctypes.c_int
    _LIB.orc_step_given_qacc.restype = ctypes.c_int
  return _LIB


def _p(a):
  return None if a is None else a.ctypes.data_as(_D)


def forward(model, qpos, qvel=None, qacc_warmstart=None, ctrl=None, time=0.0, step=False,
            nconmax=256, njmax=1024):
  """Single-world mj_forward (or mj_step with step=True); returns a dict of fp64 arrays."""
  desc, keep = make_desc(model)
  nq, nv, nu, nb, ns = model.nq, model.nv, model.nu, model.nbody, model.nsensordata
  f64 = lambda a, n: np.ascontiguousarray(a if a is not None else np.zeros(n), dtype=np.float64)
  qpos, qvel = f64(qpos, nq), f64(qvel, nv)
  qws, ctrl = f64(qacc_warmstart, nv), f64(ctrl, nu)
  out = dict(qpos=np.zeros(nq), qvel=np.zeros(nv), qacc=np.zeros(nv), qacc_smooth=np.zeros(nv),
             sensordata=np.zeros(max(ns, 1)), xpos=np.zeros((nb, 3)), xquat=np.zeros((nb, 4)),
             cvel=np.zeros((nb, 6)), subtree_com=np.zeros((nb, 3)), qfrc_bias=np.zeros(nv),
             qM=np.zeros((nv, nv)), actuator_force=np.zeros(max(nu, 1)), cacc=np.zeros((nb, 6)),
             contact=np.zeros((nconmax, 9)), efc_force=np.zeros(njmax))
  ncon, nefc, niter = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
  ov = lib().orc_forward_dump(
    ctypes.byref(desc), nconmax, njmax, _p(qpos), _p(qvel), _p(qws), _p(ctrl),
    ctypes.c_double(time), int(step), _p(out["qpos"]), _p(out["qvel"]), _p(out["qacc"]),
    _p(out["qacc_smooth"]), _p(out["sensordata"]), _p(out["xpos"]), _p(out["xquat"]),
    _p(out["cvel"]), _p(out["subtree_com"]), _p(out["qfrc_bias"]), _p(out["qM"]),
    _p(out["actuator_force"]), _p(out["cacc"]), ctypes.byref(ncon), ctypes.byref(nefc),
    _p(out["contact"]), _p(out["efc_force"]), ctypes.byref(niter))
  del keep
  out["sensordata"] = out["sensordata"][:ns]
  out["actuator_force"] = out["actuator_force"][:nu]
  out["ncon"], out["nefc"], out["niter"], out["overflow"] = ncon.value, nefc.value, niter.value, ov
  out["contact"] = out["contact"][:ncon.value]
  out["efc_force"] = out["efc_force"][:nefc.value]
  return out


def step_given_qacc(model, qpos, qvel, qacc_warmstart, ctrl, time, qacc, qfrc_constraint=None,
                    qfrc_smooth=None, nconmax=256, njmax=1024, qM=None):
  """One mj_step whose constraint stage takes `qacc` instead of solving for it (forces,
  qfrc_constraint, sensors and the integration follow from it; with `qfrc_constraint` and
  `qfrc_smooth` the integration uses those instead), plus the constraint problem's cost at
  that qacc.  With `qM` (nv x nv) the implicit integration uses that mass matrix (the
  engine's own) instead of the oracle's.  Single world; returns a dict of fp64 arrays."""
  desc, keep = make_desc(model)
  f64 = lambda a, n: np.ascontiguousarray(a if a is not None else np.zeros(n), dtype=np.float64)
  nq, nv, nu, ns = model.nq, model.nv, model.nu, model.nsensordata
  out = dict(qpos=np.zeros(nq), qvel=np.zeros(nv), sensordata=np.zeros(max(ns, 1)),
             qfrc_constraint=np.zeros(nv), efc_force=np.zeros(max(njmax, 1)))
  cost, nefc = ctypes.c_double(), ctypes.c_int()
  a = [f64(qpos, nq), f64(qvel, nv), f64(qacc_warmstart, nv), f64(ctrl, nu)]
  g = f64(qacc, nv)
  fc = None if qfrc_constraint is None else f64(qfrc_constraint, nv)
  fs = None if qfrc_smooth is None else f64(qfrc_smooth, nv)
  mq = None if qM is None else np.ascontiguousarray(qM, dtype=np.float64).reshape(nv, nv)
  ov = lib().orc_step_given_qacc(ctypes.byref(desc), nconmax, njmax, *(_p(x) for x in a),
                                 ctypes.c_double(time), _p(g), _p(fc), _p(fs), _p(mq),
                                 _p(out["qpos"]), _p(out["qvel"]),
                                 _p(out["sensordata"]), _p(out["qfrc_constraint"]), ctypes.byref(cost),
                                 _p(out["efc_force"]), ctypes.byref(nefc))
  del keep
  out["sensordata"] = out["sensordata"][:ns]
  out["efc_force"] = out["efc_force"][:nefc.value]
  out["cost"], out["overflow"] = cost.value, ov
  return out


def mass_matrix_scale(model, qpos):
  """[nv, nv] magnitudes of the terms the CRB mass matrix sums (orc_mass_matrix_scale): the
  scale of an fp32 M's formation error."""
  desc, keep = make_desc(model)
  out = np.zeros((model.nv, model.nv))
  lib().orc_mass_matrix_scale(ctypes.byref(desc), _p(np.ascontiguousarray(qpos, dtype=np.float64)),
                              _p(out))
  del keep
  return out


def qacc_error_scale(model, qpos, qvel, qacc_warmstart, ctrl, time, nconmax=256, njmax=1024,
                     extra=None):
  """Per-dof fp32 error scales (orc_qacc_error_scale): of the Newton solution, |H^-1| times
  the magnitudes of the gradient's terms at the fp64 solution; and of the implicitfast
  velocity update, h |A^-1| times the magnitudes of its right-hand side's terms.  `extra`
  (nv, already divided by eps) adds a perturbation of the problem data to the gradient's
  term magnitudes.  Returns (qacc_scale, qvel_scale)."""
  desc, keep = make_desc(model)
  f64 = lambda a, n: np.ascontiguousarray(a if a is not None else np.zeros(n), dtype=np.float64)
  nq, nv, nu = model.nq, model.nv, model.nu
  out, vout = np.zeros(nv), np.zeros(nv)
  a = [f64(qpos, nq), f64(qvel, nv), f64(qacc_warmstart, nv), f64(ctrl, nu)]
  ex = None if extra is None else f64(extra, nv)
  lib().orc_qacc_error_scale(ctypes.byref(desc), nconmax, njmax, *(_p(x) for x in a),
                             ctypes.c_double(time), _p(ex), _p(out), _p(vout))
  del keep
  return out, vout


def cost_scale(model, qpos, qvel, qacc_warmstart, ctrl, time, nconmax=256, njmax=1024) -> float:
  """fp32 evaluation scale of the Newton cost at the fp64 solution (orc_cost_scale): the
  magnitude of the terms the cost sums; a cost gap is judged in units of eps32 times it."""
  desc, keep = make_desc(model)
  f64 = lambda a, n: np.ascontiguousarray(a if a is not None else np.zeros(n), dtype=np.float64)
  a = [f64(qpos, model.nq), f64(qvel, model.nv), f64(qacc_warmstart, model.nv), f64(ctrl, model.nu)]
  out = ctypes.c_double()
  lib().orc_cost_scale(ctypes.byref(desc), nconmax, njmax, *(_p(x) for x in a), ctypes.c_double(time),
                       ctypes.byref(out))
  del keep
  return out.value


def rollout(model, qpos, qvel, qacc_warmstart, ctrl, time, nstep, nconmax=256, njmax=1024,
            nthreads=0, outputs=True):
  """Batched independent worlds, `nstep` mj_steps each (state arrays updated in place)."""
  desc, keep = make_desc(model)
  nw = qpos.shape[0]
  for a in (qpos, qvel, qacc_warmstart, ctrl, time):
    assert a.dtype == np.float64 and a.flags.c_contiguous
  res = {}
  if outputs:
    res = dict(qacc=np.zeros((nw, model.nv)), sensordata=np.zeros((nw, max(model.nsensordata, 1))),
               xpos=np.zeros((nw, model.nbody, 3)), cvel=np.zeros((nw, model.nbody, 6)),
               subtree_com=np.zeros((nw, model.nbody, 3)),
               actuator_force=np.zeros((nw, max(model.nu, 1))), ncon=np.zeros(nw, np.int32))
  g = lambda k: _p(res[k]) if k in res else None
  lib().orc_rollout(ctypes.byref(desc), nw, nstep, nconmax, njmax, _p(qpos), _p(qvel),
                    _p(qacc_warmstart), _p(ctrl), _p(time), g("qacc"), g("sensordata"),
                    g("xpos"), g("cvel"), g("subtree_com"), g("actuator_force"),
                    res["ncon"].ctypes.data_as(_I) if "ncon" in res else None, nthreads)
  del keep
  return res
