"""A `Simulation` stand-in backed by the fp64 CPU oracle -- TEST INFRASTRUCTURE ONLY.

Config 1 of BASELINE.json is "Mjlab-Velocity-Flat-Unitree-G1, num_envs=1, --agent zero, CPU
path (plumbing, no GPU)": the whole env on the host with the CPU engine (SURVEY.md section
8d).  The product refuses to run on the CPU (`mjlab_amd.sim.Simulation` raises on a non-ROCm
device), so this module provides the CPU engine behind the same surface for the two places
allowed to run the oracle: `bench.py`'s `cpu_baseline` leg (the full-env CPU figure) and
`tests/` (the oracle's own invariants).  `CpuEnv` is `ManagerBasedRlEnv` with this sim
plugged into its physics boundary (`_make_sim`); the managers run unchanged as torch CPU code.

`OracleData` wraps the oracle's `orcData` (oracle/oracle.h) with ctypes, so every stage
output (xpos, cvel, qM, qfrc_bias, subtree_angmom, cacc, ...) is readable as numpy.
"""

from __future__ import annotations

import ctypes
import dataclasses
from types import SimpleNamespace

import numpy as np
import torch

import oracle_lib as ol
from mjlab_amd._capi import make_desc

_D = ctypes.POINTER(ctypes.c_double)
_I = ctypes.POINTER(ctypes.c_int)

# orcData field order (oracle/oracle.h), up to `overflow`
_PTRS = ["qpos", "qvel", "qacc_warmstart", "ctrl", "qfrc_applied", "xfrc_applied",
         "xpos", "xquat", "xmat", "xipos", "ximat", "xanchor", "xaxis",
         "geom_xpos", "geom_xmat", "site_xpos", "site_xmat",
         "subtree_com", "cinert", "cdof", "crb", "qM",
         "cvel", "cdof_dot", "qfrc_bias", "qfrc_passive", "subtree_linvel", "subtree_angmom",
         "actuator_force", "qfrc_actuator", "qfrc_smooth", "qacc_smooth",
         "qacc", "qfrc_constraint", "cacc", "sensordata"]
_EFC = ["efc_J", "efc_pos", "efc_margin", "efc_D", "efc_R", "efc_aref", "efc_vel", "efc_force",
        "efc_diagApprox", "efc_frame_mu"]


class _OrcData(ctypes.Structure):
  _fields_ = ([("nconmax", ctypes.c_int), ("njmax", ctypes.c_int), ("time", ctypes.c_double)]
              + [(n, _D) for n in _PTRS]
              + [("ncon", ctypes.c_int), ("nefc", ctypes.c_int), ("niter", ctypes.c_int),
                 ("nlimit", ctypes.c_int), ("contact", ctypes.c_void_p), ("efc_type", _I),
                 ("efc_id", _I)]
              + [(n, _D) for n in _EFC]
              + [("overflow", ctypes.c_int)])


def _shapes(m, nconmax, njmax):
  nb, nv, nq, nu = m.nbody, m.nv, m.nq, m.nu
  return dict(qpos=(nq,), qvel=(nv,), qacc_warmstart=(nv,), ctrl=(nu,), qfrc_applied=(nv,),
              xfrc_applied=(nb, 6), xpos=(nb, 3), xquat=(nb, 4), xmat=(nb, 9), xipos=(nb, 3),
              ximat=(nb, 9), xanchor=(m.njnt, 3), xaxis=(m.njnt, 3), geom_xpos=(m.ngeom, 3),
              geom_xmat=(m.ngeom, 9), site_xpos=(m.nsite, 3), site_xmat=(m.nsite, 9),
              subtree_com=(nb, 3), cinert=(nb, 10), cdof=(nv, 6), crb=(nb, 10), qM=(nv, nv),
              cvel=(nb, 6), cdof_dot=(nv, 6), qfrc_bias=(nv,), qfrc_passive=(nv,),
              subtree_linvel=(nb, 3), subtree_angmom=(nb, 3), actuator_force=(nu,),
              qfrc_actuator=(nv,), qfrc_smooth=(nv,), qacc_smooth=(nv,), qacc=(nv,),
              qfrc_constraint=(nv,), cacc=(nb, 6), sensordata=(m.nsensordata,),
              efc_force=(njmax,))


class OracleData:
  """One world's `orcData` (fp64) with numpy views of its arrays (they alias the C memory)."""

  def __init__(self, model, nconmax: int = 64, njmax: int = 256):
    L = ol.lib()
    L.orc_data_new.restype = ctypes.POINTER(_OrcData)
    L.orc_data_free.argtypes = [ctypes.POINTER(_OrcData)]
    self.model = model
    self.desc, self._keep = make_desc(model)
    self._ptr = L.orc_data_new(ctypes.byref(self.desc), int(nconmax), int(njmax))
    self._L = L
    s = self._ptr.contents
    self.arr = {}
    for name, shape in _shapes(model, nconmax, njmax).items():
      n = int(np.prod(shape))
      self.arr[name] = (np.ctypeslib.as_array(getattr(s, name), shape=(max(n, 1),))[:n].reshape(shape)
                        if n else np.zeros(shape))

  def __getattr__(self, name):
    arr = self.__dict__.get("arr")
    if arr is not None and name in arr:
      return arr[name]
    raise AttributeError(name)

  @property
  def time(self) -> float:
    return self._ptr.contents.time

  @time.setter
  def time(self, v: float) -> None:
    self._ptr.contents.time = float(v)

  @property
  def ncon(self) -> int:
    return self._ptr.contents.ncon

  @property
  def nefc(self) -> int:
    return self._ptr.contents.nefc

  @property
  def overflow(self) -> int:
    return self._ptr.contents.overflow

  def set_model(self, model) -> None:
    """Switch to another model with the same dims (a world's domain-randomised fields)."""
    self.model = model
    self.desc, self._keep = make_desc(model)

  def reset(self):
    self._L.orc_reset(ctypes.byref(self.desc), self._ptr)

  def forward(self):
    self._L.orc_forward(ctypes.byref(self.desc), self._ptr)

  def step(self):
    self._L.orc_step(ctypes.byref(self.desc), self._ptr)

  def __del__(self):
    try:
      if self._ptr:
        self._L.orc_data_free(self._ptr)
        self._ptr = None
    except Exception:
      pass


# mjData fields the sim exposes (world-batched float32 CPU tensors), and the state fields
# copied into the oracle before every call
_DATA = ("qpos", "qvel", "qacc", "qacc_warmstart", "ctrl", "qfrc_applied", "xfrc_applied",
         "xpos", "xquat", "xmat", "xipos", "ximat", "geom_xpos", "geom_xmat", "site_xpos",
         "site_xmat", "subtree_com", "cvel", "cacc", "actuator_force", "qfrc_actuator",
         "qfrc_bias", "qfrc_passive", "qfrc_smooth", "qacc_smooth", "qfrc_constraint",
         "sensordata")
_STATE_IN = ("qpos", "qvel", "qacc_warmstart", "ctrl", "qfrc_applied", "xfrc_applied")


class _NullGuard:
  enabled = False

  def watch(self, data):
    import contextlib
    return contextlib.nullcontext()


class OracleSimulation:
  """`mjlab_amd.sim.Simulation`'s surface over one `OracleData` per world (host tensors).
  Every model field is held per world (domain randomisation writes reach that world's
  oracle model on the next call)."""

  def __init__(self, num_envs: int, cfg, model, device: str = "cpu"):
    from mjlab_amd.sim.sim import max_capacity
    self.cfg = cfg
    cfg.mujoco.apply(model)
    self._mj_model = model
    self.num_envs = int(num_envs)
    self.device = device
    # the engine's max capacity: what a world holds before a contact is dropped
    self.nconmax, self.njmax = max_capacity(cfg, model)
    self._worlds = [OracleData(model, self.nconmax, self.njmax) for _ in range(self.num_envs)]
    w0 = self._worlds[0]
    n = self.num_envs
    self.data = SimpleNamespace(**{k: torch.zeros((n,) + w0.arr[k].shape, dtype=torch.float32)
                                   for k in _DATA})
    self.data.time = torch.zeros(n, dtype=torch.float32)
    self.data.ncon = torch.zeros(n, dtype=torch.int32)
    self.data.nefc = torch.zeros(n, dtype=torch.int32)
    self.model = SimpleNamespace()
    self._model_versions = {}
    for name, a in model.arrays.items():
      a = np.asarray(a)
      if a.dtype.kind == "f":
        t = torch.as_tensor(a, dtype=torch.float32).unsqueeze(0).repeat((n,) + (1,) * a.ndim)
        setattr(self.model, name, t)
    self._default_model_fields: dict[str, torch.Tensor] = {}
    self._events = torch.zeros(3, dtype=torch.int32)
    # the engine's per-world counters ([nworld, 8]: contacts, rows, contact / row overflow and
    # unsupported-pair events, cumulative)
    self.engine_counters = torch.zeros(self.num_envs, 8, dtype=torch.int32)
    self._versions = [None] * n
    self.nan_guard = _NullGuard()
    self.reset()

  # ------------------------------------------------------------------ surface
  @property
  def mj_model(self):
    return self._mj_model

  @property
  def default_model_fields(self):
    return self._default_model_fields

  def create_graph(self) -> None:
    pass

  def expand_model_fields(self, fields) -> None:
    invalid = [f for f in fields if f not in self._mj_model.arrays]
    if invalid:
      raise ValueError(f"Fields not found in model: {invalid}")

  def get_default_field(self, field: str) -> torch.Tensor:
    if field not in self._default_model_fields:
      if field not in self._mj_model.arrays:
        raise ValueError(f"Field '{field}' not found in model")
      self._default_model_fields[field] = torch.as_tensor(
        np.asarray(self._mj_model.arrays[field]), dtype=torch.float32).clone()
    return self._default_model_fields[field]

  def overflow_events(self) -> torch.Tensor:
    return self._events

  def event_counts(self) -> torch.Tensor:
    return torch.cat([self._events, torch.zeros(1, dtype=torch.int32)])

  def stats(self) -> dict:
    return dict(max_ncon=int(self.data.ncon.max()), max_nefc=int(self.data.nefc.max()),
                con_overflow=int(self._events[0]), row_overflow=int(self._events[1]),
                unsupported=int(self._events[2]), max_niter=0, resolved=0)

  def marker(self, tag: int) -> None:
    pass

  # ------------------------------------------------------------------ world sync
  def _world(self, w: int) -> OracleData:
    """The world's oracle with its own copies of every float model field."""
    od = self._worlds[w]
    ver = tuple(t._version for t in vars(self.model).values())
    if self._versions[w] != ver:
      arrays = dict(self._mj_model.arrays)
      for name, t in vars(self.model).items():
        arrays[name] = t[w].double().numpy().reshape(np.asarray(self._mj_model.arrays[name]).shape)
      od.set_model(dataclasses.replace(self._mj_model, arrays=arrays))
      self._versions[w] = ver
    return od

  def _push(self, w: int, od: OracleData) -> None:
    for k in _STATE_IN:
      od.arr[k][...] = self.data.__dict__[k][w].double().numpy()
    od.time = float(self.data.time[w])

  def _pull(self, w: int, od: OracleData) -> None:
    for k in _DATA:
      self.data.__dict__[k][w] = torch.from_numpy(od.arr[k])
    self.data.time[w] = od.time
    self.data.ncon[w], self.data.nefc[w] = od.ncon, od.nefc
    ov = od.overflow
    for bit in range(3):
      self._events[bit] += (ov >> bit) & 1
      self.engine_counters[w, 2 + bit] += (ov >> bit) & 1
    self.engine_counters[w, 0], self.engine_counters[w, 1] = od.ncon, od.nefc

  def _run(self, mask, fn) -> None:
    for w in range(self.num_envs):
      if mask is not None and not bool(mask[w]):
        continue
      od = self._world(w)
      self._push(w, od)
      fn(od)
      self._pull(w, od)

  # ------------------------------------------------------------------ physics
  def step(self, nsubstep: int = 1) -> None:
    for _ in range(int(nsubstep)):
      self._run(None, OracleData.step)

  def forward(self, mask=None) -> None:
    self._run(mask, OracleData.forward)

  def reset(self, env_ids=None) -> None:
    mask = None
    if env_ids is not None:
      mask = torch.zeros(self.num_envs, dtype=torch.bool)
      mask[torch.as_tensor(env_ids, dtype=torch.long)] = True
    self.reset_masked(mask)

  def reset_masked(self, mask) -> None:
    for w in range(self.num_envs):
      if mask is not None and not bool(mask[w]):
        continue
      od = self._world(w)
      od.reset()
      od.arr["qacc"][...] = 0.0
      self._pull(w, od)


def make_cpu_env(task: str, num_envs: int = 1, seed: int = 42, play: bool = False):
  """The task's ManagerBasedRlEnv on the host: torch managers on CPU tensors, the fp64 oracle
  behind the physics boundary."""
  from mjlab_amd.envs import ManagerBasedRlEnv, load_env_cfg

  class CpuEnv(ManagerBasedRlEnv):
    def _make_sim(self, model, device):
      return OracleSimulation(self.cfg.scene.num_envs, self.cfg.sim, model, device)

  cfg = load_env_cfg(task, play)
  cfg.scene.num_envs = num_envs
  cfg.seed = seed
  return CpuEnv(cfg, device="cpu")
