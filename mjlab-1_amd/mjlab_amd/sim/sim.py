"""`Simulation`: the drop-in replacement of mjlab's physics boundary on MI355X.

Same classes, fields and methods as `src/mjlab/sim/sim.py:42-286`
(`MujocoCfg`, `SimulationCfg`, `Simulation.{step,forward,reset,expand_model_fields,
get_default_field,create_graph}` and the `model`/`data`/`mj_model` properties), backed
by libmjx355 (one HIP kernel per step, all worlds, one wavefront per world) instead of
MuJoCo-Warp.  `model` is the compiled host `Model` (mjlab_amd.compiler.model) where the
reference passes a `mujoco.MjModel`.
"""

from __future__ import annotations

import contextlib
import ctypes
import os
from dataclasses import dataclass, field
from typing import Literal

import numpy as np
import torch

from .._capi import make_desc
from .._lib import MjxError, check, lib
from .sim_data import DeviceBridge, field_tensor

_INTEGRATORS = {"euler": 0, "implicitfast": 1}


@dataclass
class MujocoCfg:
  """Configuration for MuJoCo simulation parameters (sim/sim.py:42-79)."""

  timestep: float = 0.002
  integrator: Literal["euler", "implicitfast"] = "implicitfast"
  impratio: float = 1.0
  cone: Literal["pyramidal", "elliptic"] = "pyramidal"
  jacobian: Literal["auto", "dense", "sparse"] = "auto"
  solver: Literal["newton", "cg", "pgs"] = "newton"
  iterations: int = 100
  tolerance: float = 1e-8
  ls_iterations: int = 50
  ls_tolerance: float = 0.01
  ccd_iterations: int = 50
  gravity: tuple[float, float, float] = (0, 0, -9.81)

  def apply(self, model) -> None:
    """Apply configuration settings to a compiled model (MujocoCfg.apply)."""
    if self.cone != "pyramidal":
      raise NotImplementedError("only pyramidal friction cones are implemented")
    if self.solver != "newton":
      raise NotImplementedError("only the Newton solver is implemented")
    model.integrator = _INTEGRATORS[self.integrator]
    model.cone = 0
    model.timestep = float(self.timestep)
    model.impratio = float(self.impratio)
    model.gravity = np.asarray(self.gravity, dtype=np.float64)
    model.iterations = int(self.iterations)
    model.tolerance = float(self.tolerance)
    model.ls_iterations = int(self.ls_iterations)
    model.ls_tolerance = float(self.ls_tolerance)


@dataclass
class NanGuardCfg:
  """`utils/nan_guard.py:16-23`."""
  enabled: bool = False
  buffer_size: int = 100
  output_dir: str = "/tmp/mjlab/nan_dumps"
  max_envs_to_dump: int = 5


class NanGuard:
  """`utils/nan_guard.py:26-181`: when enabled, a rolling buffer of the last `buffer_size`
  pre-step (qpos, qvel) states; after a step with NaN/Inf in qpos, qvel, qacc or
  qacc_warmstart of any world, the buffered states of the first `max_envs_to_dump` such worlds
  are written once to `nan_dump_<time>.npz` (keys `states_step_<n>`: [envs, nq + nv] rows,
  MuJoCo's mjSTATE_PHYSICS layout for a model without actuator activations or history) with
  the compiled model beside it and `*_latest` symlinks.  Differences, stated: the model is
  saved as this build's compiled-scene npz (`model_<time>.npz`, `scenes.load_model`), not a
  MuJoCo .mjb; `_metadata` is a JSON string (loadable without pickle), same fields.  A
  no-op when disabled; enabled, every step reads a flag back to the host (as the reference)."""

  def __init__(self, cfg: NanGuardCfg, num_envs: int, model) -> None:
    self.cfg = cfg
    self.enabled = cfg.enabled
    self.num_envs = num_envs
    if not self.enabled:
      return
    from collections import deque
    self.buffer: deque = deque(maxlen=cfg.buffer_size)
    self.output_dir = cfg.output_dir
    self.max_envs_to_dump = cfg.max_envs_to_dump
    self.step_counter = 0
    self._dumped = False
    self.model = model
    self.state_size = int(model.nq + model.nv)
    self.last_dump: str | None = None

  def capture(self, data) -> None:
    if not self.enabled:
      return
    self.buffer.append({"step": self.step_counter, "qpos": data.qpos.clone(), "qvel": data.qvel.clone()})
    self.step_counter += 1

  @contextlib.contextmanager
  def watch(self, data):
    self.capture(data)
    yield
    self.check_and_dump(data)

  @staticmethod
  def detect_nans(data) -> torch.Tensor:
    mask = torch.zeros(data.qpos.shape[0], dtype=torch.bool, device=data.qpos.device)
    for t in (data.qpos, data.qvel, data.qacc, data.qacc_warmstart):
      mask |= torch.isnan(t).any(dim=-1) | torch.isinf(t).any(dim=-1)
    return mask

  def check_and_dump(self, data) -> bool:
    if not self.enabled or self._dumped:
      return False
    mask = self.detect_nans(data)
    if bool(mask.any()):
      self._dump_buffer(torch.where(mask)[0].cpu().numpy().tolist())
      self._dumped = True
      return True
    return False

  def _dump_buffer(self, nan_env_ids: list[int]) -> None:
    import datetime
    import json
    import os
    from ..scenes import save_model
    os.makedirs(self.output_dir, exist_ok=True)
    stamp = datetime.datetime.now().strftime("%Y%m%d_%H%M%S")
    dump = os.path.join(self.output_dir, f"nan_dump_{stamp}.npz")
    model_file = os.path.join(self.output_dir, f"model_{stamp}.npz")
    envs = nan_env_ids[: self.max_envs_to_dump]
    out = {}
    for item in self.buffer:
      q, v = item["qpos"][envs].double().cpu().numpy(), item["qvel"][envs].double().cpu().numpy()
      out[f"states_step_{item['step']:06d}"] = np.concatenate([q, v], axis=1)
    meta = {"num_envs_total": self.num_envs, "num_envs_dumped": len(envs), "nan_env_ids": nan_env_ids,
            "dumped_env_ids": list(envs), "state_size": self.state_size, "buffer_size": len(self.buffer),
            "detection_step": self.step_counter, "timestamp": stamp,
            "model_file": os.path.basename(model_file),
            "note": "Rows are [qpos, qvel] (mjSTATE_PHYSICS without act / history). Model saved "
                    "as the compiled-scene npz (mjlab_amd.scenes.load_model)."}
    out["_metadata"] = np.array(json.dumps(meta))
    np.savez_compressed(dump, **out)
    save_model(self.model, model_file)
    for name, target in (("nan_dump_latest.npz", dump), ("model_latest.npz", model_file)):
      link = os.path.join(self.output_dir, name)
      if os.path.lexists(link):
        os.remove(link)
      os.symlink(os.path.basename(target), link)
    self.last_dump = dump
    print(f"[NanGuard] Detected NaN/Inf at step {self.step_counter}")
    print(f"[NanGuard] NaN/Inf found in envs: {nan_env_ids[:10]}...")
    print(f"[NanGuard] Dumped {len(self.buffer)} states of envs {envs} to: {dump}")


def load_nan_dump(path: str) -> tuple[dict, dict]:
  """Read a NanGuard dump without unpickling: ({key: states}, metadata)."""
  import json
  with np.load(path, allow_pickle=False) as z:
    states = {k: z[k] for k in z.files if k != "_metadata"}
    meta = json.loads(str(z["_metadata"]))
  return states, meta


@dataclass(kw_only=True)
class SimulationCfg:
  nconmax: int | None = None
  """Contacts per world (the engine holds at most 64 per world in LDS; the reference's is a
  per-world average of a pooled budget, so a world overflowing the fast carve is re-solved
  at 64, `max_capacity`)."""
  njmax: int | None = None
  """Constraint rows per world: the max capacity a world is re-solved at."""
  ls_parallel: bool = True
  """Accepted so the reference's configs load (`sim/sim.py:94`, default True there), and
  documented as not honoured: mujoco_warp's parallel line search evaluates a fixed set of step
  sizes and keeps the best, while this engine always runs MuJoCo-C's exact (Newton-bracketed)
  line search, which the north star's MuJoCo-C parity targets (DESIGN.md section 4).  Both
  values give the same step here; `Simulation.line_search` reports "exact"."""
  contact_sensor_maxmatch: int = 64
  """Contact-sensor matches recorded per sensor and world (`sim/sim.py:95,141`): a sensor
  reduces over its first contact_sensor_maxmatch matching contacts in contact order (the
  reference records the first that reach its atomic counter) and counts only those."""
  engine_capacity: tuple[int, int] | None = None
  """(contacts, rows) per world of the fast LDS carve every substep runs in (this build's
  knob, not the reference's).  None: 48 contacts and at most 160 rows, far above what the
  velocity and jump worlds reach; the rare world past it is re-solved at the max capacity
  (`max_capacity`: 64 contacts, `njmax` rows) within the same substep.  A task whose worlds
  reach it often may hold the reference's `njmax` here instead (tracking: (64, 256))."""
  specialize: Literal["auto", "always", "never"] = "auto"
  """Kernels for a model no compiled specialisation (csrc/specs.inc) matches (this build's
  knob; mujoco_warp specialises any model at capture, sim/sim.py:164-191): compile them at
  Simulation creation (`mjlab_amd.jit`, hipcc, cached by model and sources) -- "always";
  "auto": load a cached build, and compile one for batches of at least JIT_MIN_WORLDS (a
  compile takes ~40 s); "never": load and compile nothing (a specialisation another sim
  already loaded into the process still matches).  MJX355_JIT=0/1 overrides."""
  mujoco: MujocoCfg = field(default_factory=MujocoCfg)
  nan_guard: NanGuardCfg = field(default_factory=NanGuardCfg)


def _stream_handle(device: torch.device) -> int:
  return torch.cuda.current_stream(device).cuda_stream


def world_capacity(cfg: SimulationCfg, model) -> tuple[int, int]:
  """Per-world contact/row capacities of the fast LDS carve."""
  if os.environ.get("MJX355_WORLD_CAPACITY"):  # diagnostic: "ncon,rows"
    c, r = (int(v) for v in os.environ["MJX355_WORLD_CAPACITY"].split(","))
    return c, r
  nlim = int(np.sum(model.jnt_limited)) if model.njnt else 0
  if cfg.engine_capacity is not None:
    ncon, cap = (int(v) for v in cfg.engine_capacity)
    if not (1 <= ncon <= 64 and 1 <= cap <= 256):
      raise ValueError(f"engine_capacity {cfg.engine_capacity}: contacts 1..64, rows 1..256")
  else:
    ncon = cfg.nconmax if cfg.nconmax is not None else 48
    ncon, cap = int(min(64, max(ncon, 48))), 160
  rows = cfg.njmax if cfg.njmax is not None else cap
  rows = int(max(1, min(rows, 4 * ncon + 2 * nlim, cap)))
  return ncon, rows


MAX_CONTACTS = 512  # include/mjx355.h mjx_sim_create_ex: 8 contacts per lane of a world's wave
JIT_MIN_WORLDS = 1024  # SimulationCfg.specialize "auto": compile kernels for batches this large


def max_capacity(cfg: SimulationCfg, model) -> tuple[int, int]:
  """Per-world contacts / rows a world may reach before anything is dropped: a world that
  overflows the fast carve in a substep is re-solved at this capacity (mjx_sim_create_ex).
  The reference pools contacts over worlds ("one world may have more than nconmax",
  sim/sim.py:82-86) and bounds each world's rows by njmax (:87-91): here every world may
  hold njmax rows and as many contacts as njmax rows allow (every contact makes at least one
  row; condim-1 contacts make exactly one), up to MAX_CONTACTS -- or, with njmax unset, the
  rows 64 pyramidal contacts and every joint limit make.  MJX355_RESOLVE=0: no re-solve
  (overflow drops contacts; diagnostic)."""
  ncon, rows = world_capacity(cfg, model)
  if os.environ.get("MJX355_RESOLVE", "1") == "0" or os.environ.get("MJX355_WORLD_CAPACITY"):
    return ncon, rows
  nlim = int(np.sum(model.jnt_limited)) if model.njnt else 0
  rmax = int(cfg.njmax) if cfg.njmax is not None else 4 * 64 + 2 * nlim
  rmax = max(rows, rmax)
  cmax = min(rmax, MAX_CONTACTS)
  return max(ncon, cmax), rmax


_capacity_warned: set = set()
_generic_warned: set = set()


class GenericKernelWarning(RuntimeWarning):
  """The model has no compile-time specialised step kernels (csrc/specs.inc): it runs the
  generic kernels, whose LDS offsets, loop bounds and dof-tree factor masks are run-time
  values (mujoco_warp specialises any model when the graph is captured, sim/sim.py:164-191)."""


def _warn_generic(model, info: dict) -> None:
  if info["spec"] > 0 or os.environ.get("MJX355_NO_SPEC"):
    return
  key = (model.nq, model.nv, model.nbody, model.ngeom, model.nsensor, model.npair,
         info["nconmax"], info["njmax"])
  if key in _generic_warned:
    return
  _generic_warned.add(key)
  import warnings
  warnings.warn(
      f"mjlab_amd.Simulation: no specialised step kernels for this model (nq {model.nq}, nv "
      f"{model.nv}, nbody {model.nbody}, ngeom {model.ngeom}, nsensor {model.nsensor}, "
      f"npair {model.npair}, capacity {info['nconmax']} contacts / {info['njmax']} rows): "
      "running the generic kernels (measured slower on the shipped robots, DESIGN.md section "
      "3). Add the model to mjlab-1_amd/csrc/specs.inc (scripts/gen_specs.py) and rebuild to "
      "specialise it.", GenericKernelWarning, stacklevel=3)


def _warn_capacity(cfg: SimulationCfg, model, ncon: int, rows: int) -> None:
  """Warn once per distinct clamp: a world whose contacts or rows overflow the max
  capacity drops whole contacts (counted in `engine_counters`, `stats()` and the env's
  extras["log"]["Sim/..."] entries)."""
  asked = (cfg.nconmax, cfg.njmax)
  # rows past 4 * ncon + 2 * (limited joints) cannot occur (every row belongs to a pyramidal
  # contact or a joint limit): warn only when the capacity is below what njmax allows of that
  nlim = int(np.sum(model.jnt_limited)) if model.njnt else 0
  reachable = 4 * ncon + 2 * nlim
  if (cfg.njmax is not None and min(cfg.njmax, reachable) > rows) and asked not in _capacity_warned:
    _capacity_warned.add(asked)
    import warnings
    warnings.warn(
        f"mjlab_amd.Simulation: njmax={cfg.njmax} clamped to {rows} constraint rows per world "
        f"(nconmax {cfg.nconmax} -> {ncon} contacts per world held in LDS); contacts beyond "
        "that are dropped whole and counted as row/contact overflow events",
        RuntimeWarning, stacklevel=3)


class Simulation:
  """GPU-batched MuJoCo physics on MI355X (see module docstring)."""

  def __init__(self, num_envs: int, cfg: SimulationCfg, model, device: str):
    self.cfg = cfg
    self.device = device
    self.num_envs = int(num_envs)
    self.line_search = "exact"  # whatever cfg.ls_parallel says (see SimulationCfg.ls_parallel)
    self._default_model_fields: dict[str, torch.Tensor] = {}
    dev = torch.device(device)
    if dev.type != "cuda":
      raise MjxError("mjlab_amd.Simulation runs only on a ROCm GPU (device 'cuda:N'); "
                     "there is no CPU fallback in the product path")
    self._torch_device = torch.device("cuda", dev.index if dev.index is not None else
                                      torch.cuda.current_device())
    self._mj_model = model
    cfg.mujoco.apply(self._mj_model)
    if int(cfg.contact_sensor_maxmatch) < 1:
      raise ValueError(f"contact_sensor_maxmatch must be >= 1, got {cfg.contact_sensor_maxmatch}")
    model.contact_maxmatch = int(cfg.contact_sensor_maxmatch)
    L = lib()
    desc, keep = make_desc(model)
    self._model_ptr = ctypes.c_void_p()
    check(L.mjx_model_create(ctypes.byref(desc), self._torch_device.index,
                             ctypes.byref(self._model_ptr)))
    del keep
    # the fast carve every substep runs in, and the capacity an overflowing world is
    # re-solved at; nconmax / njmax report the latter (what a world may hold before a
    # contact is dropped)
    self.fast_capacity = world_capacity(cfg, model)
    self.nconmax, self.njmax = max_capacity(cfg, model)
    self._sim = ctypes.c_void_p()
    if not hasattr(L, "mjx_sim_create_ex"):  # an older engine build (MJX355_LIB, scripts/lib_ab.sh)
      self.nconmax, self.njmax = self.fast_capacity
      check(L.mjx_sim_create(self._model_ptr, self.num_envs, self.nconmax, self.njmax,
                             ctypes.byref(self._sim)))
    else:
      check(L.mjx_sim_create_ex(self._model_ptr, self.num_envs, self.fast_capacity[0],
                                self.fast_capacity[1], self.nconmax, self.njmax,
                                ctypes.byref(self._sim)))
      # the capacity the engine wired (a diagnostic split forced onto a model with Newton
      # row classes has no re-solve: its max is the fast carve)
      info = self.info()
      self.nconmax, self.njmax = info["nconmax_max"], info["njmax_max"]
      if self._specialise(cfg, model, info):
        check(L.mjx_sim_destroy(self._sim))
        self._sim = ctypes.c_void_p()
        check(L.mjx_sim_create_ex(self._model_ptr, self.num_envs, self.fast_capacity[0],
                                  self.fast_capacity[1], self.nconmax, self.njmax,
                                  ctypes.byref(self._sim)))
        info = self.info()
      _warn_generic(model, info)
    _warn_capacity(cfg, model, self.nconmax, self.njmax)
    self._field_names = {L.mjx_field_name(self._sim, i).decode()
                         for i in range(L.mjx_field_count(self._sim))}
    self._data_bridge = DeviceBridge(self, "", None)
    self._model_bridge = DeviceBridge(self, "model.", self.num_envs)
    self._reset_mask = torch.zeros(self.num_envs, dtype=torch.uint8, device=self._torch_device)
    self.nan_guard = NanGuard(cfg.nan_guard, self.num_envs, self._mj_model)
    self._timing = None
    self.create_graph()

  def __del__(self):
    try:
      if getattr(self, "_sim", None) and self._sim.value:
        torch.cuda.synchronize(self._torch_device)
        lib().mjx_sim_destroy(self._sim)
        self._sim = ctypes.c_void_p()
      if getattr(self, "_model_ptr", None) and self._model_ptr.value:
        lib().mjx_model_destroy(self._model_ptr)
        self._model_ptr = ctypes.c_void_p()
    except Exception:
      pass

  def create_graph(self) -> None:
    """API parity with sim/sim.py:164-191.  A step is ONE kernel launch over all worlds
    with stable device pointers, so there is nothing to capture; callers that want to
    amortise host launch cost over a whole env step capture it with torch.cuda.graph."""
    self.step_graph = None
    self.forward_graph = None
    self.reset_graph = None

  # Properties.
  @property
  def mj_model(self):
    return self._mj_model

  @property
  def data(self) -> DeviceBridge:
    return self._data_bridge

  @property
  def model(self) -> DeviceBridge:
    return self._model_bridge

  @property
  def default_model_fields(self) -> dict[str, torch.Tensor]:
    return self._default_model_fields

  # Methods.
  def expand_model_fields(self, fields: tuple[str, ...]) -> None:
    if not fields:
      return
    invalid = [f for f in fields if f not in self._mj_model.arrays]
    if invalid:
      raise ValueError(f"Fields not found in model: {invalid}")
    stream = _stream_handle(self._torch_device)
    for f in fields:
      if lib().mjx_field_is_expanded(self._sim, f.encode()):
        continue
      check(lib().mjx_expand_field(self._sim, f.encode(), stream))
    self._model_bridge.clear_cache()
    self.create_graph()

  def get_default_field(self, field: str) -> torch.Tensor:
    if field not in self._default_model_fields:
      if field not in self._mj_model.arrays:
        raise ValueError(f"Field '{field}' not found in model")
      model_field = getattr(self.model, field)
      self._default_model_fields[field] = torch.as_tensor(
        np.asarray(self._mj_model.arrays[field]), dtype=model_field.dtype,
        device=self._torch_device).reshape(model_field.shape[1:]).clone()
    return self._default_model_fields[field]

  def forward(self, mask: torch.Tensor | None = None) -> None:
    """mj_forward for all worlds, or only where the uint8/bool `mask` is set."""
    stream = _stream_handle(self._torch_device)
    if mask is None:
      check(lib().mjx_forward(self._sim, stream))
      return
    m = self._as_mask(mask)
    check(lib().mjx_forward_masked(self._sim, ctypes.c_void_p(m.data_ptr()), stream))

  def _as_mask(self, mask: torch.Tensor) -> torch.Tensor:
    if mask.dtype == torch.uint8 and mask.is_contiguous():
      return mask
    self._reset_mask.copy_(mask.to(torch.uint8))
    return self._reset_mask

  def reset_masked(self, mask: torch.Tensor) -> None:
    """mj_resetData on worlds where `mask` is set (sync-free; graph-capturable)."""
    m = self._as_mask(mask)
    check(lib().mjx_reset(self._sim, ctypes.c_void_p(m.data_ptr()),
                          _stream_handle(self._torch_device)))

  def step(self, nsubstep: int = 1) -> None:
    """One mj_step for every world (or `nsubstep` steps fused in one launch)."""
    with self.nan_guard.watch(self.data):
      if self._timing is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        check(lib().mjx_step(self._sim, int(nsubstep), _stream_handle(self._torch_device)))
        ev1.record()
        self._timing.append((ev0, ev1))
      else:
        check(lib().mjx_step(self._sim, int(nsubstep), _stream_handle(self._torch_device)))

  # Launch timing (HIP events on the launch stream) for the benchmark's roofline.
  def timing_begin(self) -> None:
    self._timing = []

  def timing_end(self) -> float:
    """Mean step-kernel launch duration in ms since timing_begin (synchronises)."""
    ev = self._timing or []
    self._timing = None
    if not ev:
      return 0.0
    torch.cuda.synchronize(self._torch_device)
    return sum(a.elapsed_time(b) for a, b in ev) / len(ev)

  def reset(self, env_ids: torch.Tensor | None = None) -> None:
    stream = _stream_handle(self._torch_device)
    if env_ids is None:
      check(lib().mjx_reset(self._sim, None, stream))
      return
    self._reset_mask.fill_(0)
    self._reset_mask[env_ids] = 1
    check(lib().mjx_reset(self._sim, ctypes.c_void_p(self._reset_mask.data_ptr()), stream))

  @property
  def engine_counters(self) -> torch.Tensor:
    """[nworld, 6] int32 device view: [0] contacts, [1] constraint rows, [2] contact
    overflow, [3] row overflow, [4] unsupported-pair events (cumulative), [5] Newton
    iterations.  No host sync (stats() is the synchronising summary).  The engine's columns
    [6] (contact output slots the last output touched) and [7] (contacts it held) are its
    private output bookkeeping and are left out of the view, so zeroing the counters to reset
    statistics cannot leave stale contact entries past ncon (reset() clears both with the
    contact slots)."""
    return self.field("engine_counters")[:, :6]

  def overflow_events(self) -> torch.Tensor:
    """Device [3] int32 view: total contact-overflow, row-overflow and unsupported-pair
    events over all worlds since creation -- work dropped past the max capacity (kept by the
    engine; no kernel, no host sync)."""
    if "engine_events" not in self._field_names:  # an older engine build (scripts/ab.sh)
      return self.engine_counters[:, 2:5].sum(dim=0)
    return self.field("engine_events")[0, :3]

  def event_counts(self) -> torch.Tensor:
    """Device [4] int32 view: overflow_events() followed by the re-solve count --
    world-substeps that overflowed the fast carve and were re-solved at the max capacity
    (nothing dropped)."""
    if "engine_events" not in self._field_names:  # an older engine build (scripts/ab.sh)
      return torch.cat([self.overflow_events(), self.overflow_events().new_zeros(1)])
    return self.field("engine_events")[0, :4]

  def mass_matrix(self, big: bool = False) -> torch.Tensor:
    """[nworld, nv, nv] fp32 joint-space inertia M as the last substep's phase A formed it
    (mjData.qM; diagnostic copy from the engine's phase hand-off scratch, mjx_sim_mass_matrix).
    `big`: the max-capacity scratch, where the overflow re-solve formed the M of the worlds
    it ran.  Stream-ordered, no host sync."""
    nv = self.mj_model.nv
    nvp = (nv + 3) & ~3
    nb = nvp // 4
    ltr = torch.empty(self.num_envs, 8 * nb * (nb + 1), dtype=torch.float32, device=self.device)
    check(lib().mjx_sim_mass_matrix(self._sim, int(big), ctypes.c_void_p(ltr.data_ptr()),
                                    _stream_handle(self._torch_device)))
    rows, cols = [], []
    for i in range(nvp):
      b, r = i >> 2, i & 3
      off = 8 * b * (b + 1) + 4 * (b + 1) * r
      rows.append(torch.arange(off, off + i + 1))
      cols.append(torch.full((i + 1,), i, dtype=torch.long))
    idx = torch.cat(rows).to(ltr.device)
    ii = torch.cat(cols).to(ltr.device)
    jj = torch.cat([torch.arange(i + 1) for i in range(nvp)]).to(ltr.device)
    full = torch.zeros(self.num_envs, nvp, nvp, dtype=torch.float32, device=ltr.device)
    full[:, ii, jj] = ltr[:, idx]
    full[:, jj, ii] = ltr[:, idx]
    return full[:, :nv, :nv]

  def stats(self) -> dict:
    """Engine counters: max contacts/rows seen, overflow and unsupported-pair events,
    re-solves."""
    out = (ctypes.c_int32 * 8)()
    check(lib().mjx_sim_stats(self._sim, out, _stream_handle(self._torch_device)))
    return dict(max_ncon=out[0], max_nefc=out[1], con_overflow=out[2], row_overflow=out[3],
                unsupported=out[4], max_niter=out[5], resolved=out[6])

  def _specialise(self, cfg: SimulationCfg, model, info: dict) -> bool:
    """Load (or build) run-time specialised kernels for the carves no compiled specs.inc
    entry matched (mjlab_amd.jit); True when the sim must be created again to pick them up."""
    policy = cfg.specialize
    env = os.environ.get("MJX355_JIT")
    if env is not None:
      policy = "always" if env != "0" else "never"
    if policy == "never" or os.environ.get("MJX355_NO_SPEC"):
      return False
    from .. import jit
    want = []
    if info["spec"] == 0:
      want.append((info["nconmax"], info["njmax"], 1))
    if info["spec_max"] == 0 and (info["nconmax_max"], info["njmax_max"]) != (info["nconmax"], info["njmax"]):
      want.append((info["nconmax_max"], info["njmax_max"], 2))
    if not want:
      return False
    compile_ok = policy == "always" or self.num_envs >= JIT_MIN_WORLDS
    loaded = False
    for ncon, rows, role in want:
      try:
        path = jit.ensure_library(model, ncon, rows, role, compile_ok=compile_ok)
        if path is not None:
          # (refused -- MjxError, a RuntimeError -- when built from other kernel headers than
          # the loaded engine library)
          jit.register(path)
          loaded = True
      except (RuntimeError, OSError) as e:
        # "always" asked for the specialisation: its failure is the caller's error.  "auto"
        # only wanted speed: the generic kernels compute the same step (GenericKernelWarning
        # fires below), so a failed compile or an unwritable cache does not abort the sim.
        if policy == "always":
          raise
        import warnings
        warnings.warn(f"mjlab_amd.Simulation: run-time specialisation unavailable ({e}); "
                      "using the generic kernels", GenericKernelWarning, stacklevel=3)
        continue
    return loaded

  def info(self) -> dict:
    """Capacities and kernels (mjx_sim_info)."""
    out = (ctypes.c_int32 * 8)()
    check(lib().mjx_sim_info(self._sim, out))
    return dict(nconmax=out[0], njmax=out[1], nconmax_max=out[2], njmax_max=out[3], spec=out[4],
                spec_max=out[5], resolve_list=out[6], row_classes=out[7])

  def profile(self) -> list[int]:
    """Per-stage cycle sums (diagnostic MJX_STAMPS build only)."""
    out = (ctypes.c_uint64 * 48)()
    check(lib().mjx_sim_profile(self._sim, out, _stream_handle(self._torch_device)))
    return list(out)

  def marker(self, tag: int) -> None:
    """Enqueue the engine's empty marker kernel on the current stream (profiling brackets:
    bench.py marks its timed region so a kernel trace can attribute those dispatches)."""
    check(lib().mjx_marker(int(tag), _stream_handle(self._torch_device)))

  def field(self, name: str) -> torch.Tensor:
    return field_tensor(self._sim, name)
