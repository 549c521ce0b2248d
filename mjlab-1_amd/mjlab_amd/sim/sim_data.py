"""Device-field bridge: attribute access -> torch tensor aliasing HBM owned by libmjx355.

Mirrors `WarpBridge` (src/mjlab/sim/sim_data.py:177-240): attributes resolve lazily to
tensors that share memory with the engine, unexpanded model fields appear with a
stride-0 world dimension (sim_data.py:23-31), and attribute assignment is refused so
device addresses stay stable (sim_data.py:217-223).  Tensors are created through
DLPack (`mjx_field` returns a DLManagedTensor*).  Because every engine call is
enqueued on torch's current stream, in-place tensor writes are ordered with the
physics without the reference's ExternalStream juggling (sim_data.py:36-67).
"""

from __future__ import annotations

import ctypes
from typing import Any

import torch
import torch.utils.dlpack

from .._lib import check, dlpack_capsule, lib


def field_tensor(sim_ptr, name: str) -> torch.Tensor:
  out = ctypes.c_void_p()
  check(lib().mjx_field(sim_ptr, name.encode(), ctypes.byref(out)))
  return torch.utils.dlpack.from_dlpack(dlpack_capsule(out.value))


class DeviceBridge:
  """Read-only attribute view over engine fields (data or model)."""

  def __init__(self, owner, prefix: str = "", nworld: int | None = None) -> None:
    object.__setattr__(self, "_owner", owner)
    object.__setattr__(self, "_prefix", prefix)
    object.__setattr__(self, "_nworld", nworld)
    object.__setattr__(self, "_wrapped_cache", {})

  def __getattr__(self, name: str) -> Any:
    cache = self._wrapped_cache
    if name in cache:
      return cache[name]
    full = self._prefix + name
    if full not in self._owner._field_names:
      raise AttributeError(f"'{type(self).__name__}' has no field '{name}'")
    t = field_tensor(self._owner._sim, full)
    if self._nworld is not None and t.dim() > 0 and t.shape[0] == 1 and self._nworld > 1:
      t = t.expand((self._nworld,) + tuple(t.shape[1:]))
    cache[name] = t
    return t

  def __setattr__(self, name: str, value: Any) -> None:
    raise AttributeError(
      f"Cannot set attribute '{name}' on WarpBridge. "
      f"This wrapper is read-only to preserve memory addresses for CUDA graphs. "
      f"Use in-place operations instead: obj.{name}[:] = value"
    )

  def __dir__(self):
    return sorted(n[len(self._prefix):] for n in self._owner._field_names
                  if n.startswith(self._prefix) and "." not in n[len(self._prefix):])

  def clear_cache(self) -> None:
    object.__setattr__(self, "_wrapped_cache", {})

  def __repr__(self) -> str:
    return f"DeviceBridge(prefix={self._prefix!r}, nworld={self._nworld})"


# Drop-in name used by mjlab code (`from mjlab.sim.sim_data import WarpBridge`).
WarpBridge = DeviceBridge
