"""Loader for the in-tree HIP engine `libmjx355.so` (built by `csrc/Makefile`).

There is deliberately no fallback: if the library is missing or fails to load, every
product entry point raises.  Parity checks live in tests/ against oracle/.
"""

from __future__ import annotations

import ctypes
import os

from ._capi import ModelDesc

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MJX355_LIB", os.path.join(_HERE, "libmjx355.so"))

# Symbols declared in include/mjx355.h (kept in sync by tests/test_capi.py).
EXPORTS = ("mjx_last_error", "mjx_abi_version", "mjx_model_desc_size", "mjx_model_create",
           "mjx_model_destroy", "mjx_sim_create", "mjx_sim_destroy", "mjx_step", "mjx_forward",
           "mjx_reset", "mjx_field", "mjx_field_count", "mjx_field_name", "mjx_expand_field",
           "mjx_field_is_expanded", "mjx_sim_stats", "mjx_sim_profile", "mjx_sim_spec",
           "mjx_forward_masked", "mjx_sim_track_air_time", "mjx_marker", "mjx_sim_create_ex",
           "mjx_sim_info", "mjx_sim_mass_matrix", "mjx_spec_register",
           # include/mjx355_task.h (fused velocity-task managers; bound in fused.py)
           "mjx_task_create", "mjx_task_destroy", "mjx_task_action", "mjx_task_substep",
           "mjx_task_post", "mjx_task_reset", "mjx_task_observe", "mjx_task_desc_size",
           "mjx_task_last_error", "mjx_quat_mul", "mjx_terrain_levels",
           # fused tracking-task managers (bound in fused_tracking.py)
           "mjx_track_create", "mjx_track_destroy", "mjx_track_action", "mjx_track_post",
           "mjx_track_reset", "mjx_track_observe", "mjx_track_desc_size", "mjx_track_last_error")

_lib = None


class MjxError(RuntimeError):
  pass


def lib() -> ctypes.CDLL:
  global _lib
  if _lib is not None:
    return _lib
  if not os.path.exists(LIB_PATH):
    raise MjxError(f"{LIB_PATH} not built: run `make -C mjlab-1_amd/csrc` "
                   "(or __graft_entry__.build())")
  L = ctypes.CDLL(LIB_PATH)
  vp, ci = ctypes.c_void_p, ctypes.c_int
  L.mjx_last_error.restype = ctypes.c_char_p
  L.mjx_abi_version.restype = ci
  L.mjx_model_desc_size.restype = ctypes.c_size_t
  L.mjx_model_create.argtypes = [ctypes.POINTER(ModelDesc), ci, ctypes.POINTER(vp)]
  L.mjx_model_destroy.argtypes = [vp]
  L.mjx_sim_create.argtypes = [vp, ci, ci, ci, ctypes.POINTER(vp)]
  if hasattr(L, "mjx_sim_create_ex"):
    L.mjx_sim_create_ex.argtypes = [vp, ci, ci, ci, ci, ci, ctypes.POINTER(vp)]
    L.mjx_sim_info.argtypes = [vp, ctypes.POINTER(ctypes.c_int32)]
  L.mjx_sim_destroy.argtypes = [vp]
  L.mjx_step.argtypes = [vp, ci, vp]
  L.mjx_forward.argtypes = [vp, vp]
  L.mjx_forward_masked.argtypes = [vp, vp, vp]
  L.mjx_reset.argtypes = [vp, vp, vp]
  L.mjx_field.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(vp)]
  L.mjx_field_count.argtypes = [vp]
  L.mjx_field_name.argtypes = [vp, ci]
  L.mjx_field_name.restype = ctypes.c_char_p
  L.mjx_expand_field.argtypes = [vp, ctypes.c_char_p, vp]
  L.mjx_field_is_expanded.argtypes = [vp, ctypes.c_char_p]
  L.mjx_sim_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_int32), vp]
  L.mjx_sim_spec.argtypes = [vp]
  L.mjx_sim_spec.restype = ctypes.c_int
  L.mjx_sim_profile.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), vp]
  if hasattr(L, "mjx_spec_register"):
    L.mjx_spec_register.argtypes = [ctypes.c_char_p]
  if hasattr(L, "mjx_sim_mass_matrix"):
    L.mjx_sim_mass_matrix.argtypes = [vp, ci, vp, vp]
  if hasattr(L, "mjx_marker"):
    L.mjx_marker.argtypes = [ci, vp]
  if hasattr(L, "mjx_terrain_levels"):
    f32, u64 = ctypes.c_float, ctypes.c_uint64
    L.mjx_terrain_levels.argtypes = [ci, vp, vp, ci, ci, vp, f32, f32, vp, vp, vp, ci, ci, vp, u64,
                                     vp, vp, vp]
  if hasattr(L, "mjx_sim_track_air_time"):
    L.mjx_sim_track_air_time.argtypes = [vp, ci, ctypes.POINTER(ctypes.c_int32)] + [vp] * 6
  missing = [n for n in EXPORTS if not hasattr(L, n)]
  if missing and not os.environ.get("MJX355_LIB"):  # MJX355_LIB: A/B against an older build
    raise MjxError(f"{LIB_PATH} lacks {missing}: rebuild it (make -C mjlab-1_amd/csrc)")
  for name in EXPORTS:
    if not hasattr(L, name):
      continue
    if name.startswith(("mjx_task_", "mjx_track_")):
      continue  # bound by mjlab_amd.fused / mjlab_amd.fused_tracking
    if name not in ("mjx_last_error", "mjx_field_name", "mjx_model_desc_size"):
      getattr(L, name).restype = ci
  from ._capi import ABI_VERSION
  if L.mjx_abi_version() != ABI_VERSION:
    raise MjxError("libmjx355 ABI version mismatch")
  if L.mjx_model_desc_size() != ctypes.sizeof(ModelDesc):
    raise MjxError("mjxModelDesc layout mismatch between include/mjx355.h and _capi.py")
  _lib = L
  return L


def check(status: int) -> None:
  if status != 0:
    raise MjxError(lib().mjx_last_error().decode())


_PyCapsule_New = ctypes.pythonapi.PyCapsule_New
_PyCapsule_New.restype = ctypes.py_object
_PyCapsule_New.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]


def dlpack_capsule(ptr: int):
  """Wrap a DLManagedTensor* in the standard 'dltensor' PyCapsule."""
  return _PyCapsule_New(ptr, b"dltensor", None)
