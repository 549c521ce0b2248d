"""ctypes mirror of `include/mjx355.h`: the model descriptor and the libmjx355 entry points.

The descriptor layout is checked against `mjx_model_desc_size()` at load time so a
header/binding mismatch fails loudly instead of corrupting memory.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

ABI_VERSION = 4
_I = ctypes.POINTER(ctypes.c_int32)
_D = ctypes.POINTER(ctypes.c_double)
_U64 = ctypes.POINTER(ctypes.c_uint64)
_U32 = ctypes.POINTER(ctypes.c_uint32)

_INT_SCALARS = ["nq", "nv", "nu", "nbody", "njnt", "ngeom", "nsite", "nsensor", "nsensordata",
                "npair", "nhfield", "nhfielddata", "nlevel", "nmaskword", "iterations", "ls_iterations",
                "integrator", "cone", "contact_maxmatch"]
_REAL_SCALARS = ["timestep", "tolerance", "ls_tolerance", "impratio", "meaninertia"]
# (name, ctype) in header order
_ARRAYS = (
  [(n, _I) for n in ("body_parentid", "body_rootid", "body_weldid", "body_jntnum", "body_jntadr",
                     "body_dofnum", "body_dofadr", "body_level", "body_childadr", "body_child",
                     "body_mocapid")]
  + [(n, _D) for n in ("body_pos", "body_quat", "body_ipos", "body_iquat", "body_mass",
                       "body_inertia", "body_subtreemass", "body_invweight0")]
  + [("level_start", _I), ("level_body", _I)]
  + [(n, _I) for n in ("jnt_type", "jnt_qposadr", "jnt_dofadr", "jnt_bodyid", "jnt_limited")]
  + [(n, _D) for n in ("jnt_pos", "jnt_axis", "jnt_range", "jnt_solref", "jnt_solimp",
                       "jnt_margin", "jnt_stiffness")]
  + [("qpos0", _D), ("qpos_spring", _D)]
  + [(n, _I) for n in ("dof_bodyid", "dof_jntid", "dof_parentid")]
  + [("dof_bodymask", _U64)]
  + [(n, _D) for n in ("dof_armature", "dof_damping", "dof_invweight0", "dof_frictionloss")]
  + [(n, _I) for n in ("geom_type", "geom_bodyid", "geom_contype", "geom_conaffinity",
                       "geom_condim", "geom_priority", "geom_dataid")]
  + [(n, _D) for n in ("geom_size", "geom_pos", "geom_quat", "geom_friction", "geom_solmix",
                       "geom_solref", "geom_solimp", "geom_margin", "geom_gap", "geom_rbound")]
  + [("site_bodyid", _I)]
  + [(n, _D) for n in ("site_pos", "site_quat")]
  + [(n, _I) for n in ("actuator_trnid", "actuator_forcelimited", "actuator_ctrllimited")]
  + [(n, _D) for n in ("actuator_gear", "actuator_gainprm", "actuator_biasprm",
                       "actuator_forcerange", "actuator_ctrlrange")]
  + [(n, _I) for n in ("sensor_type", "sensor_objtype", "sensor_objid", "sensor_reftype",
                       "sensor_refid", "sensor_adr", "sensor_dim", "sensor_intprm")]
  + [("sensor_geommask1", _U32), ("sensor_geommask2", _U32)]
  + [("pair_geom1", _I), ("pair_geom2", _I)]
  + [(n, _I) for n in ("hfield_nrow", "hfield_ncol", "hfield_adr")]
  + [("hfield_size", _D), ("hfield_data", _D)]
)


class ModelDesc(ctypes.Structure):
  _fields_ = ([("abi_version", ctypes.c_int)] + [(n, ctypes.c_int) for n in _INT_SCALARS]
              + [(n, ctypes.c_double) for n in _REAL_SCALARS]
              + [("gravity", ctypes.c_double * 3)] + list(_ARRAYS))


_DTYPES = {_I: np.int32, _D: np.float64, _U64: np.uint64, _U32: np.uint32}


def make_desc(model) -> tuple[ModelDesc, list]:
  """Build a ModelDesc pointing into contiguous copies of the model arrays.

  Returns (desc, keepalive); keep `keepalive` referenced while `desc` is in use."""
  d = ModelDesc()
  d.abi_version = ABI_VERSION
  for n in _INT_SCALARS:
    if n == "nlevel":
      d.nlevel = int(len(model.arrays["level_start"]) - 1)
    elif n == "nmaskword":
      mk = np.asarray(model.arrays["sensor_geommask1"])
      d.nmaskword = int(mk.shape[1]) if mk.ndim == 2 else max(1, (model.ngeom + 31) // 32)
    else:
      setattr(d, n, int(getattr(model, n)))
  for n in _REAL_SCALARS:
    setattr(d, n, float(getattr(model, n)))
  for i in range(3):
    d.gravity[i] = float(model.gravity[i])
  keep = []
  for name, ct in _ARRAYS:
    arr = np.ascontiguousarray(np.asarray(model.arrays[name]).reshape(-1), dtype=_DTYPES[ct])
    if arr.size == 0:
      arr = np.zeros(1, dtype=_DTYPES[ct])
    keep.append(arr)
    setattr(d, name, arr.ctypes.data_as(ct))
  return d, keep


def repo_root() -> str:
  return os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
