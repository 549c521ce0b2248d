"""C-ABI boundary checks that need no GPU: the library loads, exports exactly the symbols
include/mjx355.h declares, and the descriptor layout agrees between C and Python.

No compute entry point is called here (those need a GPU: tests/test_gpu_*.py)."""

import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("mjx355.h", "mjx355_task.h")]
LIB = os.path.join(ROOT, "mjlab-1_amd", "mjlab_amd", "libmjx355.so")


def _declared():
  text = "".join(open(h).read() for h in HEADERS)
  text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
  return sorted(set(re.findall(r"\b(mjx_[a-z_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
  if not os.path.exists(LIB):
    pytest.skip("libmjx355.so not built (run __graft_entry__.build())")
  return ctypes.CDLL(LIB)


def test_header_declares_the_api():
  names = _declared()
  for must in ("mjx_model_create", "mjx_sim_create", "mjx_step", "mjx_forward", "mjx_reset",
               "mjx_field", "mjx_expand_field", "mjx_last_error", "mjx_forward_masked",
               "mjx_task_create", "mjx_task_post", "mjx_task_observe"):
    assert must in names


def test_every_declared_symbol_is_exported(lib):
  for name in _declared():
    assert hasattr(lib, name), f"{name} declared in include/mjx355.h but not exported"


def test_exported_symbols_match_header():
  if not os.path.exists(LIB):
    pytest.skip("library not built")
  nm = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True)
  if nm.returncode != 0:
    pytest.skip("nm unavailable")
  exported = sorted(set(re.findall(r"\bT (mjx_[a-z_]+)\b", nm.stdout)))
  assert exported == _declared()


def test_python_binding_lists_every_export():
  from mjlab_amd._lib import EXPORTS
  assert sorted(EXPORTS) == _declared()


def test_abi_version_and_desc_layout(lib):
  from mjlab_amd._capi import ModelDesc
  from mjlab_amd.fused import TaskDesc
  lib.mjx_model_desc_size.restype = ctypes.c_size_t
  lib.mjx_task_desc_size.restype = ctypes.c_size_t
  from mjlab_amd._capi import ABI_VERSION
  assert lib.mjx_abi_version() == ABI_VERSION == 4
  assert lib.mjx_model_desc_size() == ctypes.sizeof(ModelDesc)
  assert lib.mjx_task_desc_size() == ctypes.sizeof(TaskDesc)


def test_last_error_is_a_string(lib):
  lib.mjx_last_error.restype = ctypes.c_char_p
  assert isinstance(lib.mjx_last_error(), bytes)


def test_null_arguments_fail_cleanly(lib):
  """Error contract: status codes + mjx_last_error, no exceptions across the ABI."""
  lib.mjx_last_error.restype = ctypes.c_char_p
  assert lib.mjx_model_create(None, 0, None) != 0
  assert b"null" in lib.mjx_last_error()
  assert lib.mjx_step(None, 1, None) != 0
  assert lib.mjx_sim_destroy(None) == 0 and lib.mjx_model_destroy(None) == 0


def test_product_path_refuses_cpu_device():
  """No CPU fallback: Simulation on a CPU device raises instead of silently degrading."""
  from mjlab_amd._lib import MjxError
  from mjlab_amd.scenes import load_scene
  from mjlab_amd.sim import Simulation, SimulationCfg
  with pytest.raises(MjxError):
    Simulation(2, SimulationCfg(), load_scene("go1_velocity"), "cpu")
