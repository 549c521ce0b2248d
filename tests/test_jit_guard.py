"""The run-time specialisation guard (no GPU): mjx_spec_register refuses a library built from
other kernel headers than libmjx355.so.  Its kernels would read the launch parameters (Params,
the LDS carves, the data arena) through another struct layout -- round 6 saw exactly that
fault the device once, when a JIT library was compiled from headers edited after the last
engine build.  Here a stand-in library exports the five jit.hip entry points with a wrong
header hash; registering it must fail with an error, before any kernel could be launched."""

import ctypes
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mjlab-1_amd", "mjlab_amd", "libmjx355.so")

FAKE = r"""
typedef struct { int v[22]; } Dims;  /* mjx::Dims: 22 ints (csrc/engine.h) */
int mjx_jit_abi(void) { return (int)sizeof(Dims); }
unsigned long long mjx_jit_hdr(void) { return HDR; }
void mjx_jit_dims(Dims* out) { for (int i = 0; i < 22; i++) out->v[i] = 1; }
int mjx_jit_tree(int* par, int cap) { if (cap > 0) par[0] = -1; return 1; }
void* mjx_jit_kernel(int ph) { (void)ph; return 0; }
"""


@pytest.fixture(scope="module")
def lib():
  if not os.path.exists(LIB):
    pytest.skip("libmjx355.so not built (run __graft_entry__.build())")
  L = ctypes.CDLL(LIB)
  L.mjx_last_error.restype = ctypes.c_char_p
  return L


def _fake(tmp_path, hdr: str, name: str) -> str:
  src = tmp_path / f"{name}.c"
  src.write_text(FAKE)
  out = tmp_path / f"{name}.so"
  r = subprocess.run(["gcc", "-shared", "-fPIC", f"-DHDR={hdr}", "-o", str(out), str(src)],
                     capture_output=True, text=True)
  if r.returncode != 0:
    pytest.skip(f"gcc unavailable: {r.stderr[-200:]}")
  return str(out)


def test_header_hash_matches_the_makefile():
  """jit.py computes the hash csrc/Makefile compiles into the engine (same files, same order)."""
  import hashlib
  from mjlab_amd import jit
  h = hashlib.sha1()
  for f in ("engine.h", "engine_impl.h", "carve.h", "fields.h"):
    h.update(open(os.path.join(ROOT, "mjlab-1_amd", "csrc", f), "rb").read())
  assert jit.header_hash() == h.hexdigest()[:15]
  mk = open(os.path.join(ROOT, "mjlab-1_amd", "csrc", "Makefile")).read()
  assert "cat engine.h engine_impl.h carve.h fields.h | sha1sum | cut -c1-15" in mk


def test_stale_jit_library_is_refused(lib, tmp_path):
  path = _fake(tmp_path, "0x1ULL", "stale")
  rc = lib.mjx_spec_register(path.encode())
  assert rc < 0
  assert "other kernel headers" in lib.mjx_last_error().decode()


def test_library_without_the_hash_is_refused(lib, tmp_path):
  src = FAKE.replace("unsigned long long mjx_jit_hdr(void) { return HDR; }", "")
  (tmp_path / "nohdr.c").write_text(src)
  out = tmp_path / "nohdr.so"
  r = subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(out), str(tmp_path / "nohdr.c")],
                     capture_output=True, text=True)
  if r.returncode != 0:
    pytest.skip("gcc unavailable")
  assert lib.mjx_spec_register(str(out).encode()) < 0
