"""Run-time specialisation of the step kernels for models no compiled csrc/specs.inc entry
matches (an edited SceneCfg: an extra sensor, another robot).

The engine's kernels take every model dimension and LDS carve offset as compile-time
constants when a specialisation exists; otherwise the generic kernels read them at run time
(measured on G1: 2.05 M against 2.70-2.81 M env-steps/s).  mujoco_warp specialises whatever
model it is given when the step is captured (`src/mjlab/sim/sim.py:164-191`); here, the
equivalent is ahead-of-time: `ensure_library` writes the model's one-entry specs file,
compiles `csrc/jit.hip` for it with hipcc (the image's ROCm toolchain, gfx950) into a shared
library, caches it by a hash of the entry and of the kernel sources, and
`mjx_spec_register` loads it into the engine, after which a sim created with those
dimensions runs the specialised kernels.

Cache: MJX355_JIT_DIR, default `mjlab_amd/jit_cache/` in the tree (so a library built here
travels with the repository), or ~/.cache/mjlab_amd/jit_cache when that is read-only.  A
compile takes about 40 s (the whole step pipeline for one model and capacity; measured on
the edited G1 scene); a cache hit costs a dlopen.
"""

from __future__ import annotations

import hashlib
import os
import subprocess
import tempfile

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")
CACHE = os.environ.get("MJX355_JIT_DIR", os.path.join(_HERE, "jit_cache"))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# the same flags as csrc/Makefile's CXXFLAGS (the kernels must round identically)
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall", "-Wno-unused-function",
         "-fno-hip-fp32-correctly-rounded-divide-sqrt", "-fvisibility=hidden", "-shared"]
SOURCES = ("jit.hip", "engine_impl.h", "engine.h", "carve.h", "fields.h")

ORDER = ["nq", "nv", "nu", "nbody", "njnt", "ngeom", "nsite", "nsensor", "nsensordata", "npair",
         "nhfield", "nhfielddata", "nlevel", "nchild", "nmocap", "ngeom_lds", "npair_all",
         "nstatic", "nstpartner", "nboxbox", "nconmax", "njmax"]


def spec_dims(m) -> dict:
  """The engine's Dims of a compiled model, as capi.cpp derives them at mjx_model_create (the
  terrain pair-tail tables included); nconmax / njmax are the caller's.  A mismatch with the
  engine's own derivation costs speed (find_spec falls back to the generic kernels), never
  correctness: the engine compares every field."""
  a = m.arrays
  gt = np.asarray(a["geom_type"]).reshape(-1)
  p1 = np.asarray(a["pair_geom1"]).reshape(-1)
  p2 = np.asarray(a["pair_geom2"]).reshape(-1)
  np_all = int(m.npair)
  body = np.asarray(a["geom_bodyid"]).reshape(-1)
  weld = np.asarray(a["body_weldid"]).reshape(-1)
  static = (gt == 1) | ((gt == 6) & (weld[body] == 0))  # capi.cpp is_static
  nreg = 0
  while nreg < np_all and not static[p1[nreg]] and not static[p2[nreg]]:
    nreg += 1
  st, partners = [], []
  for q in range(nreg, np_all):
    sg, pg = (int(p1[q]), int(p2[q])) if static[p1[q]] else (int(p2[q]), int(p1[q]))
    if not st or st[-1] != sg:
      st.append(sg)
    if pg not in partners:
      partners.append(pg)
  childadr = np.asarray(a["body_childadr"]).reshape(-1)
  mocap = np.asarray(a["body_mocapid"]).reshape(-1)
  return dict(nq=m.nq, nv=m.nv, nu=m.nu, nbody=m.nbody, njnt=m.njnt, ngeom=m.ngeom,
              nsite=m.nsite, nsensor=m.nsensor, nsensordata=m.nsensordata, npair=nreg,
              nhfield=m.nhfield, nhfielddata=m.nhfielddata,
              nlevel=len(np.asarray(a["level_start"]).reshape(-1)) - 1,
              nchild=max(1, int(childadr[m.nbody])), nmocap=int((mocap >= 0).sum()),
              ngeom_lds=int((~static).sum()), npair_all=np_all, nstatic=len(st),
              nstpartner=len(partners), nboxbox=int(((gt[p1] == 6) & (gt[p2] == 6)).sum()),
              nconmax=0, njmax=0)


def dof_tree(m) -> tuple:
  return tuple(int(p) for p in np.asarray(m.dof_parentid).reshape(-1))


# a specs file is included once per macro (MJX_SPEC, MJX_SPEC_TREE, MJX_SPEC_ROLE); the others
# default to nothing for that pass
GUARD_HEAD = ["#ifndef MJX_SPEC", "#define MJX_SPEC(...)", "#define MJX_SPEC_DEFAULTED", "#endif",
              "#ifndef MJX_SPEC_TREE", "#define MJX_SPEC_TREE(...)", "#define MJX_SPEC_TREE_DEFAULTED",
              "#endif",
              "// MJX_SPEC_ROLE(id, mask): 1 = a fast carve, 2 = a max (re-solve) carve; the kernels",
              "// only one role launches are left out of that entry (the generic ones stand in)",
              "#ifndef MJX_SPEC_ROLE", "#define MJX_SPEC_ROLE(...)", "#define MJX_SPEC_ROLE_DEFAULTED",
              "#endif"]
GUARD_TAIL = ["#ifdef MJX_SPEC_DEFAULTED", "#undef MJX_SPEC", "#undef MJX_SPEC_DEFAULTED", "#endif",
              "#ifdef MJX_SPEC_TREE_DEFAULTED", "#undef MJX_SPEC_TREE", "#undef MJX_SPEC_TREE_DEFAULTED",
              "#endif",
              "#ifdef MJX_SPEC_ROLE_DEFAULTED", "#undef MJX_SPEC_ROLE", "#undef MJX_SPEC_ROLE_DEFAULTED",
              "#endif"]


def entry_lines(sid: int, name: str, dims: dict, par: tuple, role: int | None = None) -> list[str]:
  """One specs.inc entry (scripts/gen_specs.py writes the shipped table from the same)."""
  out = [f"MJX_SPEC({sid}, {name}, " + ", ".join(str(int(dims[k])) for k in ORDER) + ")",
         f"MJX_SPEC_TREE({sid}, " + ", ".join(str(p) for p in par) + ")"]
  if role is not None:
    out.append(f"MJX_SPEC_ROLE({sid}, {role})")
  return out


HEADERS = ("engine.h", "engine_impl.h", "carve.h", "fields.h")  # csrc/Makefile HDR_HASH


def header_hash() -> str:
  """The kernel-header hash csrc/Makefile compiles into libmjx355.so (MJX_HDR_HASH): sha1 of
  the concatenated headers, 15 hex digits.  mjx_spec_register refuses a JIT library whose hash
  differs from the engine's (a Params layout mismatch would fault the device)."""
  h = hashlib.sha1()
  for f in HEADERS:
    with open(os.path.join(CSRC, f), "rb") as fh:
      h.update(fh.read())
  return h.hexdigest()[:15]


def _source_hash() -> str:
  h = hashlib.sha1()
  for f in SOURCES:
    with open(os.path.join(CSRC, f), "rb") as fh:
      h.update(fh.read())
  h.update(" ".join(FLAGS).encode())
  return h.hexdigest()


def library_path(model, nconmax: int, njmax: int, role: int) -> tuple[str, str, int]:
  """(cache path, specs-file text, entry id) of the run-time specialisation for `model` at
  capacity (nconmax, njmax); role 1 = a fast carve, 2 = a max (re-solve) carve."""
  d = spec_dims(model)
  d["nconmax"], d["njmax"] = int(nconmax), int(njmax)
  par = dof_tree(model)
  body = "\n".join(entry_lines(0, "jit", d, par, role))
  key = hashlib.sha1((body + _source_hash()).encode()).hexdigest()[:20]
  # an entry id of its own (template instantiations named apart from every other library's)
  sid = 2000 + int(key[:6], 16) % 900000
  text = "\n".join(GUARD_HEAD + entry_lines(sid, "jit", d, par, role) + GUARD_TAIL) + "\n"
  return os.path.join(CACHE, f"spec_{key}.so"), text, sid


def _user_cache() -> str:
  base = os.environ.get("XDG_CACHE_HOME") or os.path.join(os.path.expanduser("~"), ".cache")
  return os.path.join(base, "mjlab_amd", "jit_cache")


def _writable_cache() -> str:
  """The in-tree cache when it can be written, else a per-user cache dir."""
  for d in (CACHE, _user_cache()):
    try:
      os.makedirs(d, exist_ok=True)
      if os.access(d, os.W_OK):
        return d
    except OSError:
      continue
  raise OSError(f"mjlab_amd.jit: no writable kernel cache ({CACHE}, {_user_cache()})")


def _lookup(path: str) -> str | None:
  """`path` (in CACHE) or the same file name in the user cache, if either exists."""
  for p in (path, os.path.join(_user_cache(), os.path.basename(path))):
    if os.path.exists(p):
      return p
  return None


def _local_rank() -> int:
  return int(os.environ.get("LOCAL_RANK", "0"))


def ensure_library(model, nconmax: int, njmax: int, role: int, compile_ok: bool = True,
                   wait_s: float = 900.0) -> str | None:
  """The cached library for this model and capacity, compiled first if `compile_ok` (None when
  it is absent and may not be built, or hipcc is missing).

  One process per GPU builds each key once: the compile runs under an exclusive lock file
  next to the library, so ranks that ask for the same key at once wait for the first one's
  result instead of compiling it again (and a rank that is not local rank 0 only waits, up to
  `wait_s`).  The library goes to the in-tree cache, or to ~/.cache/mjlab_amd/jit_cache when
  the package directory is read-only.  Raises RuntimeError when hipcc fails, OSError when no
  cache directory can be written."""
  path, text, sid = library_path(model, nconmax, njmax, role)
  hit = _lookup(path)
  if hit is not None:
    return hit
  if not compile_ok or not os.path.exists(HIPCC):
    return None
  import fcntl
  import time
  cache = _writable_cache()
  path = os.path.join(cache, os.path.basename(path))
  with open(path + ".lock", "w") as lock:
    if _local_rank() != 0:
      # another local rank compiles; poll its lock so a crash there does not hang this one
      t0 = time.monotonic()
      while True:
        try:
          fcntl.flock(lock, fcntl.LOCK_EX | fcntl.LOCK_NB)
          break
        except BlockingIOError:
          if time.monotonic() - t0 > wait_s:
            raise RuntimeError(f"mjlab_amd.jit: timed out waiting for {path}")
          time.sleep(1.0)
    else:
      fcntl.flock(lock, fcntl.LOCK_EX)
    if os.path.exists(path):  # built while this process waited
      return path
    with tempfile.TemporaryDirectory(dir=cache) as tmp:
      inc = os.path.join(tmp, "jit_specs.inc")
      with open(inc, "w") as fh:
        fh.write(text)
      out = os.path.join(tmp, "lib.so")
      cmd = [HIPCC, *FLAGS, f"-I{CSRC}", f'-DMJX_SPECS_FILE="{inc}"', f"-DMJX_JIT_ID={sid}",
             f"-DMJX_HDR_HASH=0x{header_hash()}ULL", os.path.join(CSRC, "jit.hip"), "-o", out]
      r = subprocess.run(cmd, capture_output=True, text=True)
      if r.returncode != 0:
        raise RuntimeError(f"mjlab_amd.jit: hipcc failed for {path}:\n{r.stderr[-4000:]}")
      os.replace(out, path)  # atomic: a concurrent reader sees the whole library or none
    try:  # a waiter holding the lock finds the library once it gets the lock
      os.unlink(path + ".lock")
    except OSError:
      pass
  return path


def prebuild(targets) -> list[str]:
  """Compile the libraries of [(model, nconmax, njmax, role), ...] concurrently (cache misses
  only); returns their paths."""
  import concurrent.futures as cf
  with cf.ThreadPoolExecutor(max_workers=max(1, len(targets))) as ex:
    return list(ex.map(lambda t: ensure_library(*t), targets))


_registered: dict[str, int] = {}


def register(path: str) -> int:
  """Load a jit.hip library into the engine (once per process); returns its spec id."""
  if path in _registered:
    return _registered[path]
  from ._lib import check, lib
  sid = lib().mjx_spec_register(path.encode())
  if sid < 0:
    check(sid)
  _registered[path] = sid
  return sid
