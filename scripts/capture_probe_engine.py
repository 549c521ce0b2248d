"""Capture the engine's step with HIP's own stream-capture API (ctypes on libamdhip64) and
replay it, with or without torch in the process, printing after every stage.

Round 3 used it to locate the capture crash of a split x row-class topology; round 5 uses it
to decide whether round 4's graph-replay crash (two middle row classes + the overflow
re-solve on a stream of its own, MJX355_OVF_STREAM=1) is the engine's or the HIP runtime's:
the same topology runs under ROCm 7.2's libamdhip64 (no torch: the engine's dependency
resolves to /opt/rocm/lib) and under the HIP 7.0 runtime torch bundles (--torch: torch is
imported and initialised first, so its libamdhip64 is the one every symbol binds to).

usage: python scripts/capture_probe_engine.py [--torch] [--split 1] [--classes 24,60]
         [--ovf-stream 0|1] [--nsub 3] [--replays 20] [--pipe 1] [--n 131]
Every replay's qpos is compared with the eager run of the same steps (bit-identical).
"""
import argparse
import ctypes
import os
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--torch", action="store_true")
ap.add_argument("--split", default="1")
ap.add_argument("--classes", default="24,60")
ap.add_argument("--ovf-stream", default="1")
ap.add_argument("--nsub", type=int, default=3)
ap.add_argument("--replays", type=int, default=20)
ap.add_argument("--pipe", default="1")
ap.add_argument("--n", type=int, default=131)
ap.add_argument("--mode", type=int, default=0)  # hipStreamCaptureMode: 0 global
a = ap.parse_args()
os.environ["MJX355_SPLIT"] = a.split
os.environ["MJX355_ROW_CLASSES"] = a.classes
os.environ["MJX355_OVF_STREAM"] = a.ovf_stream
os.environ["MJX355_CLASS_PIPE"] = a.pipe

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "mjlab-1_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def say(*x):
  print(*x, flush=True)


if a.torch:
  import torch
  x = torch.ones(1024, device="cuda:0")
  (x * 2).sum().item()  # torch's HIP runtime, context and allocator in use
  hip = ctypes.CDLL("libamdhip64.so")
  say("runtime: torch", torch.__version__)
else:
  hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
  say("runtime: /opt/rocm/lib/libamdhip64.so (no torch)")
rv = ctypes.c_int()
hip.hipRuntimeGetVersion(ctypes.byref(rv))
say("hipRuntimeGetVersion", rv.value)

import numpy as np  # noqa: E402

from mjlab_amd._capi import make_desc  # noqa: E402
from mjlab_amd._lib import check, lib  # noqa: E402
from mjlab_amd.scenes import load_scene  # noqa: E402
from parity_util import g1_states  # noqa: E402

vp, byref = ctypes.c_void_p, ctypes.byref
L = lib()
m = load_scene("g1_velocity")
m.iterations, m.ls_iterations = 10, 20
n = a.n
desc, keep = make_desc(m)
model, sim = vp(), vp()
check(L.mjx_model_create(byref(desc), 0, byref(model)))
check(L.mjx_sim_create_ex(model, n, 48, 160, 64, 160, byref(sim)))
info = (ctypes.c_int32 * 8)()
check(L.mjx_sim_info(sim, info))
say("sim info", list(info), "spec", L.mjx_sim_spec(sim))


def ptr(name):
  t = vp()
  check(L.mjx_field(sim, name.encode(), byref(t)))
  return vp.from_address(t.value).value  # DLManagedTensor -> dl_tensor.data


def put(name, arr):
  arr = np.ascontiguousarray(arr, dtype=np.float32)
  assert hip.hipMemcpy(vp(ptr(name)), arr.ctypes.data_as(vp), ctypes.c_size_t(arr.nbytes), 1) == 0


def get(name, shape):
  out = np.empty(shape, np.float32)
  assert hip.hipMemcpy(out.ctypes.data_as(vp), vp(ptr(name)), ctypes.c_size_t(out.nbytes), 2) == 0
  return out


q, qv, ctrl = g1_states(m, n, seed=22)


def load():
  put("qpos", q)
  put("qvel", qv)
  put("ctrl", ctrl)
  put("qacc_warmstart", np.zeros((n, m.nv)))


s = vp()
assert hip.hipStreamCreateWithFlags(byref(s), ctypes.c_uint(1)) == 0
load()
eager = []
for r in range(a.replays):
  check(L.mjx_step(sim, a.nsub, s))
  assert hip.hipStreamSynchronize(s) == 0
  eager.append(get("qpos", (n, m.nq)))
nefc = get("nefc", (n,)).view(np.int32)
say(f"eager ok: {a.replays} x {a.nsub} substeps; rows max {nefc.max()}, worlds > 60 rows: "
    f"{int((nefc > 60).sum())}, <= 24 rows: {int((nefc <= 24).sum())}")
ev = (ctypes.c_int32 * 8)()
check(L.mjx_sim_stats(sim, ev, s))
say("stats [max ncon, max rows, con ovf, row ovf, unsupported, max niter, resolved]", list(ev)[:7])
load()
assert hip.hipDeviceSynchronize() == 0
say("begin capture rc", hip.hipStreamBeginCapture(s, ctypes.c_int(a.mode)))
check(L.mjx_step(sim, a.nsub, s))
g = vp()
say("end capture rc", hip.hipStreamEndCapture(s, byref(g)))
nn = ctypes.c_size_t(0)
say("nodes rc", hip.hipGraphGetNodes(g, None, byref(nn)), "nodes", nn.value)
ex = vp()
say("instantiate rc", hip.hipGraphInstantiate(byref(ex), g, None, None, ctypes.c_size_t(0)))
bad = 0
for r in range(a.replays):
  rc = hip.hipGraphLaunch(ex, s)
  rs = hip.hipStreamSynchronize(s)
  same = bool(np.array_equal(get("qpos", (n, m.nq)), eager[r]))
  bad += int(not same)
  say(f"replay {r + 1}: launch rc {rc} sync rc {rs} equals eager {same}")
  if rc or rs:
    sys.exit(3)
say("all replays equal eager" if bad == 0 else f"{bad} replays differ")
sys.exit(1 if bad else 0)
