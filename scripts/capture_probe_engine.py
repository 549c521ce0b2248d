"""Capture the engine's split x row-class step with HIP's own stream-capture API (ctypes on
libamdhip64), without torch.cuda.graph, printing after every stage: locates the crash that
torch.cuda.graph capture of MJX355_SPLIT=2 + row classes hits (tests/test_gpu_split.py).

usage: python scripts/capture_probe_engine.py <split> <row_classes> [capture_mode 0|1|2] [nsub] [pipe 0|1] [hip_origin 0|1]
hip_origin=1: the capture origin is a stream made by hipStreamCreateWithFlags, not by torch.
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mjlab-1_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))

split = sys.argv[1] if len(sys.argv) > 1 else "2"
classes = sys.argv[2] if len(sys.argv) > 2 else "24"
mode = int(sys.argv[3]) if len(sys.argv) > 3 else 0
nsub = int(sys.argv[4]) if len(sys.argv) > 4 else 3
os.environ["MJX355_CLASS_PIPE"] = sys.argv[5] if len(sys.argv) > 5 else "1"
os.environ["MJX355_SPLIT"] = split
os.environ["MJX355_ROW_CLASSES"] = classes

import numpy as np  # noqa: E402
import torch  # noqa: E402

from parity_util import g1_states  # noqa: E402
from mjlab_amd.scenes import load_scene  # noqa: E402
from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg  # noqa: E402


def say(*a):
  print(*a, flush=True)


hip = ctypes.CDLL("libamdhip64.so")
vp = ctypes.c_void_p
m = load_scene("g1_velocity")
n = 131
sim = Simulation(n, SimulationCfg(nconmax=48, njmax=160, mujoco=MujocoCfg(
  timestep=m.timestep, iterations=10, ls_iterations=20)), m, "cuda:0")
q, qv, ctrl = g1_states(m, n, seed=22)


def load():
  d = sim.data
  d.qpos[:] = torch.as_tensor(q, dtype=torch.float32)
  d.qvel[:] = torch.as_tensor(qv, dtype=torch.float32)
  d.ctrl[:] = torch.as_tensor(ctrl, dtype=torch.float32)
  d.qacc_warmstart[:] = 0


load()
sim.step(nsubstep=nsub)
torch.cuda.synchronize()
ref = sim.data.qpos.cpu().numpy().copy()
say(f"eager ok: split={split} classes={classes} mode={mode} nsub={nsub} pipe={os.environ['MJX355_CLASS_PIPE']}")
load()
torch.cuda.synchronize()
hip_origin = len(sys.argv) > 6 and sys.argv[6] == "1"
if hip_origin:
  hs = vp()
  say("hipStreamCreateWithFlags rc", hip.hipStreamCreateWithFlags(ctypes.byref(hs), ctypes.c_uint(1)))
  s = torch.cuda.ExternalStream(hs.value)
else:
  s = torch.cuda.Stream()
with torch.cuda.stream(s):
  h = vp(s.cuda_stream)
  say("begin capture rc", hip.hipStreamBeginCapture(h, ctypes.c_int(mode)))
  sim.step(nsubstep=nsub)
  g = vp()
  say("launches enqueued; end capture ...")
  say("end capture rc", hip.hipStreamEndCapture(h, ctypes.byref(g)))
  nn = ctypes.c_size_t(0)
  say("get nodes rc", hip.hipGraphGetNodes(g, None, ctypes.byref(nn)), "nodes", nn.value)
  ex = vp()
  say("instantiate ...")
  say("instantiate rc", hip.hipGraphInstantiate(ctypes.byref(ex), g, None, None, ctypes.c_size_t(0)))
  say("launch rc", hip.hipGraphLaunch(ex, h))
  say("sync rc", hip.hipStreamSynchronize(h))
got = sim.data.qpos.cpu().numpy()
say("replay equals eager:", bool(np.array_equal(got, ref)))
