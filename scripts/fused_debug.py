"""Per-step divergence between the torch and fused manager paths (debug aid)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd"))
import torch
from test_gpu_fused import _env
task = sys.argv[1] if len(sys.argv) > 1 else "Mjlab-Velocity-Flat-Unitree-G1"
n = 128
et = _env(task, n, "cuda:0", fused=False)
ef = _env(task, n, "cuda:0", fused=True)
g = torch.Generator(device="cuda:0").manual_seed(0)
nact = et.action_manager.total_action_dim
d = lambda a, b: float((a.float() - b.float()).abs().max())
print("init qpos", d(et.sim.data.qpos, ef.sim.data.qpos), "qvel", d(et.sim.data.qvel, ef.sim.data.qvel),
      "ctrl", d(et.sim.data.ctrl, ef.sim.data.ctrl))
for step in range(6):
  a = 0.3 * (2 * torch.rand(n, nact, device="cuda:0", generator=g) - 1)
  ot, rt, tt, ut, _ = et.step(a)
  of, rf, tf, uf, _ = ef.step(a)
  torch.cuda.synchronize()
  print(step, "ctrl", d(et.sim.data.ctrl, ef.sim.data.ctrl), "qpos", d(et.sim.data.qpos, ef.sim.data.qpos),
        "qvel", d(et.sim.data.qvel, ef.sim.data.qvel), "obs", d(ot["policy"], of["policy"]),
        "resets", int(ut.sum()), int(tt.sum()), int(uf.sum()), int(tf.sum()))
  dv = (et.sim.data.qvel - ef.sim.data.qvel).abs()
  if float(dv.max()) > 0:
    idx = torch.nonzero(dv > 1e-6)
    print("   qvel diff at", idx[:8].tolist())

# ---- ctrl rounding probe on a fresh pair
et = _env(task, 4, "cuda:0", fused=False)
ef = _env(task, 4, "cuda:0", fused=True)
a = 0.3 * (2 * torch.rand(4, nact, device="cuda:0", generator=g) - 1)
et.step(a); ef.step(a); torch.cuda.synchronize()
term = et.action_manager._terms["joint_pos"]
ct, cf = et.sim.data.ctrl, ef.sim.data.ctrl
bad = torch.nonzero(ct != cf)
print("ctrl mismatches", bad.tolist()[:10])
ctrl_ids = et.scene["robot"].indexing.ctrl_ids.tolist()
act_local = et.scene["robot"]._act_joint_local_t.tolist()
jids = term._joint_ids.tolist()
for e_, c_ in bad.tolist()[:4]:
  aidx = ctrl_ids.index(c_)
  k = jids.index(act_local[aidx])
  raw = float(a[e_, k]); s = float(term._scale[e_, k]); o = float(term._offset[e_, k])
  import numpy as np
  f32 = np.float32
  sep = f32(f32(f32(raw) * f32(s)) + f32(o)); fma = f32(np.float64(f32(raw)) * np.float64(f32(s)) + np.float64(f32(o)))
  print(f"env {e_} ctrl {c_} action {k}: torch {float(ct[e_, c_]):.9g} fused {float(cf[e_, c_]):.9g} sep {float(sep):.9g} fma {float(fma):.9g} processed {float(term._processed[e_, k]):.9g}")
