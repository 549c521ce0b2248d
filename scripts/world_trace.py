"""Per-world phase schedule of one substep (diagnostic MJX_STAMPS build): when each world's
phase A / Newton / phase C started and ended, by Newton row class."""
import os, sys
os.environ["MJX355_LIB"] = os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd", "mjlab_amd", "libmjx355_stamps.so")
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd"))
import numpy as np
import torch
from mjlab_amd.envs import make_env

task = sys.argv[1] if len(sys.argv) > 1 else "Mjlab-Velocity-Flat-Unitree-G1"
N = int(os.environ.get("NENV", "4096"))
env = make_env(task, N, "cuda:0", seed=42)
env.reset()
g = torch.Generator(device="cuda:0"); g.manual_seed(0)
for i in range(40):
  env.step(2 * torch.rand(N, env.action_manager.total_action_dim, device="cuda:0", generator=g) - 1)
torch.cuda.synchronize()
sim = env.sim
env.scene.write_data_to_sim()
sim.step()
torch.cuda.synchronize()
tr = sim.field("world_trace").cpu().numpy().view(np.uint64).reshape(N, 4, 2).astype(np.int64)
nefc = sim.field("nefc").flatten().cpu().numpy()
niter = sim.field("solver_niter").flatten().cpu().numpy()
t0 = tr[:, 0, 0].min()
us = lambda x: (x - t0) / 100.0  # s_memrealtime: 100 MHz
caps = [int(c) for c in os.environ.get("CAPS", "44,84").split(",")]
cls = np.where(nefc <= caps[0], 1, np.where(nefc <= caps[1], 2, 0))
for ph, name in ((0, "A"), (1, "B"), (2, "C")):
  s, e = us(tr[:, ph, 0]), us(tr[:, ph, 1])
  d = e - s
  print(f"{name}: start [{s.min():7.1f} .. {s.max():7.1f}]  end max {e.max():7.1f}  dur med {np.median(d):6.1f} p90 {np.percentile(d,90):6.1f} max {d.max():6.1f} us")
  if ph == 1:
    for c in (1, 2, 0):
      m = cls == c
      if m.any():
        print(f"   class {c}: {m.sum():5d} worlds nefc [{nefc[m].min()}..{nefc[m].max()}] niter mean {niter[m].mean():.2f} "
              f"start [{s[m].min():6.1f}..{s[m].max():6.1f}] dur med {np.median(d[m]):6.1f} max {d[m].max():6.1f} end max {e[m].max():6.1f}")
    for it in range(1, 11):
      m = niter == it
      if m.any():
        print(f"   niter {it:2d}: {m.sum():5d} worlds dur med {np.median(d[m]):6.1f} max {d[m].max():6.1f}  nefc mean {nefc[m].mean():.1f}")
# concurrency profile: resident worlds per phase over the substep (10 us bins), and the
# time-average against the whole span -- low tails mean idle CUs at kernel boundaries
span_end = max(us(tr[:, ph, 1]).max() for ph in range(3))
bins = np.arange(0.0, span_end + 10.0, 10.0)
print("t_us   " + "  ".join(f"{n:>5s}" for n in ("A", "B", "C")))
act = []
for ph in range(3):
  s, e = us(tr[:, ph, 0]), us(tr[:, ph, 1])
  act.append([int(((s < b + 10) & (e > b)).sum()) for b in bins])
for i, b in enumerate(bins):
  if i % 3 == 0:
    print(f"{b:6.0f} " + "  ".join(f"{act[ph][i]:5d}" for ph in range(3)))
tot = np.array(act).sum(axis=0)
print(f"mean resident worlds over the span: {tot.mean():.0f} (peak {tot.max()})")
