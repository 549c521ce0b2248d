"""Per-world schedule inside the bulk class's chained launch (diagnostic MJX_STAMPS build):
how many worlds are in flight over the launch, and how long its tail is.  One eager
Simulation.step after 40 env steps: phase A runs standalone, then each class's Newton +
phase C (the chain of the last substep carries no next phase A)."""
import os
import sys

os.environ["MJX355_LIB"] = os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd", "mjlab_amd", "libmjx355_stamps.so")
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mjlab_amd.envs import make_env  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "Mjlab-Velocity-Flat-Unitree-G1"
N = int(os.environ.get("NENV", "4096"))
env = make_env(task, N, "cuda:0", seed=42)
env.reset()
g = torch.Generator(device="cuda:0")
g.manual_seed(0)
for i in range(40):
  env.step(2 * torch.rand(N, env.action_manager.total_action_dim, device="cuda:0", generator=g) - 1)
torch.cuda.synchronize()
sim = env.sim
for rep in range(3):
  env.scene.write_data_to_sim()
  sim.step()
  torch.cuda.synchronize()
  tr = sim.field("world_trace").cpu().numpy().view(np.uint64).reshape(N, 4, 2).astype(np.int64)
  nefc = sim.field("nefc").flatten().cpu().numpy()
  niter = sim.field("solver_niter").flatten().cpu().numpy()
  cap = int(os.environ.get("CAP", "64"))
  bulk = nefc <= cap
  us = lambda x: x / 100.0  # s_memrealtime: 100 MHz
  bs, be = us(tr[:, 1, 0]), us(tr[:, 1, 1])
  ce = us(tr[:, 2, 1])
  t0 = bs[bulk].min()
  s, e = bs[bulk] - t0, ce[bulk] - t0
  dur = e - s
  print(f"rep {rep}: bulk worlds {bulk.sum()}, heavy {(~bulk).sum()}; bulk B+C launch span {e.max():.1f} us")
  print(f"  per-world B+C: median {np.median(dur):.1f} p10 {np.percentile(dur, 10):.1f} p90 {np.percentile(dur, 90):.1f} max {dur.max():.1f} us")
  print(f"  world start: median {np.median(s):.1f} p90 {np.percentile(s, 90):.1f} last {s.max():.1f} us")
  print(f"  finished: 50% at {np.percentile(e, 50):.1f}, 90% at {np.percentile(e, 90):.1f}, 99% at {np.percentile(e, 99):.1f}, all at {e.max():.1f} us")
  grid = np.arange(0, e.max() + 5, 5.0)
  inflight = [int(((s <= t) & (e > t)).sum()) for t in grid]
  print("  in flight every 5 us: " + " ".join(str(v) for v in inflight))
  late = np.argsort(-e)[:8]
  print("  last finishers (start, dur, niter, nefc): " + "; ".join(
      f"{s[k]:.0f},{dur[k]:.0f},{niter[bulk][k]},{nefc[bulk][k]}" for k in late))
