"""Per-env-step GPU time of the bench workload (HIP events around every step, no host sync
inside the loop), to see how the step time evolves from the first warm-up step on.

usage: python scripts/step_times.py [--task T] [--num-envs N] [--steps 300] [--prime-ms 0]
--prime-ms keeps the GPU busy with a throwaway kernel loop for that long before the first
step (a clock-ramp probe)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mjlab-1_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--task", default="Mjlab-Velocity-Flat-Unitree-G1")
ap.add_argument("--num-envs", type=int, default=4096)
ap.add_argument("--steps", type=int, default=300)
ap.add_argument("--prime-ms", type=float, default=0.0)
a = ap.parse_args()

from mjlab_amd.envs import make_env  # noqa: E402

dev = "cuda:0"
env = make_env(a.task, num_envs=a.num_envs, device=dev, seed=42)
env.reset()
env.enable_graph(capture=True)
gen = torch.Generator(device=dev)
gen.manual_seed(0)
nact = env.action_manager.total_action_dim
if a.prime_ms > 0:
  x = torch.randn(4096, 4096, device=dev)
  s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  s0.record()
  n = 0
  while True:
    x = x @ x.T
    x /= x.norm()
    n += 1
    if n % 8 == 0:
      s1.record()
      torch.cuda.synchronize()
      if s0.elapsed_time(s1) > a.prime_ms:
        break
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
ev[0].record()
for i in range(a.steps):
  env.step(torch.empty((a.num_envs, nact), device=dev).uniform_(-1.0, 1.0, generator=gen))
  ev[i + 1].record()
torch.cuda.synchronize()
ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(a.steps)]
for k in range(0, a.steps, 10):
  blk = ms[k:k + 10]
  print(f"steps {k:4d}-{k + len(blk) - 1:4d}: " + " ".join(f"{v:.3f}" for v in blk), flush=True)
print("mean 5..25", sum(ms[5:25]) / 20, "mean 20..220", sum(ms[20:220]) / len(ms[20:220]))
