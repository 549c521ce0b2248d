"""Constraint-row histogram of a task's worlds over bench-like random-action env steps (the
Newton row classes are chosen from it): deciles and the share above given caps."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mjlab-1_amd"))
from mjlab_amd.envs import make_env  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "Mjlab-Jump-Hfield-Unitree-G1"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 60
env = make_env(task, num_envs=n, device="cuda:0", seed=42)
env.reset()
env.enable_graph(capture=True)
g = torch.Generator(device="cuda:0")
g.manual_seed(0)
nact = env.action_manager.total_action_dim
rows = []
for i in range(steps):
  env.step(torch.empty((n, nact), device="cuda:0").uniform_(-1.0, 1.0, generator=g))
  if i >= 10:
    rows.append(env.sim.field("nefc").flatten().cpu().numpy().copy())
r = np.concatenate(rows)
print(task, n, "row classes", env.sim.info(), flush=True)
print("deciles", np.percentile(r, [10, 20, 30, 40, 50, 60, 70, 80, 90, 99]).round(1).tolist(), "max", int(r.max()))
for cap in (48, 56, 60, 64, 72, 80, 96, 112, 128):
  print(f"  > {cap}: {100 * (r > cap).mean():.1f} %")
