"""Distribution of per-world constraint rows / contacts in the bench workloads (diagnostic:
sizes the LDS row capacity classes of the Newton phase)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd"))
import numpy as np
import torch
from mjlab_amd.envs import make_env

for task in sys.argv[1:] or ["Mjlab-Velocity-Flat-Unitree-G1"]:
  N = 4096
  env = make_env(task, N, "cuda:0", seed=42)
  env.reset()
  g = torch.Generator(device="cuda:0"); g.manual_seed(0)
  ne, nc = [], []
  for i in range(120):
    env.step(2 * torch.rand(N, env.action_manager.total_action_dim, device="cuda:0", generator=g) - 1)
    if i >= 20:
      ne.append(env.sim.field("nefc").flatten().cpu().numpy())
      nc.append(env.sim.field("ncon").flatten().cpu().numpy())
  ne = np.concatenate(ne); nc = np.concatenate(nc)
  print(f"== {task}: nefc mean {ne.mean():.1f} max {ne.max()}  ncon mean {nc.mean():.1f} max {nc.max()}")
  for t in [16, 24, 32, 40, 48, 56, 64, 80, 96, 112, 128, 160]:
    print(f"  nefc <= {t:4d}: {100 * (ne <= t).mean():6.2f}%")
