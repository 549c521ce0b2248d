"""How often a world leaves its Newton row class inside one env step (design input for a
multi-substep class chain): the env runs as the bench runs it (captured fused step, seeded
uniform actions) for a warmup, then eagerly for the measured env steps with Simulation.step
wrapped to record nefc / ncon after every substep.  Per env step and world: the class at the
first substep (rows <= cap: bulk) and the first later substep, if any, at which its rows exceed
the cap or the fast carve.
usage: class_transitions.py [task] [num_envs] [cap] [steps]"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, "mjlab-1_amd")
from mjlab_amd.envs import make_env  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "Mjlab-Velocity-Flat-Unitree-G1"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
cap = int(sys.argv[3]) if len(sys.argv) > 3 else 60
nmeas = int(sys.argv[4]) if len(sys.argv) > 4 else 30

env = make_env(task, num_envs=n, device="cuda:0", seed=42)
gen = torch.Generator(device="cuda:0")
gen.manual_seed(0)
nact = env.action_manager.total_action_dim
env.reset()
env.enable_graph(capture=True)
for _ in range(60):
  env.step(2.0 * torch.rand((n, nact), device="cuda:0", generator=gen) - 1.0)
env.enable_graph(capture=False, fused=False)
sim = env.sim
rec = []
real = sim.step


def step(nsubstep=1):
  for _ in range(nsubstep):
    real()
    rec.append(sim.data.nefc.reshape(-1).clone())


sim.step = step
fc, fr = sim.fast_capacity
per = []
for _ in range(nmeas):
  rec.clear()
  env.step(2.0 * torch.rand((n, nact), device="cuda:0", generator=gen) - 1.0)
  torch.cuda.synchronize()
  per.append(torch.stack(rec).cpu().numpy())  # [dec, n]
rows = np.stack(per)  # [steps, dec, n]
dec = rows.shape[1]
bulk0 = rows[:, 0, :] <= cap
esc = np.zeros_like(bulk0)
esc_at = np.full(bulk0.shape, -1)
for s in range(1, dec):
  e = bulk0 & ~esc & (rows[:, s, :] > cap)
  esc_at[e] = s
  esc |= e
heavy0 = ~bulk0
back = heavy0 & (rows[:, 1:, :] <= cap).all(axis=1)
out = dict(task=task, num_envs=n, cap=cap, decimation=dec, steps=nmeas,
           heavy_first_substep=float(heavy0.mean()), bulk_escape_per_env_step=float(esc.mean()),
           escape_worlds_per_env_step=float(esc.sum(axis=1).mean()),
           escape_at_substep={int(s): int((esc_at == s).sum()) for s in range(1, dec)},
           heavy_all_substeps_bulk_after=float(back.mean()),
           world_substeps_over_cap=float((rows > cap).mean()),
           max_rows=int(rows.max()), fast_carve_rows=fr)
print(json.dumps(out))
