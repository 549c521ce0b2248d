"""Run a task's captured fused env step for N steps from a fixed seed and save every mjData
output (tests/parity_util.DATA_FIELDS) to an .npz, so two engine configurations (an
environment knob such as MJX355_NEWTON_JG, or two library builds) can be compared bit for bit
across processes: `step_digest.py <task> <num_envs> <steps> <out.npz>`, then
`step_digest.py --compare a.npz b.npz`."""
import sys

import numpy as np

sys.path[:0] = ["mjlab-1_amd", "tests"]

if sys.argv[1] == "--compare":
  a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
  bad = {k: int((a[k] != b[k]).reshape(a[k].shape[0], -1).any(axis=1).sum()) for k in a.files
         if a[k].shape != b[k].shape or not np.array_equal(a[k], b[k])}
  print("identical" if not bad else f"DIFFERENT (worlds per field): {bad}")
  sys.exit(1 if bad else 0)

import torch  # noqa: E402

from mjlab_amd.envs import make_env  # noqa: E402
from parity_util import DATA_FIELDS  # noqa: E402

task, n, steps, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
env = make_env(task, num_envs=n, device="cuda:0", seed=11)
gen = torch.Generator(device="cuda:0")
gen.manual_seed(11)
nact = env.action_manager.total_action_dim
env.reset()
env.enable_graph(capture=True)
for _ in range(steps):
  env.step(2.0 * torch.rand((n, nact), device="cuda:0", generator=gen) - 1.0)
torch.cuda.synchronize()
d = env.sim.data
np.savez(out, **{k: getattr(d, k).cpu().numpy() for k in DATA_FIELDS})
print(task, n, steps, "max rows", int(d.nefc.max()), "saved", out)
