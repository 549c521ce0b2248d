"""Per-stage cycle breakdown of the step kernel (diagnostic -DMJX_STAMPS build)."""
import os, sys
os.environ["MJX355_LIB"] = os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd", "mjlab_amd", "libmjx355_stamps.so")
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd"))
import torch
from mjlab_amd.envs import make_env
NAMES = ["kinematics", "com/cinert/cdof", "crb+M", "collision", "contact sort+params",
         "constraints", "velocity+rne+act", "smooth solve", "subtree mom", "newton",
         "post acc", "sensors", "outputs", "integrate", "phase hand-off out", "phase hand-off in"]
for task in sys.argv[1:] or ["Mjlab-Velocity-Flat-Unitree-G1"]:
  N = int(os.environ.get("NENV", "4096"))
  env = make_env(task, N, "cuda:0", seed=42)
  env.reset()
  g = torch.Generator(device="cuda:0"); g.manual_seed(0)
  for i in range(40):
    env.step(2 * torch.rand(N, env.action_manager.total_action_dim, device="cuda:0", generator=g) - 1)
  p0 = env.sim.profile()
  for i in range(20):
    env.step(2 * torch.rand(N, env.action_manager.total_action_dim, device="cuda:0", generator=g) - 1)
  p1 = env.sim.profile()
  d = [b - a for a, b in zip(p0, p1)]
  tot = sum(d[:16])
  # world-substeps counted (MJX355_STAMP_MINROWS filters to the heavy worlds): 3 flushes
  # (phases A, B, C) per counted world-substep
  nsub = max(d[47] // 3, 1)
  print(f"   counted world-substeps {nsub} of {20 * env.cfg.decimation * N}")
  print(f"== {task}: {tot / nsub:.0f} cycles per world-substep (s_memtime ticks)")
  for i, n in enumerate(NAMES):
    print(f"  {n:22s} {d[i] / nsub:10.0f}  {100 * d[i] / max(tot, 1):5.1f}%")
  SUB = ["  nt: warmstart", "  nt: grad (active, J^T w)", "  nt: H assembly", "  nt: cholesky",
         "  nt: solve", "  nt: M s, J s, dots", "  nt: line search", "  nt: update+cost",
         "  nt: final forces", "  int: damping", "  int: actuator bias", "  int: factor+solve",
         "  int: joints", "  A: preamble rest (act)", "  A: kinematics levels", "  A: pre: state+xfrc",
         "  A: pre: body recs", "  A: pre: dof recs"]
  for i, n in enumerate(SUB):
    print(f"  {n:22s} {d[16 + i] / nsub:10.0f}  {100 * d[16 + i] / max(tot, 1):5.1f}%")
  it = max(d[40], 1)
  print(f"  newton: iterations {d[40] / nsub:.2f}/world-substep, refactors after the first {d[41] / nsub:.2f}, "
        f"changed rows per later iteration {d[42] / max(d[40] - nsub, 1):.2f}, refactors with <=4 changes {d[43] / nsub:.2f}, "
        f"active rows at iteration 0 {d[44] / nsub:.1f}")
  print(f"  factor form: {d[39]} of {d[38]} Newton solves dense (a contact across two branches of the dof tree)")
  print(f"  line search: {d[45] / max(d[46], 1):.2f} evaluations per search, {d[46] / nsub:.2f} searches per world-substep")
  print("  stats", env.sim.stats(), "mean niter", float(env.sim.field("solver_niter").float().mean()))
