"""Physics-only loop for counter collection: N worlds, K substep launches."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd"))
import torch
from mjlab_amd.envs import make_env
task = sys.argv[1] if len(sys.argv) > 1 else "Mjlab-Velocity-Flat-Unitree-G1"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
env = make_env(task, N, "cuda:0", seed=42)
env.reset()
g = torch.Generator(device="cuda:0"); g.manual_seed(0)
for i in range(10):
  env.step(2 * torch.rand(N, env.action_manager.total_action_dim, device="cuda:0", generator=g) - 1)
torch.cuda.synchronize()
for i in range(20):
  env.sim.step()
torch.cuda.synchronize()
print("done")
