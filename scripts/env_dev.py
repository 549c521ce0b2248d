"""Developer probe: build the G1/Go1 velocity envs, step with random actions, time."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd"))
import torch
from mjlab_amd.envs import make_env
for task in ("Mjlab-Velocity-Flat-Unitree-G1", "Mjlab-Velocity-Flat-Unitree-Go1"):
  N = 4096
  env = make_env(task, N, "cuda:0", seed=42)
  obs, _ = env.reset()
  print(task, {k: tuple(v.shape) for k, v in obs.items()}, "act", env.action_manager.total_action_dim)
  g = torch.Generator(device="cuda:0"); g.manual_seed(0)
  for i in range(30):
    a = 2 * torch.rand(N, env.action_manager.total_action_dim, device="cuda:0", generator=g) - 1
    obs, rew, term, trunc, ex = env.step(a)
  torch.cuda.synchronize()
  print("reward mean", rew.mean().item(), "term", term.sum().item(), "obs finite", all(torch.isfinite(v).all().item() for v in obs.values()))
  t0 = time.time(); K = 50
  env.sim.timing_begin()
  for i in range(K):
    a = 2 * torch.rand(N, env.action_manager.total_action_dim, device="cuda:0", generator=g) - 1
    env.step(a)
  torch.cuda.synchronize(); dt = time.time() - t0
  ms = env.sim.timing_end()
  print(f"{task}: env.step {dt/K*1e3:.2f} ms -> {N*K/dt:.3e} env-steps/s; step kernel {ms:.3f} ms/launch", env.sim.stats())
  for cap in (False, True):
    env.enable_graph(capture=cap)
    for i in range(5):
      a = 2 * torch.rand(N, env.action_manager.total_action_dim, device="cuda:0", generator=g) - 1
      env.step(a)
    torch.cuda.synchronize(); t0 = time.time()
    for i in range(K):
      a = 2 * torch.rand(N, env.action_manager.total_action_dim, device="cuda:0", generator=g) - 1
      obs, rew, term, trunc, ex = env.step(a)
    torch.cuda.synchronize(); dt = time.time() - t0
    print(f"  sync-free graph={cap}: {dt/K*1e3:.2f} ms -> {N*K/dt:.3e} env-steps/s; rew {rew.mean().item():.4f} resets {int(term.sum().item())} obs finite {all(torch.isfinite(v).all().item() for v in obs.values())}")
