"""Developer parity probe: prints per-field max errors GPU vs oracle (not a test)."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import numpy as np, torch
from parity_util import g1_states, oracle_step
from mjlab_amd.scenes import load_scene
from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg

for scene in ("g1_velocity", "go1_velocity"):
  m = load_scene(scene)
  n = 32
  sim = Simulation(n, SimulationCfg(nconmax=48, njmax=160, mujoco=MujocoCfg(timestep=m.timestep, iterations=10, ls_iterations=20)), m, "cuda:0")
  q, qv, ctrl = g1_states(m, n, seed=2)
  d = sim.data
  d.qpos[:] = torch.tensor(q, dtype=torch.float32); d.qvel[:] = torch.tensor(qv, dtype=torch.float32)
  d.ctrl[:] = torch.tensor(ctrl, dtype=torch.float32); d.qacc_warmstart[:] = 0
  sim.step(); torch.cuda.synchronize()
  ref = oracle_step(m, q, qv, np.zeros_like(qv), ctrl, step=True)
  for f in ("xpos", "subtree_com", "cvel", "qacc_smooth", "qacc", "qvel", "qpos", "sensordata", "actuator_force"):
    g = getattr(d, f).cpu().numpy()
    e = max(np.abs(g[i] - ref[i][f]).max() for i in range(n))
    s = max(np.abs(ref[i][f]).max() for i in range(n))
    print(f"{scene} {f:15s} maxerr {e:.3e}  scale {s:.3e}")
  print("ncon gpu", d.ncon.cpu().numpy()[:16], "\nncon ref", [r["ncon"] for r in ref][:16])
  print("niter gpu", d.solver_niter.cpu().numpy()[:16], "\nniter ref", [r["niter"] for r in ref][:16])
  print("stats", sim.stats())
  # timing
  for N in (4096,):
    sim2 = Simulation(N, SimulationCfg(nconmax=48, njmax=160, mujoco=MujocoCfg(timestep=m.timestep, iterations=10, ls_iterations=20)), m, "cuda:0")
    qq = torch.tensor(np.tile(m.key_qpos, (N, 1)), dtype=torch.float32, device="cuda:0")
    sim2.data.qpos[:] = qq
    jq = torch.tensor([m.jnt_qposadr[j] for j in m.actuator_trnid], device="cuda:0")
    sim2.data.ctrl[:] = qq[:, jq]
    for _ in range(20): sim2.step()
    torch.cuda.synchronize(); t0 = time.time()
    K = 100
    for _ in range(K): sim2.step()
    torch.cuda.synchronize(); dt = time.time() - t0
    print(f"{scene} N={N}: {dt/K*1e3:.3f} ms/substep -> {N*K/dt/4:.3e} env-steps/s (dec 4)", sim2.stats())
