"""Time Simulation.step at N worlds (standing keyframe hold), print ms/substep."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mjlab-1_amd"))
import numpy as np, torch
from mjlab_amd.scenes import load_scene
from mjlab_amd.sim import MujocoCfg, Simulation, SimulationCfg
scene = sys.argv[1] if len(sys.argv) > 1 else "g1_velocity"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
m = load_scene(scene)
sim = Simulation(N, SimulationCfg(nconmax=48, njmax=160, mujoco=MujocoCfg(timestep=m.timestep, iterations=10, ls_iterations=20)), m, "cuda:0")
qq = torch.tensor(np.tile(m.key_qpos, (N, 1)), dtype=torch.float32, device="cuda:0")
sim.data.qpos[:] = qq
jq = torch.tensor([m.jnt_qposadr[j] for j in m.actuator_trnid], device="cuda:0")
sim.data.ctrl[:] = qq[:, jq]
for _ in range(20): sim.step()
torch.cuda.synchronize(); t0 = time.time()
K = 100
for _ in range(K): sim.step()
torch.cuda.synchronize(); dt = time.time() - t0
print(f"{scene} N={N} pad={os.environ.get('MJX355_LDS_PAD', '0')}: {dt/K*1e3:.3f} ms/substep", sim.stats())
