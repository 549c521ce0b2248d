"""Benchmark: env-steps/s for Mjlab-Velocity-Flat-Unitree-G1, num_envs=4096 per GPU.

Contract (see task README): `python bench.py --gpus N --steps K --warmup W`; for N>1
launched by torch.distributed.run, one rank per GPU.  Prints ONE JSON line on rank 0.

Workload semantics follow the reference's scripts/benchmarks/measure_throughput.py:
  - env-steps/s = steps * num_envs / elapsed (:82-118), device-synchronised brackets,
    W warm-up steps then K timed steps;
  - `--mode env` (default) times the full ManagerBasedRlEnv.step (action manager ->
    decimation x physics -> terminations/rewards/resets/commands/events/observations);
    `--mode physics` times decimation x Simulation.step only (measure_physics_sps).
Actions are uniform[-1,1) from a torch Generator seeded 0 (scripts/play.py:173-176).

roofline: dominant kernel = one Simulation.step launch group (step_phase<NR,0|1|2>, the
three phases of one substep); algorithmic bytes per env-step
B_env = 4*[dec*(2nq+5nv+2nu+ns+1) + 16*nbody + 72], per launch
B_env/dec per world; achieved = bytes/launch / mean launch time (HIP events on the
launch stream); peak 8 TB/s (MI355X_MICROARCH.md).  `traffic` = HBM bytes per launch from
the committed PMC measurements profiles/*_hbm_traffic.json (FETCH_SIZE x2 + WRITE_SIZE,
separate rocprofv3 passes, scripts/profile_round.sh) when one was taken on this task /
num_envs / nv (latest round first), else null.
cpu_baseline: the fp64 CPU oracle (oracle/liboracle.so, "port"), OpenMP over worlds on
the box's host cores, bounded sample.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mjlab-1_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "env-steps/sec, Unitree-G1 velocity task num_envs=4096, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0


def b_env(m, dec):
  return 4 * (dec * (2 * m.nq + 5 * m.nv + 2 * m.nu + m.nsensordata + 1) + 16 * m.nbody + 72)


def measured_traffic(task, num_envs, nv):
  import glob
  for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_hbm_traffic.json")), reverse=True):
    try:
      with open(path) as fh:
        t = json.load(fh)
    except (OSError, ValueError):
      continue
    if (t.get("task"), t.get("num_envs"), t.get("nv")) == (task, num_envs, nv):
      return float(t["traffic_bytes_per_launch"])
  return None


def cpu_baseline(model, dec, budget_s=12.0):
  """Time the fp64 CPU oracle on a bounded sample of the same workload."""
  import oracle_lib as ol
  threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
  if threads <= 0:
    threads = len(os.sched_getaffinity(0))
  threads = max(1, min(threads, 16))
  nw = 8 * threads
  rng = np.random.default_rng(0)
  q = np.tile(model.key_qpos, (nw, 1)).astype(np.float64)
  qv = np.zeros((nw, model.nv))
  qws = np.zeros((nw, model.nv))
  jq = np.array([model.jnt_qposadr[j] for j in model.actuator_trnid])
  ctrl = q[:, jq] + 0.1 * rng.uniform(-1, 1, (nw, model.nu))
  tm = np.zeros(nw)
  # calibrate with one env step, then run for ~budget_s
  t0 = time.perf_counter()
  ol.rollout(model, q, qv, qws, ctrl, tm, dec, nthreads=threads, outputs=False)
  one = max(time.perf_counter() - t0, 1e-4)
  nsteps = int(max(1, min(200, budget_s / one)))
  t0 = time.perf_counter()
  ol.rollout(model, q, qv, qws, ctrl, tm, nsteps * dec, nthreads=threads, outputs=False)
  el = time.perf_counter() - t0
  return {"value": nw * nsteps / el, "unit": "env-steps/s", "cores": threads, "kind": "port",
          "sample": f"{nw} worlds x {nsteps} env-steps ({dec} substeps each), G1 velocity "
                    f"scene, PD hold of the init keyframe + U(-0.1,0.1) ctrl noise, fp64 oracle"}


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--gpus", type=int, default=1)
  ap.add_argument("--steps", type=int, default=200)
  ap.add_argument("--warmup", type=int, default=50)
  ap.add_argument("--num-envs", type=int, default=4096)
  ap.add_argument("--task", default="Mjlab-Velocity-Flat-Unitree-G1")
  ap.add_argument("--mode", choices=["env", "physics"], default="env")
  ap.add_argument("--no-cpu-baseline", action="store_true")
  ap.add_argument("--eager", action="store_true", help="reference-style eager env.step (host syncs)")
  args = ap.parse_args()

  from mjlab_amd import distributed as mjdist
  world, rank, local = mjdist.world_info()
  dist = None
  torch.cuda.set_device(local)
  if world > 1:
    import torch.distributed as dist
    mjdist.init("nccl", torch.device("cuda", local))
  device = f"cuda:{local}"

  from mjlab_amd.envs import make_env
  env = make_env(args.task, num_envs=args.num_envs, device=device, seed=mjdist.rank_seed(42, rank))
  m = env.sim.mj_model
  dec = env.cfg.decimation
  gen = torch.Generator(device=device)
  gen.manual_seed(0 + rank)
  nact = env.action_manager.total_action_dim
  env.reset()
  if args.mode == "env" and not args.eager:
    env.enable_graph(capture=True)

  def one_step():
    a = 2.0 * torch.rand((args.num_envs, nact), device=device, generator=gen) - 1.0
    if args.mode == "env":
      env.step(a)
    else:
      env.action_manager.process_action(a)
      for _ in range(dec):
        env.action_manager.apply_action()
        env.scene.write_data_to_sim()
        env.sim.step()

  for _ in range(args.warmup):
    one_step()
  if dist is not None:
    dist.barrier()
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  for _ in range(args.steps):
    one_step()
  torch.cuda.synchronize()
  if dist is not None:
    dist.barrier()
  el = time.perf_counter() - t0
  # Step-kernel launch duration for the roofline: HIP events around individual
  # Simulation.step launches (the timed env steps run inside a HIP graph).
  env.sim.timing_begin()
  for _ in range(10):
    env.scene.write_data_to_sim()
    env.sim.step()
  launch_ms = env.sim.timing_end()
  if dist is not None:
    el = mjdist.max_over_ranks(el, device)
    # episode statistics: one packed all-gather over RCCL
    mjdist.gather_stats(env.packed_episode_stats())

  total = args.steps * args.num_envs * world
  value = total / el
  if rank == 0:
    bytes_launch = b_env(m, dec) / dec * args.num_envs
    achieved = bytes_launch / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0
    traffic = measured_traffic(args.task, args.num_envs, m.nv)
    out = {
      "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world,
      "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
      "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
      "data": "synthetic (random-init state from the compiled G1 MJCF; uniform random actions)",
      "config": {"workload": f"{args.task} {'env.step' if args.mode == 'env' else 'physics-only decimation x sim.step'}",
                 "task": args.task, "num_envs_per_gpu": args.num_envs, "decimation": dec,
                 "parallelism": f"dp{world}", "mode": args.mode,
                 "step_path": ("eager" if (args.eager or args.mode != "env") else
                               "sync-free, HIP-graph captured" +
                               (", fused HIP managers" if getattr(env, "_fused", None) is not None else ""))},
      "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": achieved / HBM_PEAK_GBS,
                   "traffic": traffic,
                   "kernel": "mjx::step_phase<NR,0|1|2> (one Simulation.step)", "launch_ms": launch_ms,
                   "bytes_per_launch": bytes_launch,
                   # the HBM roofline is the north star's pricing; what actually bounds the
                   # kernel is per-world dependency latency and VALU issue,
                   # as the measured traffic rate next to the peak shows
                   "limiter": "latency/VALU issue (not HBM)",
                   "traffic_gbps": (traffic / (launch_ms * 1e-3) / 1e9
                                    if traffic is not None and launch_ms > 0 else None)},
      "cpu_baseline": None,
    }
    if not args.no_cpu_baseline and world == 1:
      out["cpu_baseline"] = cpu_baseline(m, dec)
    print(json.dumps(out))
  if dist is not None:
    dist.destroy_process_group()


if __name__ == "__main__":
  main()
