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

roofline: the dominant "kernel" is one env step exactly as the timed region runs it (the
HIP graph of decimation x physics phases A/B/C + the fused manager kernels); algorithmic
bytes per env-step B_env = 4*[dec*(2nq+5nv+2nu+ns+1) + 16*nbody + 72] (SURVEY.md section
8d) x num_envs per launch; achieved = bytes / mean launch time (HIP event pairs around
`--launch-reps` further steps, on the stream the graph is replayed on); peak 8 TB/s
(MI355X_MICROARCH.md).  `traffic` = HBM bytes per env step of the same captured step from
the committed PMC measurement profiles/*_hbm_traffic.json (FETCH_SIZE x2 + WRITE_SIZE,
separate rocprofv3 passes over bench.py itself, scripts/profile_round.sh) when one was
taken on this task / num_envs / nv, else null.  `bound` is the larger of the HBM and MFMA
fractions.
overflow: contact/row overflow events counted by the engine over the timed steps (dropped
contact work past the max capacity); non-zero makes the run exit 3 after printing the line
(--allow-overflow).  resolved_events: world-substeps that overflowed the fast LDS carve and
were re-solved at the max capacity inside the same step (nothing dropped; their cost is in
the timing).
cpu_baseline: the fp64 CPU oracle (oracle/liboracle.so, "port") on the allotted host cores
over the bench's own worlds with random actions, plus config 1 (num_envs=1, zero action,
one thread).
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


def cpu_threads():
  """Host threads for the CPU leg: OMP_NUM_THREADS when set (the GPU box sets it to its CPU
  share), else every core of the affinity mask."""
  aff = len(os.sched_getaffinity(0))
  t = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
  return (t if t > 0 else aff), aff


def cgroup_cpus():
  try:
    with open("/sys/fs/cgroup/cpu.max") as fh:
      q, p = fh.read().split()[:2]
    return None if q == "max" else float(q) / float(p)
  except (OSError, ValueError):
    return None


def ctrl_affine(env):
  """ctrl = A @ action + b for world 0, probed through the env's own action path
  (JointPositionAction: a * scale + offset - encoder_bias, then the actuator order of
  write_ctrl; managers/action_manager.py:113-130, entity/data.py:168-180)."""
  nact = env.action_manager.total_action_dim
  n = env.num_envs

  def ctrl_of(a):
    env.action_manager.process_action(a)
    env.action_manager.apply_action()
    env.scene.write_data_to_sim()
    torch.cuda.synchronize()
    return env.sim.data.ctrl[0].double().cpu().numpy().copy()

  z = torch.zeros(n, nact, device=env.device)
  b = ctrl_of(z)
  A = np.zeros((b.size, nact))
  for k in range(nact):
    e = z.clone()
    e[:, k] = 1.0
    A[:, k] = ctrl_of(e) - b
  return A, b


def cpu_baseline(env, dec, budget_s=12.0, config1_s=4.0):
  """The fp64 CPU oracle ("port") on the box's host cores, physics only (decimation x
  mj_step per env step; the managers are not included):
    - the bench's own worlds: the first <= 4096 worlds' states as the timed region left
      them, a new uniform[-1, 1) action per env step mapped through the action scale and
      offset (ctrl_affine), OpenMP over worlds on every allotted core;
    - config 1 (BASELINE.json): num_envs = 1, zero actions (`--agent zero`), one thread,
      from the init keyframe."""
  import oracle_lib as ol
  m = env.sim.mj_model
  threads, aff = cpu_threads()
  A, b = ctrl_affine(env)
  nact = A.shape[1]
  nw = min(4096, env.num_envs)
  d = env.sim.data
  f64 = lambda t: np.ascontiguousarray(t[:nw].double().cpu().numpy())
  q, qv, qws, tm = f64(d.qpos), f64(d.qvel), f64(d.qacc_warmstart), f64(d.time).reshape(nw)
  rng = np.random.default_rng(0)

  def env_step():
    a = rng.uniform(-1.0, 1.0, (nw, nact))
    ctrl = np.ascontiguousarray(a @ A.T + b)
    ol.rollout(m, q, qv, qws, ctrl, tm, dec, nthreads=threads, outputs=False)

  t0 = time.perf_counter()
  env_step()
  one = max(time.perf_counter() - t0, 1e-4)
  nsteps = int(max(3, min(200, budget_s / one)))
  t0 = time.perf_counter()
  for _ in range(nsteps):
    env_step()
  el = time.perf_counter() - t0
  # config 1: one world, zero action, single thread
  q1 = np.ascontiguousarray(m.key_qpos.reshape(1, -1), dtype=np.float64)
  v1, w1, t1 = np.zeros((1, m.nv)), np.zeros((1, m.nv)), np.zeros(1)
  c1 = np.ascontiguousarray(b.reshape(1, -1))
  t0 = time.perf_counter()
  ol.rollout(m, q1, v1, w1, c1, t1, 50 * dec, nthreads=1, outputs=False)
  one1 = max((time.perf_counter() - t0) / 50, 1e-6)
  n1 = int(max(50, min(200000, config1_s / one1)))
  t0 = time.perf_counter()
  ol.rollout(m, q1, v1, w1, c1, t1, n1 * dec, nthreads=1, outputs=False)
  el1 = time.perf_counter() - t0
  # config 1 full env: the task's ManagerBasedRlEnv on the host (torch managers on CPU
  # tensors, the oracle behind the physics boundary, tests/oracle_sim.py), num_envs = 1,
  # zero actions, measure_throughput.py's 50 warm-up + 200 timed env steps
  from oracle_sim import make_cpu_env
  task = getattr(env, "_bench_task", "Mjlab-Velocity-Flat-Unitree-G1")
  torch_threads = torch.get_num_threads()
  torch.set_num_threads(1)
  try:
    cenv = make_cpu_env(task, num_envs=1, seed=42)
    cenv.reset()
    za = torch.zeros(1, cenv.action_manager.total_action_dim)
    for _ in range(50):
      cenv.step(za)
    t0 = time.perf_counter()
    for _ in range(200):
      cenv.step(za)
    el_full = time.perf_counter() - t0
  finally:
    torch.set_num_threads(torch_threads)
  return {"value": nw * nsteps / el, "unit": "env-steps/s", "cores": threads, "kind": "port",
          "label": "CPU restatement of MuJoCo semantics (fp64 oracle, oracle/oracle.c), not MuJoCo-C",
          "sample": f"{nw} of the bench's worlds (states as the timed region left them) x "
                    f"{nsteps} env-steps ({dec} substeps each), new uniform[-1,1) actions per "
                    "env step through the action scale/offset, fp64 oracle, physics only",
          "host_cores_visible": aff, "cgroup_cpus": cgroup_cpus(),
          "config1": {"value": n1 / el1, "unit": "env-steps/s", "cores": 1, "num_envs": 1,
                      "sample": f"1 world x {n1} env-steps from the init keyframe, zero action "
                                "(--agent zero), single thread, fp64 oracle, physics only",
                      "full_env": {"value": 200 / el_full, "unit": "env-steps/s", "cores": 1,
                                   "sample": f"{task} ManagerBasedRlEnv on the host, num_envs=1, "
                                             "zero action, 50 warm-up + 200 timed env.step calls; "
                                             "torch managers on CPU tensors (1 thread) + fp64 oracle "
                                             "physics (tests/oracle_sim.py)"}}}


def traffic_profile(task, num_envs, nv):
  """Measured HBM traffic per captured env step (profiles/*_hbm_traffic.json taken by
  scripts/profile_round.sh on this task / num_envs / nv with the env-step graph path),
  latest round first."""
  import glob
  for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_hbm_traffic.json")), reverse=True):
    try:
      with open(path) as fh:
        t = json.load(fh)
    except (OSError, ValueError):
      continue
    if (t.get("task"), t.get("num_envs"), t.get("nv"), t.get("path")) == (task, num_envs, nv, "env_step_graph"):
      return t, os.path.relpath(path, ROOT)
  return None, None


MFMA_F32_PEAK_TFLOPS = 157.3  # dense fp32 MFMA (MI355X_MICROARCH.md: Peak FP32 (matrix))
# VALU issue ceiling: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles per SIMD
# (MI355X_MICROARCH.md), at the 2.4 GHz peak engine clock
N_SIMD, VALU_CYCLES_PER_INST, CLOCK_HZ = 1024, 2, 2.4e9


def reduce_over_ranks(el: float, dropped, stats: torch.Tensor, device):
  """The bench's cross-rank bookkeeping, no data-path collective:
    - episode statistics: one packed fp32 all-gather on a side stream (StatsGather),
      started first and collected last, so it overlaps the two reductions below;
    - the timed region: MAX over ranks (the slowest rank sets the job's time);
    - dropped-contact events: SUM over ranks, so every rank takes the same exit decision.
  Returns (elapsed, dropped, gathered [world, len(stats)])."""
  from mjlab_amd import distributed as mjdist
  gather = mjdist.StatsGather(int(stats.numel()), torch.device(device))
  gather.start(stats)
  el = mjdist.max_over_ranks(el, device)
  dropped = [int(v) for v in mjdist.sum_over_ranks(dropped, device)]
  return el, dropped, gather.wait()


def _launch_ranks(args_gpus: int) -> int:
  """`bench.py --gpus N` started without a launcher: start the N ranks through
  torch.distributed.run (one process per GPU, 127.0.0.1 rendezvous) before this process
  touches the GPU, and return their exit status."""
  import socket
  import subprocess
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
  cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args_gpus}",
         "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__),
         *sys.argv[1:]]
  return subprocess.call(cmd)


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
  ap.add_argument("--launch-reps", type=int, default=20,
                  help="env steps timed one by one with HIP events after the timed region")
  ap.add_argument("--engine-capacity", default=None,
                  help="diagnostic: 'C,R' or 'none' overrides the task's SimulationCfg.engine_capacity "
                       "(the fast LDS carve; worlds past it are re-solved at the max capacity)")
  ap.add_argument("--edited-scene", nargs="?", const="full", default=None, choices=["full", "sensor"],
                  help="diagnostic: the G1 velocity task with a tests/scene_edits.py cfg.scene edit, full (a heavier torso, foot friction, a contact sensor) or sensor (the contact sensor only) "
                       "(no compiled specialisation matches it: run-time specialised kernels)")
  ap.add_argument("--allow-overflow", action="store_true",
                  help="exit 0 even if contacts were dropped in the timed steps")
  args = ap.parse_args()

  from mjlab_amd import distributed as mjdist
  world, rank, local = mjdist.world_info()
  if args.gpus < 1:
    print(f"bench.py: --gpus {args.gpus} must be >= 1", file=sys.stderr)
    sys.exit(2)
  if "WORLD_SIZE" not in os.environ and args.gpus > 1:
    sys.exit(_launch_ranks(args.gpus))  # nothing has touched the GPU yet
  if world != args.gpus:
    print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
          "(torch.distributed.run --nproc-per-node N), or drop the launcher", file=sys.stderr)
    sys.exit(2)
  dist = None
  torch.cuda.set_device(local)
  if world > 1:
    import torch.distributed as dist
    mjdist.init("nccl", torch.device("cuda", local))
  device = f"cuda:{local}"

  from mjlab_amd.envs import make_env
  if args.edited_scene:
    from mjlab_amd.envs import ManagerBasedRlEnv
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests"))
    from scene_edits import edited_g1_cfg, sensor_only_g1_cfg
    cfg = (edited_g1_cfg if args.edited_scene == "full" else sensor_only_g1_cfg)(args.num_envs)
    cfg.seed = mjdist.rank_seed(42, rank)
    env = ManagerBasedRlEnv(cfg, device=device)
  elif args.engine_capacity is None:
    env = make_env(args.task, num_envs=args.num_envs, device=device, seed=mjdist.rank_seed(42, rank))
  else:
    from mjlab_amd.envs import ManagerBasedRlEnv, load_env_cfg
    cfg = load_env_cfg(args.task)
    cfg.scene.num_envs, cfg.seed = args.num_envs, mjdist.rank_seed(42, rank)
    cap = args.engine_capacity
    cfg.sim.engine_capacity = None if cap == "none" else tuple(int(v) for v in cap.split(","))
    env = ManagerBasedRlEnv(cfg, device=device)
  env._bench_task = args.task
  sim = env.sim
  m = sim.mj_model
  dec = env.cfg.decimation
  gen = torch.Generator(device=device)
  gen.manual_seed(0 + rank)
  nact = env.action_manager.total_action_dim
  env.reset()
  if args.mode == "env" and not args.eager:
    env.enable_graph(capture=True)

  def draw():
    # uniform[-1, 1) random actions, one kernel (2 * rand - 1 was three)
    return torch.empty((args.num_envs, nact), device=device).uniform_(-1.0, 1.0, generator=gen)

  def one_step(a):
    if args.mode == "env":
      env.step(a)
    else:
      env.action_manager.process_action(a)
      for _ in range(dec):
        env.action_manager.apply_action()
        env.scene.write_data_to_sim()
        sim.step()

  for _ in range(args.warmup):
    one_step(draw())
  ev_before = sim.event_counts().clone()
  sim.marker(1)  # kernel-trace bracket (outside the timing: it completes before t0)
  torch.cuda.synchronize()
  if dist is not None:
    dist.barrier()
  torch.cuda.synchronize()
  # HIP events on the launch stream around the timed steps: the per-step launch time of the
  # dominant "kernel" (one env step) as the timed region ran it, back to back
  stream = torch.cuda.current_stream()
  r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  t0 = time.perf_counter()
  r0.record(stream)
  for _ in range(args.steps):
    one_step(draw())
  r1.record(stream)
  torch.cuda.synchronize()
  if dist is not None:
    dist.barrier()
  el = time.perf_counter() - t0
  sim.marker(2)
  # contacts dropped in the timed steps (a world whose contacts or rows overflow the max
  # capacity drops whole contacts; the engine counts the events every substep) and the
  # re-solves of worlds that overflowed the fast carve
  events = (sim.event_counts() - ev_before).cpu().tolist()
  region_ms = r0.elapsed_time(r1) / args.steps
  # and, for reference, HIP events around each of `launch_reps` further single steps on the
  # stream they are launched on (torch's current stream; graph replays and the engine's
  # launches both go there): isolated replays, no overlap with a neighbour
  acts = [draw() for _ in range(args.launch_reps)]
  pairs = []
  for a in acts:
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    one_step(a)
    e1.record(stream)
    pairs.append((e0, e1))
  torch.cuda.synchronize()
  single_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in pairs]))
  launch_ms = float(region_ms)
  st = sim.stats()
  if dist is not None:
    el, events, _ = reduce_over_ranks(el, events, env.packed_episode_stats(), device)
  dropped, resolved = events[:3], int(events[3])

  total = args.steps * args.num_envs * world
  value = total / el
  if rank == 0:
    ms_step = el / args.steps * 1e3
    bytes_launch = b_env(m, dec) * args.num_envs
    launch_s = launch_ms * 1e-3
    achieved = bytes_launch / launch_s / 1e9
    graph_path = args.mode == "env" and not args.eager
    prof, prof_path = traffic_profile(args.task, args.num_envs, m.nv) if graph_path else (None, None)
    traffic = float(prof["traffic_bytes_per_env_step"]) if prof else None
    traffic_gbps = traffic / launch_s / 1e9 if traffic else None
    mfma_flops = float(prof.get("mfma_flops_per_env_step", 0.0)) if prof else 0.0
    frac_hbm = max(achieved, traffic_gbps or 0.0) / HBM_PEAK_GBS
    frac_mfma = mfma_flops / launch_s / 1e12 / MFMA_F32_PEAK_TFLOPS
    valu = float(prof["valu_insts_per_env_step"]) if prof and prof.get("valu_insts_per_env_step") else None
    frac_valu = (valu * VALU_CYCLES_PER_INST / (N_SIMD * CLOCK_HZ * launch_s)) if valu else None
    bound = "hbm" if frac_hbm >= frac_mfma else "mfma"
    step_path = ("eager" if not graph_path else "sync-free, HIP-graph captured" +
                 (", fused HIP managers" if getattr(env, "_fused", None) is not None else ""))
    out = {
      "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world,
      "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step,
      "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
      "data": "synthetic (random-init state from the compiled G1 MJCF; uniform random actions)",
      "config": {"workload": f"{args.task}{f' (tests/scene_edits.py {args.edited_scene} edit)' if args.edited_scene else ''} {'env.step' if args.mode == 'env' else 'physics-only decimation x sim.step'}",
                 "task": args.task, "num_envs_per_gpu": args.num_envs, "decimation": dec,
                 "parallelism": f"dp{world}", "mode": args.mode, "step_path": step_path,
                 "kernels": ("generic" if sim.info()["spec"] == 0 else
                             "specialised at run time (mjlab_amd.jit)" if sim.info()["spec"] >= 1000
                             else "specialised (csrc/specs.inc entry %d)" % sim.info()["spec"]),
                 "capacity": {"contacts_per_world": sim.nconmax, "rows_per_world": sim.njmax,
                              "asked": {"nconmax": env.cfg.sim.nconmax, "njmax": env.cfg.sim.njmax}}},
      "overflow": {"timed_steps": args.steps, "contact_overflow_events": int(dropped[0]),
                   "row_overflow_events": int(dropped[1]), "unsupported_pair_events": int(dropped[2]),
                   "resolved_events": resolved,
                   "fast_capacity": {"contacts_per_world": sim.fast_capacity[0],
                                     "rows_per_world": sim.fast_capacity[1]},
                   "max_contacts_seen": st["max_ncon"], "max_rows_seen": st["max_nefc"]},
      "roofline": {"bound": bound, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                   "kernel": f"one env step ({step_path}; {dec} substeps x phases A/B/C"
                             + (" + the fused manager kernels" if graph_path else "") + ")",
                   "launch_ms": launch_ms, "launch_timing": "HIP events around the timed steps / steps",
                   "single_launch_ms": single_ms, "launch_reps": args.launch_reps,
                   "bytes_per_launch": bytes_launch,
                   "bytes_per_env": b_env(m, dec),
                   "traffic_gbps": traffic_gbps, "traffic_profile": prof_path,
                   "frac_hbm_measured_traffic": (traffic_gbps / HBM_PEAK_GBS) if traffic_gbps else None,
                   "frac_mfma": frac_mfma, "mfma_flops_per_launch": mfma_flops,
                   # the ceiling that applies to this latency/issue-bound path: VALU issue
                   # slots used (SQ_INSTS_VALU of the committed SQ pass x 2 cycles over 1,024
                   # SIMDs x 2.4 GHz x launch time) and each engine kernel's waiting share
                   "frac_valu_issue": frac_valu, "valu_insts_per_launch": valu,
                   "wait_share_per_kernel": (prof or {}).get("wait_share_per_kernel"),
                   # what actually bounds the step: per-world dependency latency and issue
                   # (SQ counters in the profile), DESIGN.md section 3
                   "limiter": (prof or {}).get("limiter", "latency/VALU issue (not HBM)")},
      "cpu_baseline": None,
    }
    if not args.no_cpu_baseline and world == 1:
      out["cpu_baseline"] = cpu_baseline(env, dec)
    print(json.dumps(out), flush=True)
  if dist is not None:
    dist.destroy_process_group()
  if any(dropped) and not args.allow_overflow:
    if rank == 0:
      print(f"bench.py: contacts were dropped in the timed steps (overflow events {dropped}, "
            "all ranks); the line above reports them", file=sys.stderr)
    sys.exit(3)


if __name__ == "__main__":
  main()
