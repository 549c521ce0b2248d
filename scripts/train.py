"""Train a policy with PPO on the MI355X env step (the reference's `scripts/train.py` flow
with rsl_rl's OnPolicyRunner).

  python scripts/train.py --task Mjlab-Velocity-Flat-Unitree-G1 --num-envs 4096 --max-iterations 100
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 scripts/train.py ...

One process per GPU: each rank steps its own num_envs worlds with seed + rank
(`scripts/train.py:59` in the reference), rank 0's parameters are broadcast at start and
gradients are all-reduced over RCCL every mini-batch.  Prints one JSON line per iteration
(rank 0) and the final summary.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mjlab-1_amd"))

import torch  # noqa: E402


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--task", default="Mjlab-Velocity-Flat-Unitree-G1")
  ap.add_argument("--num-envs", type=int, default=4096)
  ap.add_argument("--max-iterations", type=int, default=None)
  ap.add_argument("--log-dir", default=None)
  ap.add_argument("--no-graph", action="store_true", help="eager env step (host syncs)")
  ap.add_argument("--seed", type=int, default=None)
  args = ap.parse_args()

  from mjlab_amd import distributed as mjdist
  from mjlab_amd.envs import make_env
  from mjlab_amd.rl import OnPolicyRunner, RslRlVecEnvWrapper, load_rl_cfg

  world, rank, local = mjdist.world_info()
  torch.cuda.set_device(local)
  device = f"cuda:{local}"
  if world > 1:
    mjdist.init("nccl", torch.device("cuda", local))
  cfg = load_rl_cfg(args.task)
  if args.max_iterations is not None:
    cfg.max_iterations = args.max_iterations
  seed = mjdist.rank_seed(args.seed if args.seed is not None else cfg.seed, rank)
  torch.manual_seed(seed)
  env = make_env(args.task, num_envs=args.num_envs, device=device, seed=seed)
  vec = RslRlVecEnvWrapper(env, clip_actions=cfg.clip_actions)   # resets the env
  if not args.no_graph:
    env.enable_graph(capture=True)
  log_dir = args.log_dir if rank == 0 else None
  runner = OnPolicyRunner(vec, cfg, log_dir=log_dir, device=device)
  t0 = time.perf_counter()
  hist = runner.learn(cfg.max_iterations, init_at_random_ep_len=True)
  el = time.perf_counter() - t0
  if rank == 0:
    for h in hist:
      print(json.dumps({k: v for k, v in h.items() if isinstance(v, (int, float)) or v is None}))
    print(json.dumps({"task": args.task, "num_envs_per_gpu": args.num_envs, "n_gpus": world,
                      "iterations": len(hist), "env_steps": runner.tot_timesteps,
                      "seconds": el, "env_steps_per_s": runner.tot_timesteps / el,
                      "final_mean_reward": hist[-1]["mean_reward"]}))
  if world > 1:
    import torch.distributed as dist
    dist.destroy_process_group()


if __name__ == "__main__":
  main()
