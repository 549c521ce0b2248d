#!/bin/bash
# Bench line of every BASELINE.json config on one GPU (config 4/5 per-GPU workloads);
# JSON lines into gpurun_out/bench_<task>.json
set -e
mkdir -p gpurun_out
run() {
  timeout -k 10 300 python bench.py --task "$1" --num-envs "$2" --steps "${3:-100}" --warmup 20 $4 > "gpurun_out/bench_$1.log" 2>&1
  grep '^{' "gpurun_out/bench_$1.log" | tail -1 > "gpurun_out/bench_$1.json"
  python3 -c "import json; d=json.load(open('gpurun_out/bench_$1.json')); print('$1', $2, round(d['value']), 'env-steps/s', round(d['ms_per_step'], 3), 'ms/step')"
}
run Mjlab-Velocity-Flat-Unitree-G1 4096 200
run Mjlab-Velocity-Flat-Unitree-Go1 8192 200 --no-cpu-baseline
run Mjlab-Tracking-Flat-Unitree-G1 4096 100 --no-cpu-baseline
run Mjlab-Jump-Flat-Unitree-G1 16384 60 --no-cpu-baseline
run Mjlab-Jump-Hfield-Unitree-G1 16384 60 --no-cpu-baseline
# SURVEY 8f row f3 (not BASELINE configs): the rough box-stair tasks
run Mjlab-Velocity-Rough-Unitree-G1 4096 200 --no-cpu-baseline
run Mjlab-Velocity-Rough-Unitree-Go1 8192 200 --no-cpu-baseline
