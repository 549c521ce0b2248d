#!/bin/bash
# Rollout parity measurement (soft) + the bench profile passes for G1.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
MJX_PARITY_SOFT=1 MJX_PARITY_STATS=gpurun_out/parity timeout -k 10 900 python -u -m pytest \
  tests/test_gpu_rollout_parity.py -x -v -s $T > gpurun_out/r03_parity.log 2>&1 \
  || { tail -40 gpurun_out/r03_parity.log; exit 1; }
tail -3 gpurun_out/r03_parity.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_random.py tests/test_gpu_fused.py tests/test_gpu_sim.py \
  -v $T > gpurun_out/r03_new.log 2>&1 && rc=0 || rc=$?
tail -15 gpurun_out/r03_new.log
[ $rc -le 1 ] || exit 1   # 1 = test failures (read the log); anything else = stop here
TAG=g1 bash scripts/profile_round.sh
python scripts/profile_bench.py gpurun_out/prof_g1 r03 Mjlab-Velocity-Flat-Unitree-G1 4096 35 20 > gpurun_out/prof_g1/summary.txt 2>&1 || true
# engine capture probe (may crash: last step)
timeout -k 10 120 python -u scripts/capture_probe_engine.py 2 24 0 > gpurun_out/r03_cprobe.log 2>&1 || { cat gpurun_out/r03_cprobe.log; exit 1; }
cat gpurun_out/r03_cprobe.log
