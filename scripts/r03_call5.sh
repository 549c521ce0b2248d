#!/bin/bash
# LTR hand-off build: GPU suite + rollout parity (soft stats) + bench + profile, then the
# engine capture bisection (a crash ends the chain: the last printed configuration is the
# first that fails).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "not rollout and not split" $T \
  > gpurun_out/r03_gpu5.log 2>&1 || { tail -40 gpurun_out/r03_gpu5.log; exit 1; }
tail -2 gpurun_out/r03_gpu5.log
MJX_PARITY_SOFT=1 MJX_PARITY_STATS=gpurun_out/parity3 timeout -k 10 900 python -u -m pytest \
  tests/test_gpu_rollout_parity.py -x -v -s $T > gpurun_out/r03_parity3.log 2>&1 \
  || { tail -40 gpurun_out/r03_parity3.log; exit 1; }
tail -3 gpurun_out/r03_parity3.log
timeout -k 10 400 python bench.py > gpurun_out/r03_bench5.log 2>&1 || { tail -20 gpurun_out/r03_bench5.log; exit 1; }
grep '^{' gpurun_out/r03_bench5.log | cut -c1-400
TAG=g1ltr bash scripts/profile_round.sh
for v in "2 24 0 1 0" "2 24 0 3 0" "2 24 0 1 1" "2 24 2 3 1"; do
  timeout -k 10 120 python -u scripts/capture_probe_engine.py $v >> gpurun_out/r03_cprobe5.log 2>&1 \
    || { cat gpurun_out/r03_cprobe5.log; exit 1; }
done
cat gpurun_out/r03_cprobe5.log
