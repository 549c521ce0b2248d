#!/bin/bash
# Capture crash bisection (a crash ends the chain) + the stamps breakdown of heavy worlds.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
MJX_PARITY_SOFT=1 MJX_PARITY_STATS=gpurun_out/parity4 timeout -k 10 900 python -u -m pytest \
  tests/test_gpu_rollout_parity.py -x -v -s $T > gpurun_out/r03_parity4.log 2>&1 \
  || { tail -40 gpurun_out/r03_parity4.log; exit 1; }
tail -3 gpurun_out/r03_parity4.log
MJX355_STAMP_MINROWS=61 timeout -k 10 300 python -u scripts/stage_profile.py > gpurun_out/r03_stamps_heavy.log 2>&1 \
  || { tail -20 gpurun_out/r03_stamps_heavy.log; exit 1; }
timeout -k 10 300 python -u scripts/stage_profile.py > gpurun_out/r03_stamps_all.log 2>&1 \
  || { tail -20 gpurun_out/r03_stamps_all.log; exit 1; }
cat gpurun_out/r03_stamps_heavy.log gpurun_out/r03_stamps_all.log
for v in "2 1 1 0 0 0" "2 1 3 1 0 15"; do
  timeout -k 10 120 python -u scripts/capture_probe_torch.py $v >> gpurun_out/r03_cprobe6.log 2>&1 \
    || { cat gpurun_out/r03_cprobe6.log; exit 1; }
done
timeout -k 10 120 python -u scripts/capture_probe_engine.py 2 24 0 1 0 1 >> gpurun_out/r03_cprobe6.log 2>&1 \
  || { cat gpurun_out/r03_cprobe6.log; exit 1; }
cat gpurun_out/r03_cprobe6.log
