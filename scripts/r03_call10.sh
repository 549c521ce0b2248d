#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
MJX_PARITY_SOFT=1 MJX_PARITY_STATS=gpurun_out/parity8 timeout -k 10 900 python -u -m pytest \
  tests/test_gpu_rollout_parity.py -x -v -s $T > gpurun_out/r03_parity8.log 2>&1 \
  || { tail -40 gpurun_out/r03_parity8.log; exit 1; }
tail -2 gpurun_out/r03_parity8.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_rollout_parity.py -x -q $T \
  > gpurun_out/r03_parity8_hard.log 2>&1 || { tail -40 gpurun_out/r03_parity8_hard.log; exit 1; }
tail -2 gpurun_out/r03_parity8_hard.log
