#!/bin/bash
# Rollout parity error statistics (soft mode: violations recorded, not raised) of the
# current build, per config, into gpurun_out/parity/.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
MJX_PARITY_SOFT=1 MJX_PARITY_STATS=gpurun_out/parity timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_rollout_parity.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/s4_parity.log 2>&1 \
  || { tail -40 gpurun_out/s4_parity.log; exit 1; }
tail -3 gpurun_out/s4_parity.log
ls gpurun_out/parity
