#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "not rollout" $T \
  > gpurun_out/r03_gpu9.log 2>&1 || { tail -40 gpurun_out/r03_gpu9.log; exit 1; }
tail -2 gpurun_out/r03_gpu9.log
MJX_PARITY_SOFT=1 MJX_PARITY_STATS=gpurun_out/parity7 timeout -k 10 900 python -u -m pytest \
  tests/test_gpu_rollout_parity.py -x -v -s $T > gpurun_out/r03_parity7.log 2>&1 \
  || { tail -40 gpurun_out/r03_parity7.log; exit 1; }
tail -2 gpurun_out/r03_parity7.log
LIBS="libmjx355_base.so libmjx355.so" ROUNDS="1 2" \
  TASKS="Mjlab-Velocity-Flat-Unitree-G1:4096 Mjlab-Velocity-Flat-Unitree-Go1:8192 Mjlab-Jump-Hfield-Unitree-G1:16384" \
  bash scripts/lib_ab.sh
