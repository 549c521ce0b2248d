#!/bin/bash
# GPU suite on the current build, then base vs current bench A/B (G1, Go1, jump hfield).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q $T > gpurun_out/s2ab_gpu.log 2>&1 \
  || { tail -60 gpurun_out/s2ab_gpu.log; exit 1; }
tail -2 gpurun_out/s2ab_gpu.log
TASKS=${TASKS:-"Mjlab-Velocity-Flat-Unitree-G1:4096 Mjlab-Velocity-Flat-Unitree-Go1:8192 Mjlab-Jump-Hfield-Unitree-G1:16384"} \
  ./scripts/lib_ab.sh
