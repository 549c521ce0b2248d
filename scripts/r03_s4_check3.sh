#!/bin/bash
# Round 3, session 4: GPU suite + smoke on the v4 build (warmstart's two J q products in one
# pass), then the main / v4 library A/B.  Each step has its own limit.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
V=$PWD/mjlab-1_amd/mjlab_amd/libmjx355_v5.so
MJX355_LIB=$V timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v $T > gpurun_out/s4c3_gpu.log 2>&1 \
  || { tail -60 gpurun_out/s4c3_gpu.log; exit 1; }
tail -3 gpurun_out/s4c3_gpu.log
LIBS="libmjx355.so libmjx355_v4.so libmjx355_v5.so" TASKS="Mjlab-Velocity-Flat-Unitree-G1:4096 Mjlab-Jump-Hfield-Unitree-G1:16384" \
  ROUNDS="1 2" bash scripts/lib_ab.sh 2>&1 | tee gpurun_out/s4_libab3.txt
