#!/bin/bash
# Round 3, session 3: tree-form SPD factors (rows_chol_tree).  Factor + solve microbenchmark,
# the full GPU suite on the new build, then an interleaved A/B against the HEAD build.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/chol_bench.sh > gpurun_out/s3_chol.log 2>&1 || { tail -20 gpurun_out/s3_chol.log; exit 1; }
cat gpurun_out/s3_chol.log
T="--timeout 300 --timeout-method thread"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v $T > gpurun_out/s3t_gpu.log 2>&1 \
  || { tail -60 gpurun_out/s3t_gpu.log; exit 1; }
tail -2 gpurun_out/s3t_gpu.log
TASKS="Mjlab-Velocity-Flat-Unitree-G1:4096 Mjlab-Velocity-Flat-Unitree-Go1:8192 Mjlab-Jump-Hfield-Unitree-G1:16384" \
  bash scripts/lib_ab.sh
