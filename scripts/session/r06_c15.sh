#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="--timeout 300 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf $T -k "fused or curriculum or jump" > gpurun_out/r06c15_gpu.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed|^E  " gpurun_out/r06c15_gpu.log | tail -20 | cut -c1-600; [ $rc -eq 0 ] || exit $rc
ROUNDS="1 2" STEPS=100 LIBS="libmjx355_base.so libmjx355.so" \
TASKS="Mjlab-Velocity-Flat-Unitree-G1:4096 Mjlab-Velocity-Flat-Unitree-Go1:8192" timeout -k 10 700 bash scripts/lib_ab.sh
