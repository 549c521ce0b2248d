#!/bin/bash
# lean specialisation (Go1 flat at 16 / 64, phase B and chain at 4 waves / SIMD): full GPU suite,
# then A/B against the previous build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06c18_stats
T="--timeout 300 --timeout-method thread"
MJX_PARITY_STATS=gpurun_out/r06c18_stats timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf $T > gpurun_out/r06c18_gpu.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed|^E  " gpurun_out/r06c18_gpu.log | tail -20 | cut -c1-600; [ $rc -eq 0 ] || exit $rc
ROUNDS="1 2" STEPS=100 LIBS="libmjx355_base.so libmjx355.so" \
TASKS="Mjlab-Velocity-Flat-Unitree-Go1:8192 Mjlab-Velocity-Rough-Unitree-Go1:8192" timeout -k 10 600 bash scripts/lib_ab.sh
