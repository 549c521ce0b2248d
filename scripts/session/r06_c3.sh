#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06c3_stats
T="--timeout 300 --timeout-method thread"
MJX_PARITY_STATS=gpurun_out/r06c3_stats timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf $T > gpurun_out/r06c3_gpu.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed|^E  " gpurun_out/r06c3_gpu.log | tail -30 | cut -c1-600; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/class_transitions.py Mjlab-Velocity-Flat-Unitree-G1 4096 60 30 > gpurun_out/r06c3_trans_g1.log 2>&1 || exit $?
tail -1 gpurun_out/r06c3_trans_g1.log
timeout -k 10 300 python -u scripts/class_transitions.py Mjlab-Jump-Hfield-Unitree-G1 16384 60 20 > gpurun_out/r06c3_trans_jh.log 2>&1 || exit $?
tail -1 gpurun_out/r06c3_trans_jh.log
