#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06c6_stats
T="--timeout 300 --timeout-method thread"
MJX_PARITY_STATS=gpurun_out/r06c6_stats timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf $T > gpurun_out/r06c6_gpu.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed|^E  " gpurun_out/r06c6_gpu.log | tail -30 | cut -c1-700; exit $rc
