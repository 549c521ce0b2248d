#!/bin/bash
# round 6, call 2: full GPU suite with parity statistics (new: all-output fused == single
# steps, kinematics-error decomposition, fp32 cost-gap scale, descriptor validation)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06c2_stats
T="--timeout 300 --timeout-method thread"
MJX_PARITY_STATS=gpurun_out/r06c2_stats timeout -k 10 1100 python -u -m pytest tests -m gpu -v -rf $T > gpurun_out/r06c2_gpu.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed|^E  " gpurun_out/r06c2_gpu.log | tail -30 | cut -c1-300; exit $rc
