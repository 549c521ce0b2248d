#!/bin/bash
# Rollout parity measurement (soft) + the bench profile passes for G1.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
MJX_PARITY_SOFT=1 MJX_PARITY_STATS=gpurun_out/parity timeout -k 10 900 python -u -m pytest \
  tests/test_gpu_rollout_parity.py -x -v -s $T > gpurun_out/r03_parity.log 2>&1 \
  || { tail -40 gpurun_out/r03_parity.log; exit 1; }
tail -3 gpurun_out/r03_parity.log
TAG=g1 bash scripts/profile_round.sh
