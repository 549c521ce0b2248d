#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
MJX_PARITY_SOFT=1 MJX_PARITY_STATS=gpurun_out/parity2 timeout -k 10 900 python -u -m pytest \
  tests/test_gpu_rollout_parity.py -x -v -s $T > gpurun_out/r03_parity2.log 2>&1 \
  || { tail -40 gpurun_out/r03_parity2.log; exit 1; }
tail -3 gpurun_out/r03_parity2.log
bash scripts/r03_mfma_ab.sh > gpurun_out/r03_mfma_ab.log 2>&1 || { tail -30 gpurun_out/r03_mfma_ab.log; exit 1; }
cat gpurun_out/r03_mfma_ab.log
for f in 1 2 4 8 15; do
  timeout -k 10 60 ./scripts/capture_probe 2 1 3 1 0 $f >> gpurun_out/r03_probe2.log 2>&1 || { cat gpurun_out/r03_probe2.log; exit 1; }
done
cat gpurun_out/r03_probe2.log
