#!/bin/bash
# Round-3 GPU check: split x row-class capture, rollout parity (soft, with stats), the GPU
# suite, the default bench line and the counter list.  Each step has its own time limit;
# the first failure ends the script.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
MJX_PARITY_SOFT=1 MJX_PARITY_STATS=gpurun_out/parity timeout -k 10 900 python -u -m pytest \
  tests/test_gpu_rollout_parity.py -x -v -s $T > gpurun_out/r03_parity.log 2>&1 \
  || { tail -40 gpurun_out/r03_parity.log; exit 1; }
tail -3 gpurun_out/r03_parity.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -k "not rollout and not split" $T \
  > gpurun_out/r03_gpu.log 2>&1 || { tail -40 gpurun_out/r03_gpu.log; exit 1; }
tail -3 gpurun_out/r03_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/r03_bench.log 2>&1 || { tail -20 gpurun_out/r03_bench.log; exit 1; }
grep '^{' gpurun_out/r03_bench.log
timeout -k 10 120 rocprofv3 -L > gpurun_out/r03_counters.txt 2>&1 || true
grep -i mfma gpurun_out/r03_counters.txt | head -20 || true
# capture topology probes, known-good first; a crash ends the chain (the last printed
# configuration is the first that fails)
for v in "1 1 3 1" "2 0 3 0" "2 1 1 0" "2 1 3 0" "2 1 3 1" "2 2 3 1" "2 1 3 1 1"; do
  timeout -k 10 60 ./scripts/capture_probe $v >> gpurun_out/r03_probe.log 2>&1 || { cat gpurun_out/r03_probe.log; exit 1; }
done
cat gpurun_out/r03_probe.log
