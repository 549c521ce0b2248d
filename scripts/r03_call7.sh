#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
MJX_PARITY_SOFT=1 MJX_PARITY_STATS=gpurun_out/parity5 timeout -k 10 900 python -u -m pytest \
  tests/test_gpu_rollout_parity.py -x -v -s $T > gpurun_out/r03_parity5.log 2>&1 \
  || { tail -40 gpurun_out/r03_parity5.log; exit 1; }
tail -2 gpurun_out/r03_parity5.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "not rollout and not split" $T \
  > gpurun_out/r03_gpu7.log 2>&1 || { tail -40 gpurun_out/r03_gpu7.log; exit 1; }
tail -2 gpurun_out/r03_gpu7.log
for r in 1 2; do
  for sp in 1 2; do
    MJX355_SPLIT=$sp timeout -k 10 200 python bench.py --mode physics --steps 100 --warmup 20 --no-cpu-baseline \
      > gpurun_out/r03_splitab_${sp}_$r.log 2>&1 || { tail -5 gpurun_out/r03_splitab_${sp}_$r.log; exit 1; }
    grep '^{' gpurun_out/r03_splitab_${sp}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('physics G1 split=$sp r$r', round(d['value']), round(d['ms_per_step'],4))"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v $T > gpurun_out/r03_split7.log 2>&1 \
  || { tail -30 gpurun_out/r03_split7.log; exit 1; }
tail -4 gpurun_out/r03_split7.log
mkdir -p /tmp/hip70 && ln -sf /usr/local/lib/python3.10/dist-packages/torch/lib/libamdhip64.so /tmp/hip70/libamdhip64.so.7
LD_LIBRARY_PATH=/tmp/hip70:$LD_LIBRARY_PATH timeout -k 10 60 ./scripts/capture_probe 2 1 1 0 0 0 > gpurun_out/r03_probe_hip70.log 2>&1 \
  || { cat gpurun_out/r03_probe_hip70.log; exit 1; }
cat gpurun_out/r03_probe_hip70.log
