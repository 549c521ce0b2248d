#!/bin/bash
# Round 3, session 4: full GPU suite, smoke, the default bench line, and the tracking line
# with overflow enforced (engine_capacity 64 / 250).  Each step has its own limit.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v $T > gpurun_out/s4_gpu.log 2>&1 \
  || { tail -60 gpurun_out/s4_gpu.log; exit 1; }
tail -3 gpurun_out/s4_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s4_smoke.log 2>&1 \
  || { tail -20 gpurun_out/s4_smoke.log; exit 1; }
tail -1 gpurun_out/s4_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/s4_bench.log 2>&1 || { tail -20 gpurun_out/s4_bench.log; exit 1; }
grep '^{' gpurun_out/s4_bench.log | cut -c1-200
timeout -k 10 300 python bench.py --task Mjlab-Tracking-Flat-Unitree-G1 --steps 100 --warmup 20 --no-cpu-baseline \
  > gpurun_out/s4_track.log 2>&1 || { tail -20 gpurun_out/s4_track.log; exit 1; }
grep '^{' gpurun_out/s4_track.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), d['ms_per_step'], d['overflow'], d['config']['capacity'])"
