#!/bin/bash
# Round 3, session 3: full GPU suite, smoke, the default bench line.  Each step has its own
# limit; the first failure ends the script.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v $T > gpurun_out/s3_gpu.log 2>&1 \
  || { tail -60 gpurun_out/s3_gpu.log; exit 1; }
tail -3 gpurun_out/s3_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3_smoke.log 2>&1 \
  || { tail -20 gpurun_out/s3_smoke.log; exit 1; }
tail -1 gpurun_out/s3_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/s3_bench.log 2>&1 || { tail -20 gpurun_out/s3_bench.log; exit 1; }
grep '^{' gpurun_out/s3_bench.log
