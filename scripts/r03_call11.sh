#!/bin/bash
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q $T > gpurun_out/r03_gpu11.log 2>&1 \
  || { tail -40 gpurun_out/r03_gpu11.log; exit 1; }
tail -2 gpurun_out/r03_gpu11.log
