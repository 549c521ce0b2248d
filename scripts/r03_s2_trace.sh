#!/bin/bash
# Kernel trace of the timed G1 env step (chain spans per substep) + per-world phase times.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TASK=${1:-Mjlab-Velocity-Flat-Unitree-G1}
NENV=${2:-4096}
rm -rf gpurun_out/s2tr
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/s2tr -o tr -- \
  python3 bench.py --task $TASK --num-envs $NENV --steps 30 --warmup 20 --no-cpu-baseline > gpurun_out/s2tr.log 2>&1
python3 scripts/chain_spans.py gpurun_out/s2tr > gpurun_out/s2tr_spans.txt
cat gpurun_out/s2tr_spans.txt
CAPS=60,1000 NENV=$NENV timeout -k 10 200 python3 scripts/world_trace.py $TASK > gpurun_out/s2_wtrace.txt 2>&1
cat gpurun_out/s2_wtrace.txt | grep -v Warn
