#!/bin/bash
# round 6: kernel trace of the captured G1 env step, per-substep spans by queue (chain_spans)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_g1t
timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d gpurun_out/prof_g1t/kt -o kt -- python3 bench.py \
  --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_g1t/bench_prof.log 2>&1 || exit $?
python3 scripts/chain_spans.py gpurun_out/prof_g1t/kt 60 > gpurun_out/r06c24_chain_spans.txt 2>&1
cat gpurun_out/r06c24_chain_spans.txt
