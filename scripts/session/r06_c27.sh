#!/bin/bash
# round 6: kernel timeline of the unified two-class chain (MJX355_UNIFIED=1), G1 4,096
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_g1u
MJX355_UNIFIED=1 timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d gpurun_out/prof_g1u/kt -o kt -- python3 bench.py \
  --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_g1u/bench_prof.log 2>&1 || exit $?
python3 scripts/step_timeline.py gpurun_out/prof_g1u/kt 2 > gpurun_out/r06c27_timeline.txt
cat gpurun_out/r06c27_timeline.txt
