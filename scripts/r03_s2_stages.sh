#!/bin/bash
# Heavy-world stage breakdown (stamps build) and a kernel trace of the timed G1 env step.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python scripts/stage_profile.py > gpurun_out/s2_stages_all.txt 2>&1
MJX355_STAMP_MINROWS=61 timeout -k 10 200 python scripts/stage_profile.py > gpurun_out/s2_stages_heavy.txt 2>&1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s2_trace -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 20 > $GRAFT_REPO_ROOT/gpurun_out/s2_trace.log 2>&1
