#!/bin/bash
# GPU-box profiling recipe (run under gpurun from the repo root):
#   1. kernel trace + stats of the default bench command (short K/W);
#   2. HBM bytes: FETCH_SIZE and WRITE_SIZE in separate --pmc passes over the physics loop;
#   3. SQ instruction / wait counters in their own pass.
# Outputs land in gpurun_out/prof_<tag>/; scripts/profile_summary.py turns them into
# the profiles/<round>_* files that are committed.
set -e
TASK=${TASK:-Mjlab-Velocity-Flat-Unitree-G1}
NENV=${NENV:-4096}
TAG=${TAG:-g1}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o kt -- \
  python3 bench.py --task "$TASK" --num-envs "$NENV" --steps 50 --warmup 20 --no-cpu-baseline \
  > "$OUT/bench_prof.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/fetch" -o fetch -- \
  python3 scripts/physics_loop.py "$TASK" "$NENV" > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/write" -o write -- \
  python3 scripts/physics_loop.py "$TASK" "$NENV" > "$OUT/write.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU \
  SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM -f csv -d "$OUT/sq" -o sq -- \
  python3 scripts/physics_loop.py "$TASK" "$NENV" > "$OUT/sq.log" 2>&1
echo "profile_round done: $OUT"
