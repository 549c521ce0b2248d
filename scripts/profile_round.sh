#!/bin/bash
# GPU-box profiling recipe (run under gpurun from the repo root).  Every pass runs bench.py
# itself -- the HIP-graph-captured fused env step the bench line times -- and
# scripts/profile_bench.py attributes the dispatches between the two marker kernels that
# bracket the timed region:
#   1. kernel trace + stats (span per env step, per-kernel durations);
#   2. HBM bytes: FETCH_SIZE and WRITE_SIZE in separate --pmc passes;
#   3. SQ instruction / wait counters in their own pass (+ SQ2: optional second SQ pass).
# Outputs land in gpurun_out/prof_<tag>/; then, in the container:
#   python scripts/profile_bench.py gpurun_out/prof_<tag> <round> <task> <num_envs> <nv> <steps>
set -e
TASK=${TASK:-Mjlab-Velocity-Flat-Unitree-G1}
NENV=${NENV:-4096}
TAG=${TAG:-g1}
STEPS=${STEPS:-20}
OUT=gpurun_out/prof_${TAG}
SQ=${SQ:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM"}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --task $TASK --num-envs $NENV --steps $STEPS --warmup 5 --launch-reps 4 --no-cpu-baseline --allow-overflow"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt" -o kt -- python3 $B \
  > "$OUT/bench_prof.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/fetch" -o fetch -- python3 $B \
  > "$OUT/fetch.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/write" -o write -- python3 $B \
  > "$OUT/write.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc $SQ -f csv -d "$OUT/sq" -o sq -- python3 $B > "$OUT/sq.log" 2>&1
if [ -n "$SQ2" ]; then
  timeout -s KILL 150 rocprofv3 --pmc $SQ2 -f csv -d "$OUT/sq2" -o sq2 -- python3 $B > "$OUT/sq2.log" 2>&1
fi
echo "profile_round done: $OUT"
