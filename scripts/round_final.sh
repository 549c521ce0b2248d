#!/bin/bash
# End-of-session GPU pass: bench line of every config (scripts/bench_configs.sh), then the
# profile recipe (scripts/profile_round.sh) for G1 and Go1, summarised on the box into
# profiles/<ROUND>_* copies under gpurun_out/profiles_new/ (the raw rocprof traces exceed
# gpurun's 64 MiB return limit and are deleted after summarising).
set -e
ROUND=${ROUND:-r02}
mkdir -p gpurun_out/profiles_new
[ -z "$NO_BENCH" ] && bash scripts/bench_configs.sh > gpurun_out/final_bench.txt 2>&1
# PROF_SPECS: "tag task num_envs nv" entries separated by ';' (default: G1 and Go1)
PROF_SPECS=${PROF_SPECS:-"g1 Mjlab-Velocity-Flat-Unitree-G1 4096 35;go1 Mjlab-Velocity-Flat-Unitree-Go1 8192 18"}
IFS=';' read -ra SPECS <<< "$PROF_SPECS"
for spec in "${SPECS[@]}"; do
  set -- $spec
  TAG=$1 TASK=$2 NENV=$3 bash scripts/profile_round.sh > gpurun_out/final_prof_$1.txt 2>&1
  python3 scripts/profile_bench.py gpurun_out/prof_$1 "$ROUND" "$2" "$3" "$4" 20 >> gpurun_out/final_prof_$1.txt 2>&1
  cp profiles/${ROUND}_$1_* gpurun_out/profiles_new/
  rm -rf gpurun_out/prof_$1
done
echo "round_final done"
