#!/bin/bash
# round 6: rocprof sets for configs 4 and 5 (tracking 4,096, jump hfield 16,384) and the
# per-stage breakdown of heavy G1 / jump-hfield worlds (stamps build)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
NO_BENCH=1 ROUND=r06 PROF_SPECS="tracking Mjlab-Tracking-Flat-Unitree-G1 4096 35;jump_hfield Mjlab-Jump-Hfield-Unitree-G1 16384 35" \
  timeout -k 10 900 bash scripts/round_final.sh > gpurun_out/r06c11_final.log 2>&1
rc=$?; tail -3 gpurun_out/r06c11_final.log; [ $rc -eq 0 ] || exit $rc
MJX355_STAMP_MINROWS=61 timeout -k 10 200 python3 scripts/stage_profile.py Mjlab-Velocity-Flat-Unitree-G1 > gpurun_out/r06c11_stages_g1_heavy.txt 2>&1 || exit $?
timeout -k 10 200 python3 scripts/stage_profile.py Mjlab-Velocity-Flat-Unitree-G1 > gpurun_out/r06c11_stages_g1.txt 2>&1 || exit $?
NENV=16384 MJX355_STAMP_MINROWS=61 timeout -k 10 300 python3 scripts/stage_profile.py Mjlab-Jump-Hfield-Unitree-G1 > gpurun_out/r06c11_stages_jh_heavy.txt 2>&1 || exit $?
head -8 gpurun_out/r06c11_stages_g1_heavy.txt; head -8 gpurun_out/r06c11_stages_jh_heavy.txt
