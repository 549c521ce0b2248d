#!/bin/bash
# round 6: rocprof sets for configs 4 and 5 (tracking 4,096, jump hfield 16,384) and the
# per-stage breakdown of heavy G1 worlds (stamps build)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
NO_BENCH=1 ROUND=r06 PROF_SPECS="tracking Mjlab-Tracking-Flat-Unitree-G1 4096 35;jump_hfield Mjlab-Jump-Hfield-Unitree-G1 16384 35" \
  timeout -k 10 900 bash scripts/round_final.sh > gpurun_out/r06c5_final.log 2>&1
rc=$?; tail -3 gpurun_out/r06c5_final.log; [ $rc -eq 0 ] || exit $rc
MJX355_STAMP_MINROWS=61 timeout -k 10 200 python3 scripts/stage_profile.py Mjlab-Velocity-Flat-Unitree-G1 > gpurun_out/r06c5_stages_g1_heavy.txt 2>&1 || exit $?
timeout -k 10 200 python3 scripts/stage_profile.py Mjlab-Velocity-Flat-Unitree-G1 > gpurun_out/r06c5_stages_g1.txt 2>&1 || exit $?
NENV=16384 MJX355_STAMP_MINROWS=61 timeout -k 10 300 python3 scripts/stage_profile.py Mjlab-Jump-Hfield-Unitree-G1 > gpurun_out/r06c5_stages_jh_heavy.txt 2>&1 || exit $?
head -20 gpurun_out/r06c5_stages_g1_heavy.txt
# row-class sweep on the current build (G1 driver-like lines, 100 steps)
for rc in default "60,120" "52,116" "60,96"; do
  if [ "$rc" = default ]; then E=""; else E="MJX355_ROW_CLASSES=$rc"; fi
  env $E timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r06c5_rc_${rc/,/_}.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c5_rc_${rc/,/_}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('classes $rc', round(d['value']), d['ms_per_step'])"
done
