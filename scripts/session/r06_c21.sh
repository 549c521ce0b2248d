#!/bin/bash
# round 6 final build: rocprof sets (kernel stats, timed region, HBM traffic, SQ) of G1, Go1,
# tracking and jump hfield; G1 row-class sweep
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
NO_BENCH=1 ROUND=r06 PROF_SPECS="g1 Mjlab-Velocity-Flat-Unitree-G1 4096 35;go1 Mjlab-Velocity-Flat-Unitree-Go1 8192 18;tracking Mjlab-Tracking-Flat-Unitree-G1 4096 35;jump_hfield Mjlab-Jump-Hfield-Unitree-G1 16384 35" \
  timeout -k 10 1000 bash scripts/round_final.sh > gpurun_out/r06c21_final.log 2>&1
rc=$?; tail -3 gpurun_out/r06c21_final.log; [ $rc -eq 0 ] || exit $rc
line() {  # tag steps env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r06c21_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c21_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4))"
}
for r in 1 2; do
  line g1_default_$r MJX355_X=0
  line g1_c52_$r MJX355_ROW_CLASSES=52
  line g1_c56_$r MJX355_ROW_CLASSES=56
done
