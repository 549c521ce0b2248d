#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {  # tag task n steps env...
  local tag=$1 task=$2 n=$3 st=$4; shift 4
  env "$@" timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps $st --warmup 20 --no-cpu-baseline > gpurun_out/r06c9_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c9_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4))"
}
for r in 1 2; do
  line jh_auto_$r Mjlab-Jump-Hfield-Unitree-G1 16384 60 MJX355_X=0
  line jh_noclass_jg2_$r Mjlab-Jump-Hfield-Unitree-G1 16384 60 MJX355_NEWTON_JG=2 MJX355_ROW_CLASSES=
  line jp_jg0_$r Mjlab-Jump-Flat-Unitree-G1 16384 60 MJX355_NEWTON_JG=0
  line jp_auto_$r Mjlab-Jump-Flat-Unitree-G1 16384 60 MJX355_X=0
  line g1_jg2_$r Mjlab-Velocity-Flat-Unitree-G1 4096 100 MJX355_NEWTON_JG=2
  line g1_auto_$r Mjlab-Velocity-Flat-Unitree-G1 4096 100 MJX355_X=0
  line tr_jg2_$r Mjlab-Tracking-Flat-Unitree-G1 4096 100 MJX355_NEWTON_JG=2
  line tr_auto_$r Mjlab-Tracking-Flat-Unitree-G1 4096 100 MJX355_X=0
done
