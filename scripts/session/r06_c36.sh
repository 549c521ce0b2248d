#!/bin/bash
# round 6: G1 row-class cap with the capped / raised-priority heavy Newton (the heavy path now
# ends ~40 us ahead of the bulk chain): default (60) vs 56 / 52 / 48
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {  # tag task n env...
  local tag=$1 task=$2 n=$3; shift 3
  env "$@" timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r06c36_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c36_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4), d['overflow']['resolved_events'])"
}
for r in 1 2; do
  line g1_def_$r Mjlab-Velocity-Flat-Unitree-G1 4096 MJX355_X=0
  line g1_c56_$r Mjlab-Velocity-Flat-Unitree-G1 4096 MJX355_ROW_CLASSES=56
  line g1_c52_$r Mjlab-Velocity-Flat-Unitree-G1 4096 MJX355_ROW_CLASSES=52
  line g1_c48_$r Mjlab-Velocity-Flat-Unitree-G1 4096 MJX355_ROW_CLASSES=48
done
