#!/bin/bash
# round 6: Go1 batch ranges on the final build: 2 (default) vs 3 / 4
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {  # tag task n steps env...
  local tag=$1 task=$2 n=$3 st=$4; shift 4
  env "$@" timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps $st --warmup 20 --no-cpu-baseline > gpurun_out/r06c45_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c45_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4), d['overflow']['resolved_events'])"
}
for r in 1 2; do
  line go1_s2_$r Mjlab-Velocity-Flat-Unitree-Go1 8192 200 MJX355_X=0
  line go1_s3_$r Mjlab-Velocity-Flat-Unitree-Go1 8192 200 MJX355_SPLIT=3
  line go1_s4_$r Mjlab-Velocity-Flat-Unitree-Go1 8192 200 MJX355_SPLIT=4
done
