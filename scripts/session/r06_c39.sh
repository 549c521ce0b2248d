#!/bin/bash
# round 6: Go1's masked forward (reset worlds, nearly every env step) fused in the max carve
# (MJX355_MASKED_BIG=1) vs three fast-carve launches (the default above 4,096 worlds)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {  # tag task n env...
  local tag=$1 task=$2 n=$3; shift 3
  env "$@" timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r06c39_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c39_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4), d['overflow']['resolved_events'])"
}
for r in 1 2; do
  line go1_def_$r Mjlab-Velocity-Flat-Unitree-Go1 8192 MJX355_X=0
  line go1_mb_$r Mjlab-Velocity-Flat-Unitree-Go1 8192 MJX355_MASKED_BIG=1
  line rgo1_def_$r Mjlab-Velocity-Rough-Unitree-Go1 8192 MJX355_X=0
  line rgo1_mb_$r Mjlab-Velocity-Rough-Unitree-Go1 8192 MJX355_MASKED_BIG=1
  line jf_def_$r Mjlab-Jump-Flat-Unitree-G1 16384 MJX355_X=0
  line jf_mb_$r Mjlab-Jump-Flat-Unitree-G1 16384 MJX355_MASKED_BIG=1
done
