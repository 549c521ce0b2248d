#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {  # tag task n steps env...
  local tag=$1 task=$2 n=$3 st=$4; shift 4
  env "$@" timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps $st --warmup 20 --no-cpu-baseline > gpurun_out/r06c10_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c10_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4))"
}
for t in "jh Mjlab-Jump-Hfield-Unitree-G1" "jp Mjlab-Jump-Flat-Unitree-G1"; do
  set -- $t
  line ${1}_auto $2 16384 60 MJX355_X=0
  line ${1}_c52 $2 16384 60 MJX355_ROW_CLASSES=52
  line ${1}_c72 $2 16384 60 MJX355_ROW_CLASSES=72
  line ${1}_c88 $2 16384 60 MJX355_ROW_CLASSES=88
  line ${1}_chain2 $2 16384 60 MJX355_CHAIN=2
  line ${1}_c60_120 $2 16384 60 MJX355_ROW_CLASSES=60,120
done
