#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06c14_stats
T="--timeout 300 --timeout-method thread"
MJX_PARITY_STATS=gpurun_out/r06c14_stats timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf $T > gpurun_out/r06c14_gpu.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed|^E  " gpurun_out/r06c14_gpu.log | tail -20 | cut -c1-600; [ $rc -eq 0 ] || exit $rc
line() {  # tag task n steps env...
  local tag=$1 task=$2 n=$3 st=$4; shift 4
  env "$@" timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps $st --warmup 20 --no-cpu-baseline > gpurun_out/r06c14_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c14_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4))"
}
for r in 1 2; do
  line jh_auto_$r Mjlab-Jump-Hfield-Unitree-G1 16384 60 MJX355_X=0
  line jh_chain2_$r Mjlab-Jump-Hfield-Unitree-G1 16384 60 MJX355_CHAIN=2
  line jh_c52_$r Mjlab-Jump-Hfield-Unitree-G1 16384 60 MJX355_ROW_CLASSES=52
done
