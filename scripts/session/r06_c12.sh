#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06c12_stats
T="--timeout 300 --timeout-method thread"
MJX_PARITY_STATS=gpurun_out/r06c12_stats timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf $T -k "rollout or jump or hfield or overflow or carve" > gpurun_out/r06c12_gpu.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed|^E  " gpurun_out/r06c12_gpu.log | tail -20 | cut -c1-600; [ $rc -eq 0 ] || exit $rc
line() {  # tag task n steps env...
  local tag=$1 task=$2 n=$3 st=$4; shift 4
  env "$@" timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps $st --warmup 20 --no-cpu-baseline > gpurun_out/r06c12_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c12_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4))"
}
for r in 1 2; do
  line jh_jg0_$r Mjlab-Jump-Hfield-Unitree-G1 16384 60 MJX355_NEWTON_JG=0
  line jh_auto_$r Mjlab-Jump-Hfield-Unitree-G1 16384 60 MJX355_X=0
  line jp_jg0_$r Mjlab-Jump-Flat-Unitree-G1 16384 60 MJX355_NEWTON_JG=0
  line jp_auto_$r Mjlab-Jump-Flat-Unitree-G1 16384 60 MJX355_X=0
done
