#!/bin/bash
# round 6: in-line re-solve grid 1 as the default: GPU suite, then Go1 / rough Go1 / G1 lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=8 > gpurun_out/r06c34_gpu_tests.log 2>&1
rc=$?; tail -14 gpurun_out/r06c34_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
line() {  # tag task n env...
  local tag=$1 task=$2 n=$3; shift 3
  env "$@" timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r06c34_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c34_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4), d['overflow']['resolved_events'])"
}
for r in 1 2; do
  line go1_def_$r Mjlab-Velocity-Flat-Unitree-Go1 8192 MJX355_X=0
  line go1_g32_$r Mjlab-Velocity-Flat-Unitree-Go1 8192 MJX355_OVF_GRID=32
  line rgo1_def_$r Mjlab-Velocity-Rough-Unitree-Go1 8192 MJX355_X=0
  line rgo1_g32_$r Mjlab-Velocity-Rough-Unitree-Go1 8192 MJX355_OVF_GRID=32
done
