#!/bin/bash
# round 6: masked forward in the max carve by default (except large heightfield batches): GPU
# suite, then Go1 / rough Go1 / jump flat / jump hfield lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c41_gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06c41_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
line() {  # tag task n steps
  env timeout -k 10 200 python3 bench.py --task $2 --num-envs $3 --steps $4 --warmup 20 --no-cpu-baseline > gpurun_out/r06c41_$1.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c41_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', round(d['value']), round(d['ms_per_step'],4), d['overflow']['resolved_events'])"
}
line go1 Mjlab-Velocity-Flat-Unitree-Go1 8192 200
line rgo1 Mjlab-Velocity-Rough-Unitree-Go1 8192 200
line jf Mjlab-Jump-Flat-Unitree-G1 16384 60
line hf Mjlab-Jump-Hfield-Unitree-G1 16384 60
