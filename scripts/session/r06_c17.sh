#!/bin/bash
# Go1: phase B / chain at 128 VGPRs (4 waves / SIMD) and a 16 / 64 fast carve (16 worlds / CU)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {  # tag lib task n steps extra...
  local tag=$1 lib=$2 task=$3 n=$4 st=$5; shift 5
  MJX355_LIB=$PWD/mjlab-1_amd/mjlab_amd/$lib timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps $st --warmup 20 --no-cpu-baseline "$@" > gpurun_out/r06c17_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c17_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); o=d['overflow']; print('$tag', round(d['value']), round(d['ms_per_step'],4), d['config'].get('kernels'), 'resolved', o['resolved_events'])"
}
for r in 1 2; do
  line go1_base_$r libmjx355_base.so Mjlab-Velocity-Flat-Unitree-Go1 8192 100
  line go1_b4_$r libmjx355.so Mjlab-Velocity-Flat-Unitree-Go1 8192 100
  line go1_b4c16_$r libmjx355.so Mjlab-Velocity-Flat-Unitree-Go1 8192 100 --engine-capacity 16,64
  line rgo1_base_$r libmjx355_base.so Mjlab-Velocity-Rough-Unitree-Go1 8192 100
  line rgo1_b4c16_$r libmjx355.so Mjlab-Velocity-Rough-Unitree-Go1 8192 100 --engine-capacity 16,64
done
