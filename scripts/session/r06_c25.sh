#!/bin/bash
# round 6: the full-capacity class's latency Newton at 168 VGPRs (MJX355_HEAVY_CAP=1)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {  # tag task n env...
  local tag=$1 task=$2 n=$3; shift 3
  env "$@" timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r06c25_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c25_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4), d['overflow']['resolved_events'])"
}
for r in 1 2; do
  line g1_def_$r Mjlab-Velocity-Flat-Unitree-G1 4096 MJX355_X=0
  line g1_cap_$r Mjlab-Velocity-Flat-Unitree-G1 4096 MJX355_HEAVY_CAP=1
  line g1_capjg_$r Mjlab-Velocity-Flat-Unitree-G1 4096 MJX355_HEAVY_CAP=1 MJX355_NEWTON_JG=1
  line tr_def_$r Mjlab-Tracking-Flat-Unitree-G1 4096 MJX355_X=0
  line tr_cap_$r Mjlab-Tracking-Flat-Unitree-G1 4096 MJX355_HEAVY_CAP=1
done
