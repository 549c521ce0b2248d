#!/bin/bash
# round 6: both row classes in one chain launch (MJX355_UNIFIED=1) and the register-capped heavy
# Newton (MJX355_HEAVY_CAP=1) against the default; bit-equality of the unified step (step_digest)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/step_digest.py Mjlab-Velocity-Flat-Unitree-G1 1024 12 gpurun_out/r06c26_def.npz > gpurun_out/r06c26_dig.log 2>&1 || { tail -5 gpurun_out/r06c26_dig.log; exit 1; }
MJX355_UNIFIED=1 timeout -k 10 120 python3 scripts/step_digest.py Mjlab-Velocity-Flat-Unitree-G1 1024 12 gpurun_out/r06c26_uni.npz >> gpurun_out/r06c26_dig.log 2>&1 || { tail -5 gpurun_out/r06c26_dig.log; exit 1; }
python3 scripts/step_digest.py --compare gpurun_out/r06c26_def.npz gpurun_out/r06c26_uni.npz
line() {  # tag task n env...
  local tag=$1 task=$2 n=$3; shift 3
  env "$@" timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r06c26_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c26_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4), d['overflow']['resolved_events'])"
}
for r in 1 2; do
  line g1_def_$r Mjlab-Velocity-Flat-Unitree-G1 4096 MJX355_X=0
  line g1_uni_$r Mjlab-Velocity-Flat-Unitree-G1 4096 MJX355_UNIFIED=1
  line g1_cap_$r Mjlab-Velocity-Flat-Unitree-G1 4096 MJX355_HEAVY_CAP=1
  line g1_capjg_$r Mjlab-Velocity-Flat-Unitree-G1 4096 MJX355_HEAVY_CAP=1 MJX355_NEWTON_JG=1
  line tr_def_$r Mjlab-Tracking-Flat-Unitree-G1 4096 MJX355_X=0
  line tr_uni_$r Mjlab-Tracking-Flat-Unitree-G1 4096 MJX355_UNIFIED=1
done
