#!/bin/bash
# round 6: jump hfield's masked forward Newton (16,384-workgroup grid) with J in global memory
# (carve kLdsJG) vs J in LDS; digest equality of the two
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {  # tag task n steps env...
  local tag=$1 task=$2 n=$3 st=$4; shift 4
  env "$@" timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps $st --warmup 20 --no-cpu-baseline > gpurun_out/r06c42_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c42_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4), d['overflow']['resolved_events'])"
}
for r in 1 2; do
  line hf_def_$r Mjlab-Jump-Hfield-Unitree-G1 16384 60 MJX355_X=0
  line hf_nojg_$r Mjlab-Jump-Hfield-Unitree-G1 16384 60 MJX355_MASKED_JG=0
done
timeout -k 10 150 python3 scripts/step_digest.py Mjlab-Jump-Hfield-Unitree-G1 8192 12 /tmp/hf_a.npz > gpurun_out/r06c42_dig.log 2>&1 || exit 1
MJX355_MASKED_JG=0 timeout -k 10 150 python3 scripts/step_digest.py Mjlab-Jump-Hfield-Unitree-G1 8192 12 /tmp/hf_b.npz >> gpurun_out/r06c42_dig.log 2>&1 || exit 1
python3 scripts/step_digest.py --compare /tmp/hf_a.npz /tmp/hf_b.npz
