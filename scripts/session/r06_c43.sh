#!/bin/bash
# round 6: jump 16,384 topology knobs on the current build: bulk chain at any size
# (MJX355_CHAIN=2), the full-capacity class's J mode (MJX355_NEWTON_JG 0 / 1)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {  # tag task n steps env...
  local tag=$1 task=$2 n=$3 st=$4; shift 4
  env "$@" timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps $st --warmup 20 --no-cpu-baseline > gpurun_out/r06c43_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c43_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4), d['overflow']['resolved_events'])"
}
for r in 1 2; do
  line jf_def_$r Mjlab-Jump-Flat-Unitree-G1 16384 60 MJX355_X=0
  line jf_ch2_$r Mjlab-Jump-Flat-Unitree-G1 16384 60 MJX355_CHAIN=2
  line jf_jg1_$r Mjlab-Jump-Flat-Unitree-G1 16384 60 MJX355_NEWTON_JG=1
  line hf_def_$r Mjlab-Jump-Hfield-Unitree-G1 16384 60 MJX355_X=0
  line hf_ch2_$r Mjlab-Jump-Hfield-Unitree-G1 16384 60 MJX355_CHAIN=2
done
