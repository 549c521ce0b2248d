#!/bin/bash
# round 6: unified two-class chain with the re-solve in line ahead of it; timeline + A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_g1u2
MJX355_UNIFIED=1 timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d gpurun_out/prof_g1u2/kt -o kt -- python3 bench.py \
  --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_g1u2/bench_prof.log 2>&1 || exit $?
python3 scripts/step_timeline.py gpurun_out/prof_g1u2/kt 2 > gpurun_out/r06c28_timeline.txt
cat gpurun_out/r06c28_timeline.txt
line() {  # tag task n env...
  local tag=$1 task=$2 n=$3; shift 3
  env "$@" timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r06c28_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c28_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4), d['overflow']['resolved_events'])"
}
for r in 1 2; do
  line g1_def_$r Mjlab-Velocity-Flat-Unitree-G1 4096 MJX355_X=0
  line g1_uni_$r Mjlab-Velocity-Flat-Unitree-G1 4096 MJX355_UNIFIED=1
  line tr_def_$r Mjlab-Tracking-Flat-Unitree-G1 4096 MJX355_X=0
  line tr_uni_$r Mjlab-Tracking-Flat-Unitree-G1 4096 MJX355_UNIFIED=1
done
