#!/bin/bash
# round 6: the capped, raised-priority heavy Newton as the default for <= 160-row fast carves:
# GPU suite, smoke, and A/B against MJX355_HEAVY_CAP=0
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c31_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06c31_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06c31_smoke.log 2>&1 || { tail -5 gpurun_out/r06c31_smoke.log; exit 1; }
tail -1 gpurun_out/r06c31_smoke.log
line() {  # tag task n env...
  local tag=$1 task=$2 n=$3; shift 3
  env "$@" timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r06c31_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c31_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4), d['overflow']['resolved_events'])"
}
for r in 1 2; do
  line g1_def_$r Mjlab-Velocity-Flat-Unitree-G1 4096 MJX355_X=0
  line g1_cap0_$r Mjlab-Velocity-Flat-Unitree-G1 4096 MJX355_HEAVY_CAP=0
  line hf_def_$r Mjlab-Jump-Hfield-Unitree-G1 16384 MJX355_X=0
done
