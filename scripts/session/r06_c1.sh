#!/bin/bash
# round 6, first call: smoke + driver command twice (baseline of this round's build)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06c1_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r06c1_smoke.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06c1_driver$i.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c1_driver$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver', round(d['value']), d['ms_per_step'])"
done
timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r06c1_long.log 2>&1 || exit $?
grep '^{' gpurun_out/r06c1_long.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('long', round(d['value']), d['ms_per_step'])"
