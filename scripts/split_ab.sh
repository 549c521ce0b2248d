#!/bin/bash
# A/B of the batch split (MJX355_SPLIT=1: one launch set per phase, 2: concurrent halves)
# on bench.py lines.  TASKS="task:num_envs ..." selects the workloads.
set -e
TASKS=${TASKS:-"Mjlab-Velocity-Flat-Unitree-G1:4096 Mjlab-Velocity-Flat-Unitree-Go1:8192"}
SPLITS=${SPLITS:-"1 2"}
for tn in $TASKS; do
  for sp in $SPLITS; do
    out=gpurun_out/split_${tn%%:*}_$sp.log
    MJX355_SPLIT=$sp timeout -k 10 150 python3 bench.py --task "${tn%%:*}" --num-envs "${tn##*:}" \
      --steps 100 --warmup 20 --no-cpu-baseline > "$out" 2>&1
    grep '^{' "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('${tn%%:*} split $sp', round(d['value']), 'env-steps/s', round(d['ms_per_step'],3), 'ms/step')"
  done
done
