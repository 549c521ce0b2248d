#!/bin/bash
# A/B of one engine environment knob on bench.py lines: VAR=<name> VALS="<a> <b>"
# TASKS="task:num_envs ...".
set -e
TASKS=${TASKS:-"Mjlab-Velocity-Flat-Unitree-G1:4096"}
for tn in $TASKS; do
  for v in $VALS; do
    out=gpurun_out/envab_${tn%%:*}_${VAR}_$v.log
    env "$VAR=$v" timeout -k 10 150 python3 bench.py --task "${tn%%:*}" --num-envs "${tn##*:}" \
      --steps ${STEPS:-100} --warmup 20 --no-cpu-baseline > "$out" 2>&1
    grep '^{' "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('${tn%%:*} $VAR=$v', round(d['value']), 'env-steps/s', round(d['ms_per_step'],3), 'ms/step')"
  done
done
