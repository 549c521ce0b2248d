#!/bin/bash
# Newton row-class capacity sweep on bench lines (MJX355_ROW_CLASSES; "default" = the rule).
set -e -o pipefail
mkdir -p gpurun_out
TASKS=${TASKS:-"Mjlab-Velocity-Flat-Unitree-G1:4096 Mjlab-Tracking-Flat-Unitree-G1:4096 Mjlab-Jump-Hfield-Unitree-G1:16384"}
for round in ${ROUNDS:-1}; do
  for tn in $TASKS; do
    for cap in ${CAPS:-default 44 52 68 76}; do
      if [ "$cap" = default ]; then unset MJX355_ROW_CLASSES; else export MJX355_ROW_CLASSES=$cap; fi
      out=gpurun_out/cap_${tn%%:*}_${cap}_$round.log
      timeout -k 10 150 python3 bench.py --task "${tn%%:*}" --num-envs "${tn##*:}" --steps ${STEPS:-100} \
        --warmup 20 --no-cpu-baseline > "$out" 2>&1 || true
      grep '^{' "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('${tn%%:*} cap $cap r$round', round(d['value']), round(d['ms_per_step'],3))"
    done
  done
done
