#!/bin/bash
# Newton row-class capacities (MJX355_ROW_CLASSES = row caps, "" = one full-carve launch) on
# the bench workload: per-phase medians of a kernel-traced short bench for each setting.
set -e
export TMPDIR=/tmp
TASK=${TASK:-Mjlab-Velocity-Flat-Unitree-G1}
NENV=${NENV:-4096}
for cfg in ${CFGS:-"44,84" "44" "60" "84" "none"}; do
  out=gpurun_out/cs_${cfg/,/_}
  rm -rf "$out"
  v=$cfg; [ "$cfg" = none ] && v=""
  if [ "$cfg" = default ]; then unset MJX355_ROW_CLASSES; else export MJX355_ROW_CLASSES=$v; fi
  timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d "$out" -o cs -- \
    python3 bench.py --task "$TASK" --num-envs "$NENV" --steps 60 --warmup 20 --no-cpu-baseline > "$out.log" 2>&1
  echo "row classes: $cfg"
  python3 scripts/phase_span.py "$out"
done
