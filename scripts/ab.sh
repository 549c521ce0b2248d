#!/bin/bash
# A/B of step-kernel builds on the bench workload: for each library (default: the baseline
# copy libmjx355_base.so and the current libmjx355.so) a kernel-traced short bench, then
# the per-phase medians (scripts/phase_span.py).  TASK / NENV select the workload.
set -e
export TMPDIR=/tmp
TASK=${TASK:-Mjlab-Velocity-Flat-Unitree-G1}
NENV=${NENV:-4096}
LIBS=${LIBS:-"libmjx355_base.so libmjx355.so"}
for lib in $LIBS; do
  out=gpurun_out/ab_${lib%.so}
  rm -rf "$out"
  MJX355_LIB=$PWD/mjlab-1_amd/mjlab_amd/$lib timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d "$out" -o ab -- \
    python3 bench.py --task "$TASK" --num-envs "$NENV" --steps 60 --warmup 20 --no-cpu-baseline > "$out.log" 2>&1
  python3 scripts/phase_span.py "$out"
  grep '^{' "$out.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   bench', round(d['value']), 'env-steps/s', round(d['ms_per_step'],3), 'ms/step')"
done
