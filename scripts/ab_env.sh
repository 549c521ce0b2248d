#!/bin/bash
# A/B of one library under two environment settings (ENV_A / ENV_B), kernel-traced bench.
set -e
export TMPDIR=/tmp
TASK=${TASK:-Mjlab-Velocity-Flat-Unitree-G1}
NENV=${NENV:-4096}
for tag in A B; do
  var=ENV_$tag; out=gpurun_out/abenv_$tag; rm -rf "$out"
  env ${!var} timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d "$out" -o ab -- \
    python3 bench.py --task "$TASK" --num-envs "$NENV" --steps 60 --warmup 20 --no-cpu-baseline > "$out.log" 2>&1
  echo "${!var}"; python3 scripts/phase_span.py "$out"
  grep '^{' "$out.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   bench', round(d['value']), 'env-steps/s', round(d['ms_per_step'],3), 'ms/step')"
done
