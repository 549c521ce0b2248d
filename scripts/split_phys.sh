#!/bin/bash
# Eager physics-mode A/B of the batch split (no graph capture): G1 4096.
set -e
for sp in ${SPLITS:-1 2}; do
  out=gpurun_out/split_phys_$sp.log
  MJX355_SPLIT=$sp timeout -k 10 150 python3 bench.py --mode physics --steps 100 --warmup 20 --no-cpu-baseline > "$out" 2>&1
  grep '^{' "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('physics split $sp', round(d['value']), 'env-steps/s', round(d['ms_per_step'],3), 'ms/step')"
done
