#!/bin/bash
# Phase-A residency probe: unused LDS padding per world (MJX355_LDS_PAD0 bytes) lowers the
# resident worlds per CU; per-phase medians of a kernel-traced short bench for each setting.
set -e
export TMPDIR=/tmp
for pad in ${PADS:-0 3000 6000}; do
  out=gpurun_out/pad_$pad; rm -rf "$out"
  MJX355_LDS_PAD0=$pad timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d "$out" -o cs -- \
    python3 bench.py --steps 60 --warmup 20 --no-cpu-baseline > "$out.log" 2>&1
  echo "pad $pad"; python3 scripts/phase_span.py "$out"
done
