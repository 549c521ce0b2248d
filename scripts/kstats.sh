#!/bin/bash
# Kernel-trace stats of a short bench run: the top kernels by total time (TASK, NENV).
set -e
TASK=${TASK:-Mjlab-Velocity-Flat-Unitree-G1}; NENV=${NENV:-4096}; OUT=gpurun_out/ks_${TAG:-x}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o ks -- \
  python3 bench.py --task "$TASK" --num-envs "$NENV" --steps 50 --warmup 20 --no-cpu-baseline > "$OUT/bench.log" 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/ks_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
  print(f"{r['Name'][:60]:60s} calls {r['Calls']:>6} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
