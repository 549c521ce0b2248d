#!/bin/bash
# Quick per-kernel timing of the default bench workload (kernel trace only), for
# iterating on the step kernels: prints the average duration of each step phase.
set -e
TASK=${TASK:-Mjlab-Velocity-Flat-Unitree-G1}
NENV=${NENV:-4096}
OUT=gpurun_out/pt_${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o pt -- \
  python3 bench.py --task "$TASK" --num-envs "$NENV" --steps 40 --warmup 10 --no-cpu-baseline \
  > "$OUT/bench.log" 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/pt_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
  n = r["Name"]
  if "step_phase" in n or "mjxt::" in n or "reset_kernel" in n:
    print(f"{float(r['AverageNs'])/1e3:9.1f} us  x{r['Calls']:>5}  {n.split('(')[0]}")
PY
grep "^{" "$OUT/bench.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', round(d['value']), 'ms/step', round(d['ms_per_step'],3), 'launch_ms', round(d['roofline']['launch_ms'],3))"
