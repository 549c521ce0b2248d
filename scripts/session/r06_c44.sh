#!/bin/bash
# round 6 final build (heavy cap, in-line re-solve grid 1): smoke, full GPU suite with parity statistics,
# the driver's command twice
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06c44_stats
T="--timeout 300 --timeout-method thread"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06c44_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r06c44_smoke.log; [ $rc -eq 0 ] || exit $rc
MJX_PARITY_STATS=gpurun_out/r06c44_stats timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf $T > gpurun_out/r06c44_gpu.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed|^E  " gpurun_out/r06c44_gpu.log | tail -12 | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1200 bash scripts/bench_configs.sh > gpurun_out/r06c44_bench.txt 2>&1
rc=$?; cat gpurun_out/r06c44_bench.txt | grep -v "^$" | tail -8; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06c44_driver$i.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c44_driver$i.log | tail -1 > gpurun_out/r06c44_driver$i.json
  python3 -c "import json; d=json.load(open('gpurun_out/r06c44_driver$i.json')); print('driver', round(d['value']), d['ms_per_step'], d['roofline'], d['cpu_baseline'])"
done
NO_BENCH=1 ROUND=r06 PROF_SPECS="g1 Mjlab-Velocity-Flat-Unitree-G1 4096 35;go1 Mjlab-Velocity-Flat-Unitree-Go1 8192 18;jump_hfield Mjlab-Jump-Hfield-Unitree-G1 16384 35" timeout -k 10 900 bash scripts/round_final.sh > gpurun_out/r06c44_final.log 2>&1
rc=$?; tail -2 gpurun_out/r06c44_final.log; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/prof_g1t2
timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d gpurun_out/prof_g1t2/kt -o kt -- python3 bench.py \
  --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_g1t2/bench_prof.log 2>&1 || exit $?
python3 scripts/step_timeline.py gpurun_out/prof_g1t2/kt 2 > gpurun_out/r06c44_g1_timeline.txt
rm -rf gpurun_out/prof_g1t2
mkdir -p gpurun_out/prof_go1t2
timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d gpurun_out/prof_go1t2/kt -o kt -- python3 bench.py --task Mjlab-Velocity-Flat-Unitree-Go1 --num-envs 8192 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_go1t2/bench_prof.log 2>&1 || exit $?
python3 scripts/step_timeline.py gpurun_out/prof_go1t2/kt 2 > gpurun_out/r06c44_go1_timeline.txt
rm -rf gpurun_out/prof_go1t2
