#!/bin/bash
# Round 3, session 4: GPU suite + smoke on the v2 build (register rows across the Newton
# loop), then the default bench line, the tracking line with overflow enforced and the
# v1 / v2 library A/B.  Each step has its own limit; the first failure ends the script.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
V2=$PWD/mjlab-1_amd/mjlab_amd/libmjx355_v3.so
MJX355_LIB=$V2 timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v $T > gpurun_out/s4_gpu.log 2>&1 \
  || { tail -60 gpurun_out/s4_gpu.log; exit 1; }
tail -3 gpurun_out/s4_gpu.log
MJX355_LIB=$V2 timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s4_smoke.log 2>&1 \
  || { tail -20 gpurun_out/s4_smoke.log; exit 1; }
tail -1 gpurun_out/s4_smoke.log
timeout -k 10 300 python bench.py --task Mjlab-Tracking-Flat-Unitree-G1 --steps 100 --warmup 20 --no-cpu-baseline \
  > gpurun_out/s4_track.log 2>&1 || { tail -20 gpurun_out/s4_track.log; exit 1; }
grep '^{' gpurun_out/s4_track.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tracking', round(d['value']), d['ms_per_step'], d['overflow'], d['config']['capacity'])"
LIBS="libmjx355.so libmjx355_v2.so libmjx355_v3.so" TASKS="Mjlab-Velocity-Flat-Unitree-G1:4096 Mjlab-Jump-Hfield-Unitree-G1:16384" \
  bash scripts/lib_ab.sh 2>&1 | tee gpurun_out/s4_libab2.txt
timeout -k 10 200 python scripts/stage_profile.py > gpurun_out/s4_stages_all.txt 2>&1
