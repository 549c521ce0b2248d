#!/bin/bash
# round 6: Go1 8,192 env-step timeline; per-stage cycles (MJX_STAMPS build) of jump hfield and G1
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_go1t
timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d gpurun_out/prof_go1t/kt -o kt -- python3 bench.py \
  --task Mjlab-Velocity-Flat-Unitree-Go1 --num-envs 8192 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_go1t/bench_prof.log 2>&1 || exit $?
python3 scripts/step_timeline.py gpurun_out/prof_go1t/kt 2 > gpurun_out/r06c32_go1_timeline.txt
cat gpurun_out/r06c32_go1_timeline.txt
NENV=16384 timeout -k 10 300 python3 scripts/stage_profile.py Mjlab-Jump-Hfield-Unitree-G1 > gpurun_out/r06c32_hf_stages.txt 2>&1 || { tail -5 gpurun_out/r06c32_hf_stages.txt; exit 1; }
cat gpurun_out/r06c32_hf_stages.txt
NENV=4096 timeout -k 10 300 python3 scripts/stage_profile.py Mjlab-Velocity-Flat-Unitree-G1 > gpurun_out/r06c32_g1_stages.txt 2>&1 || { tail -5 gpurun_out/r06c32_g1_stages.txt; exit 1; }
cat gpurun_out/r06c32_g1_stages.txt
