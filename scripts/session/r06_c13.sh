#!/bin/bash
# phase A at most 168 VGPRs (terrain specs 182-189 -> 3 waves / SIMD): A/B against the previous build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS="1 2" STEPS=60 LIBS="libmjx355_base.so libmjx355.so" \
TASKS="Mjlab-Jump-Hfield-Unitree-G1:16384 Mjlab-Velocity-Rough-Unitree-G1:4096 Mjlab-Velocity-Rough-Unitree-Go1:8192 Mjlab-Velocity-Flat-Unitree-G1:4096" \
  timeout -k 10 1000 bash scripts/lib_ab.sh
