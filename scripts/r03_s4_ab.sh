#!/bin/bash
# Round 3, session 4: register-row line search A/B (lib), then the per-world capacity A/B.
set -e
mkdir -p gpurun_out
LIBS="libmjx355.so libmjx355_ls.so" TASKS="Mjlab-Velocity-Flat-Unitree-G1:4096 Mjlab-Jump-Hfield-Unitree-G1:16384" \
  bash scripts/lib_ab.sh 2>&1 | tee gpurun_out/s4_libab.txt
ROUNDS=1 RUNS="Mjlab-Velocity-Flat-Unitree-G1:4096:default/48,208/48,224 Mjlab-Tracking-Flat-Unitree-G1:4096:default/48,208/48,224 Mjlab-Velocity-Flat-Unitree-Go1:8192:default/48,216 Mjlab-Jump-Hfield-Unitree-G1:16384:default/48,224" \
  bash scripts/wcap_ab.sh 2>&1 | tee gpurun_out/s4_wcap.txt
