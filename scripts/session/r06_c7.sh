#!/bin/bash
# round 6: the J-in-global heavy Newton (MJX355_NEWTON_JG): bit equality, then A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "Mjlab-Velocity-Flat-Unitree-G1 4096 30" "Mjlab-Jump-Hfield-Unitree-G1 16384 20"; do
  set -- $spec
  for v in 0 1; do
    MJX355_NEWTON_JG=$v timeout -k 10 240 python3 scripts/step_digest.py $1 $2 $3 gpurun_out/r06c7_dig_$1_$v.npz > gpurun_out/r06c7_dig_$1_$v.log 2>&1 || exit $?
  done
  python3 scripts/step_digest.py --compare gpurun_out/r06c7_dig_$1_0.npz gpurun_out/r06c7_dig_$1_1.npz; echo "$1 JG equality rc=$?"
  rm -f gpurun_out/r06c7_dig_$1_*.npz
done
for round in 1 2; do
  VAR=MJX355_NEWTON_JG VALS="0 1" TASKS="Mjlab-Velocity-Flat-Unitree-G1:4096 Mjlab-Jump-Hfield-Unitree-G1:16384 Mjlab-Tracking-Flat-Unitree-G1:4096" STEPS=100 timeout -k 10 600 bash scripts/env_ab.sh || exit $?
done
