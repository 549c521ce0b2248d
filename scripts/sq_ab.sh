#!/bin/bash
# SQ instruction / issue counters of the step phases for two engine builds (LIBS), summed
# over all dispatches of each phase per substep (scripts/sq_sum.py).
set -e
export TMPDIR=/tmp
TASK=${TASK:-Mjlab-Velocity-Flat-Unitree-G1}
NENV=${NENV:-4096}
LIBS=${LIBS:-"libmjx355_base.so libmjx355.so"}
for lib in $LIBS; do
  out=gpurun_out/sq_${lib%.so}
  rm -rf "$out"
  MJX355_LIB=$PWD/mjlab-1_amd/mjlab_amd/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY \
    -f csv -d "$out" -o sq -- python3 scripts/physics_loop.py "$TASK" "$NENV" > "$out.log" 2>&1
  echo "== $lib"
  python3 scripts/sq_sum.py "$out" "$NENV"
done
