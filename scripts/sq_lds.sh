#!/bin/bash
# LDS pipe counters of the step phases (bank conflicts vs LDS-array busy cycles), one pass
set -e
export TMPDIR=/tmp
TASK=${TASK:-Mjlab-Velocity-Flat-Unitree-G1}
NENV=${NENV:-4096}
out=gpurun_out/sq_lds
rm -rf "$out"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS \
  SQ_ACTIVE_INST_LDS SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES \
  -f csv -d "$out" -o sq -- python3 scripts/physics_loop.py "$TASK" "$NENV" > "$out.log" 2>&1
python3 scripts/sq_sum.py "$out" "$NENV"
