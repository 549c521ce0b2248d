#!/bin/bash
# LDS / issue counters of the captured G1 env step (two SQ passes), summarised per world.
set -e
export TMPDIR=/tmp
TAG=g1lds SQ="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_INSTS_LDS_STORE_BANDWIDTH SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
  SQ2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES" \
  bash scripts/profile_round.sh > gpurun_out/lds_prof.txt 2>&1
python3 scripts/profile_bench.py gpurun_out/prof_g1lds r03l Mjlab-Velocity-Flat-Unitree-G1 4096 35 20 >> gpurun_out/lds_prof.txt 2>&1
mkdir -p gpurun_out/profiles_new && cp profiles/r03l_g1lds_pmc_sq.txt gpurun_out/profiles_new/
rm -rf gpurun_out/prof_g1lds
