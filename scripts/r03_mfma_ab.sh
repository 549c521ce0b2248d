#!/bin/bash
# A/B of the Newton J^T D J on MFMA (libmjx355_mfma.so, -DMJX_JTDJ_MFMA=1) against the VALU
# register tiles (libmjx355.so): parity of the MFMA build, interleaved bench rounds, and
# the SQ counters (VALU / MFMA instructions, MFMA busy) of both builds' timed regions.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T="--timeout 300 --timeout-method thread"
MJX355_LIB=$PWD/mjlab-1_amd/mjlab_amd/libmjx355_mfma.so timeout -k 10 300 python -u -m pytest \
  tests/test_gpu_parity.py tests/test_gpu_rowclass.py -x -q $T > gpurun_out/r03_mfma_parity.log 2>&1 \
  || { tail -30 gpurun_out/r03_mfma_parity.log; exit 1; }
tail -2 gpurun_out/r03_mfma_parity.log
LIBS="libmjx355.so libmjx355_mfma.so" ROUNDS="1 2" TASKS="Mjlab-Velocity-Flat-Unitree-G1:4096 Mjlab-Velocity-Flat-Unitree-Go1:8192" \
  bash scripts/lib_ab.sh
B="bench.py --steps 20 --warmup 5 --launch-reps 4 --no-cpu-baseline --allow-overflow"
for lib in libmjx355.so libmjx355_mfma.so; do
  MJX355_LIB=$PWD/mjlab-1_amd/mjlab_amd/$lib timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU \
    SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_WAIT_ANY SQ_INSTS_MFMA -f csv -d gpurun_out/mfma_sq_${lib%.so} -o sq -- python3 $B > gpurun_out/mfma_sq_${lib%.so}.log 2>&1 \
    || { tail -5 gpurun_out/mfma_sq_${lib%.so}.log; exit 1; }
done
echo done
