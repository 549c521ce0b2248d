#!/bin/bash
# scripts/chol_bench.hip on the box: factor + solve latency of the register-row forms.
set -e
mkdir -p gpurun_out/cb
python scripts/chol_bench_gen.py gpurun_out/cb > gpurun_out/cb/gen.txt
for nw in 1 256 2560; do
  for mode in 0 6 3 7 5 4; do
    timeout -k 5 30 ./scripts/chol_bench gpurun_out/cb/H_nat.bin gpurun_out/cb/b_nat.bin $mode $nw 200
  done
done
