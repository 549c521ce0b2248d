#!/bin/bash
# Iteration loop on the GPU box: GPU tests, substep timing and a short bench, each step
# under its own time limit; stops at the first failure.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/chk_pytest.log 2>&1 || { tail -30 gpurun_out/chk_pytest.log; exit 1; }
tail -2 gpurun_out/chk_pytest.log
timeout -k 10 60 python scripts/time_step.py g1_velocity 4096 2>&1 | grep ms/sub
timeout -k 10 120 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/chk_bench.log 2>&1
grep '^{' gpurun_out/chk_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', round(d['value']), 'env-steps/s', round(d['ms_per_step'],3), 'ms/step', 'launch_ms', round(d['roofline']['launch_ms'],4))"
