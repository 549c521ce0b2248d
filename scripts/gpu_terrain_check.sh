set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/chk_pytest.log 2>&1 || { tail -40 gpurun_out/chk_pytest.log; exit 1; }
tail -3 gpurun_out/chk_pytest.log
for s in g1_velocity g1_jump_hfield g1_velocity_rough; do timeout -k 10 90 python scripts/time_step.py $s 4096 2>&1 | grep ms/sub; done
