# Per-phase kernel durations vs world count (latency vs throughput regime of each phase).
set -e
export TMPDIR=/tmp
for n in 256 1024 2048 4096 8192; do
  timeout -k 10 90 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/ns_$n -o ns -- \
    python3 scripts/time_step.py g1_velocity $n > gpurun_out/ns_$n.log 2>&1
done
