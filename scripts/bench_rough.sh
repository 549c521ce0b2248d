set -e
mkdir -p gpurun_out
for t in "Mjlab-Velocity-Rough-Unitree-G1 4096" "Mjlab-Velocity-Rough-Unitree-Go1 8192" "Mjlab-Velocity-Flat-Unitree-G1 4096"; do
  set -- $t
  timeout -k 10 300 python bench.py --task $1 --num-envs $2 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_$1.log 2>&1
  grep '^{' gpurun_out/bench_$1.log | tail -1 > gpurun_out/bench_$1.json
  python3 -c "import json; d=json.load(open('gpurun_out/bench_$1.json')); print('$1', round(d['value']), round(d['ms_per_step'],3))"
done
