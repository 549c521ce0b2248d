#!/bin/bash
# round 6: JG variants (throughput form, heavy chain) -- bit equality, then A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
dig() {  # tag task n steps env...
  local tag=$1 task=$2 n=$3 st=$4; shift 4
  env "$@" timeout -k 10 240 python3 scripts/step_digest.py $task $n $st gpurun_out/r06c8_dig_$tag.npz > gpurun_out/r06c8_dig_$tag.log 2>&1 || exit $?
}
dig jh0 Mjlab-Jump-Hfield-Unitree-G1 16384 20 MJX355_NEWTON_JG=0
dig jh2 Mjlab-Jump-Hfield-Unitree-G1 16384 20 MJX355_NEWTON_JG=2
python3 scripts/step_digest.py --compare gpurun_out/r06c8_dig_jh0.npz gpurun_out/r06c8_dig_jh2.npz; echo "jh JG2 equality rc=$?"
dig g0 Mjlab-Velocity-Flat-Unitree-G1 4096 30 MJX355_NEWTON_JG=0
dig gc Mjlab-Velocity-Flat-Unitree-G1 4096 30 MJX355_NEWTON_JG=1 MJX355_CHAIN=1
python3 scripts/step_digest.py --compare gpurun_out/r06c8_dig_g0.npz gpurun_out/r06c8_dig_gc.npz; echo "g1 chain-JG equality rc=$?"
rm -f gpurun_out/r06c8_dig_*.npz
line() {  # tag task n steps env...
  local tag=$1 task=$2 n=$3 st=$4; shift 4
  env "$@" timeout -k 10 200 python3 bench.py --task $task --num-envs $n --steps $st --warmup 20 --no-cpu-baseline > gpurun_out/r06c8_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06c8_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['ms_per_step'],4))"
}
for r in 1 2; do
  line jh_jg0_$r Mjlab-Jump-Hfield-Unitree-G1 16384 60 MJX355_NEWTON_JG=0
  line jh_jg1_$r Mjlab-Jump-Hfield-Unitree-G1 16384 60 MJX355_NEWTON_JG=1
  line jh_jg2_$r Mjlab-Jump-Hfield-Unitree-G1 16384 60 MJX355_NEWTON_JG=2
  line g1_jg0_$r Mjlab-Velocity-Flat-Unitree-G1 4096 100 MJX355_NEWTON_JG=0
  line g1_chjg_$r Mjlab-Velocity-Flat-Unitree-G1 4096 100 MJX355_NEWTON_JG=1 MJX355_CHAIN=1
done
