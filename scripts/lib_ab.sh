#!/bin/bash
# A/B of engine library builds on bench.py lines: LIBS="libmjx355_base.so libmjx355.so"
# TASKS="task:num_envs ...", each bench under its own time limit, rounds interleaved so
# box drift hits every build alike.
set -e
TASKS=${TASKS:-"Mjlab-Velocity-Flat-Unitree-G1:4096"}
LIBS=${LIBS:-"libmjx355_base.so libmjx355.so"}
for round in ${ROUNDS:-1 2}; do
  for tn in $TASKS; do
    for lib in $LIBS; do
      out=gpurun_out/libab_${tn%%:*}_${lib%.so}_$round.log
      MJX355_LIB=$PWD/mjlab-1_amd/mjlab_amd/$lib timeout -k 10 150 python3 bench.py --task "${tn%%:*}" \
        --num-envs "${tn##*:}" --steps ${STEPS:-100} --warmup 20 --no-cpu-baseline > "$out" 2>&1
      grep '^{' "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('${tn%%:*} $lib r$round', round(d['value']), 'env-steps/s', round(d['ms_per_step'],3), 'ms/step')"
    done
  done
done
