#!/bin/bash
# Per-world capacity A/B on bench lines (MJX355_WORLD_CAPACITY="contacts,rows"; "default" =
# sim.world_capacity's rule), with the overflow events of the timed steps.  Rounds interleave
# so box drift hits every capacity alike.  RUNS="task:num_envs:cap1/cap2/..."
set -e -o pipefail
mkdir -p gpurun_out
RUNS=${RUNS:-"Mjlab-Velocity-Flat-Unitree-G1:4096:default/48,208/48,224"}
for round in ${ROUNDS:-1 2}; do
  for run in $RUNS; do
    IFS=: read -r task n caps <<< "$run"
    for cap in ${caps//\// }; do
      if [ "$cap" = default ]; then unset MJX355_WORLD_CAPACITY; else export MJX355_WORLD_CAPACITY=$cap; fi
      out=gpurun_out/wcap_${task}_${cap/,/_}_$round.log
      timeout -k 10 150 python3 bench.py --task "$task" --num-envs "$n" --steps ${STEPS:-100} \
        --warmup 20 --no-cpu-baseline --allow-overflow > "$out" 2>&1
      grep '^{' "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); o=d['overflow']; print('$task cap $cap r$round', round(d['value']), round(d['ms_per_step'],3), 'ovf c/r', o['contact_overflow_events'], o['row_overflow_events'], 'max c/r', o['max_contacts_seen'], o['max_rows_seen'])"
    done
  done
done
