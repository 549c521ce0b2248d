set -e
for p in 0 400 3400 7300 12800; do
  MJX355_LDS_PAD0=$p timeout -k 10 60 python scripts/time_step.py g1_velocity 4096
done
for p in 0 400 3400 7300; do
  MJX355_LDS_PAD1=$p timeout -k 10 60 python scripts/time_step.py g1_velocity 4096
done
