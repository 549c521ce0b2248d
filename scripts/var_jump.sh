for lib in libmjx355_base.so libmjx355.so libmjx355_base.so libmjx355.so; do
  MJX355_LIB=$PWD/mjlab-1_amd/mjlab_amd/$lib timeout -k 10 120 python bench.py --task Mjlab-Jump-Flat-Unitree-G1 --num-envs 16384 --steps 60 --warmup 20 --no-cpu-baseline 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['value']), round(d['ms_per_step'],3))"
done
