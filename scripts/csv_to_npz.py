"""CLI of `src/mjlab/scripts/csv_to_npz.py` on the MI355X engine: a retargeted G1 clip (CSV
rows: root position, root quaternion xyzw, 29 joint positions) -> tracking motion npz.

  python scripts/csv_to_npz.py --input-file clip.csv --output-file motion.npz \\
      [--input-fps 30] [--output-fps 50] [--line-range 1 300] [--device cuda:0]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mjlab-1_amd"))


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--input-file", required=True)
  ap.add_argument("--output-file", required=True)
  ap.add_argument("--input-fps", type=float, default=30.0)
  ap.add_argument("--output-fps", type=float, default=50.0)
  ap.add_argument("--line-range", type=int, nargs=2, default=None)
  ap.add_argument("--device", default="cuda:0")
  a = ap.parse_args()
  from mjlab_amd.motion_csv import csv_to_npz
  out = csv_to_npz(a.input_file, a.output_file, a.input_fps, a.output_fps, a.device,
                   tuple(a.line_range) if a.line_range else None)
  print(f"wrote {a.output_file}: {out['joint_pos'].shape[0]} frames at {a.output_fps} fps")


if __name__ == "__main__":
  main()
