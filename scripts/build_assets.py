"""Compile the task scenes from the reference robot MJCF into `mjlab_amd/assets/*.npz`.

Runs in the build container only (the reference tree is not on the GPU box).  The
output is numeric model data (like a compiled .mjb), not reference source.
"""

import os
import sys

REF = os.environ.get("MJLAB_REFERENCE", "/root/reference/src/mjlab/asset_zoo/robots")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mjlab-1_amd"))

from mjlab_amd import scenes  # noqa: E402


def main():
  os.makedirs(scenes.ASSET_DIR, exist_ok=True)
  for name, (rel, fn) in scenes.SCENE_BUILDERS.items():
    m = fn(os.path.join(REF, rel))
    out = os.path.join(scenes.ASSET_DIR, f"{name}.npz")
    scenes.save_model(m, out)
    print(f"{name}: nq={m.nq} nv={m.nv} nu={m.nu} nbody={m.nbody} ngeom={m.ngeom} "
          f"npair={m.npair} nsensordata={m.nsensordata} -> {out}")


if __name__ == "__main__":
  main()
