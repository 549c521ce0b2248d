"""Robot descriptions (`mjlab_amd/assets/robots/*.json`, the parsed MJCF) and the compiled
task scenes (`mjlab_amd/assets/*.npz`) from the reference robot MJCF.

Runs in the build container only (the reference tree is not on the GPU box).  The
output is numeric model data (like a compiled .mjb), not reference source.
"""

import os
import sys

REF = os.environ.get("MJLAB_REFERENCE", "/root/reference/src/mjlab/asset_zoo/robots")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mjlab-1_amd"))

from mjlab_amd import scenes  # noqa: E402


ROBOTS = {"unitree_g1": "unitree_g1/xmls/g1.xml", "unitree_go1": "unitree_go1/xmls/go1.xml"}


def main():
  import json
  from mjlab_amd import asset_zoo
  from mjlab_amd.compiler.mjcf import parse_mjcf, xmodel_to_dict
  os.makedirs(scenes.ASSET_DIR, exist_ok=True)
  # robot descriptions as parsed MJCF data (the robot EntityCfg's spec_fn reads them; the
  # env scenes are assembled from them at env construction)
  os.makedirs(asset_zoo.ROBOT_DIR, exist_ok=True)
  for name, rel in ROBOTS.items():
    text = json.dumps(xmodel_to_dict(parse_mjcf(os.path.join(REF, rel))), indent=0, sort_keys=True)
    out = os.path.join(asset_zoo.ROBOT_DIR, f"{name}.json")
    if not os.path.exists(out) or open(out).read() != text:
      with open(out, "w") as fh:
        fh.write(text)
    print(f"{name}: -> {out}")
  # compiled task scenes (regression targets of the SceneCfg assembly; test fixtures)
  for name, (rel, fn) in scenes.SCENE_BUILDERS.items():
    m = fn(os.path.join(REF, rel))
    out = os.path.join(scenes.ASSET_DIR, f"{name}.npz")
    scenes.save_model(m, out)
    print(f"{name}: nq={m.nq} nv={m.nv} nu={m.nu} nbody={m.nbody} ngeom={m.ngeom} "
          f"npair={m.npair} nsensordata={m.nsensordata} -> {out}")


if __name__ == "__main__":
  main()
