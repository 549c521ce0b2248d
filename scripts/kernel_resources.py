"""Register / scratch / occupancy of every step kernel of the given specs.inc entries, from the
compiler's own accounting (hipcc -Rpass-analysis=kernel-resource-usage on spec.hip; same flags as
csrc/Makefile).  usage: kernel_resources.py <spec id> ... > profiles/<round>_kernel_resources.txt"""
import os
import re
import subprocess
import sys
import tempfile

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mjlab-1_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-function",
         "-fno-hip-fp32-correctly-rounded-divide-sqrt", "-DMJX_HDR_HASH=0x1ULL"]
names = {}
for line in open(os.path.join(CSRC, "specs.inc")):
  m = re.match(r"MJX_SPEC\((\d+), (\w+),.*, (\d+), (\d+)\)$", line.strip())
  if m:
    names[m.group(1)] = f"{m.group(2)} {m.group(3)}/{m.group(4)}"
print(f"{'spec':28s} {'kernel':34s} {'VGPR':>5s} {'AGPR':>5s} {'scratch B/lane':>14s} {'waves/SIMD':>10s}")
for sid in sys.argv[1:]:
  with tempfile.TemporaryDirectory() as tmp:
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, f"-DMJX_SPEC_ID={sid}", "-c", "-o",
                        os.path.join(tmp, "s.o"), "spec.hip", "-Rpass-analysis=kernel-resource-usage"],
                       cwd=CSRC, capture_output=True, text=True)
  cur, rows = None, {}
  for line in r.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
      cur = m.group(1)
      rows[cur] = {}
      continue
    for key, pat in (("v", r"VGPRs: (\d+)"), ("a", r"AGPRs: (\d+)"), ("s", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("o", r"Occupancy \[waves/SIMD\]: (\d+)")):
      m = re.search(pat, line)
      if m and cur:
        rows[cur][key] = m.group(1)
  for k, v in rows.items():
    dm = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
    dm = dm.replace("mjx::", "").split("(")[0]
    print(f"{sid + ' ' + names.get(sid, ''):28s} {dm:34s} {v.get('v', '-'):>5s} {v.get('a', '-'):>5s} "
          f"{v.get('s', '-'):>14s} {v.get('o', '-'):>10s}")
