"""Per-substep span of the Newton launches (row classes run concurrently) from a rocprofv3
kernel trace: prints each class's mean duration and the mean wall span of phase B."""
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + "/**/pt_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
spans, groups, cur = [], defaultdict(list), []
for r in rows:
  n = r["Kernel_Name"]
  if "step_phase" not in n:
    continue
  ph = n.split("step_phase<")[1].split(">")[0].split(",")[1].strip()
  s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
  if ph == "1":
    cur.append((s, e))
  elif cur:
    spans.append((min(a for a, _ in cur), max(b for _, b in cur)))
    for i, (a, b) in enumerate(sorted(cur)):
      groups[i].append(b - a)
    cur = []
for i in sorted(groups):
  print(f"  B launch #{i} (by start): mean {sum(groups[i]) / len(groups[i]) / 1e3:7.1f} us")
print(f"  B span: mean {sum(b - a for a, b in spans) / len(spans) / 1e3:7.1f} us over {len(spans)} substeps")
