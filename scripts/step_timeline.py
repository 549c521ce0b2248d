"""Timeline of one env step from a rocprofv3 kernel trace of the bench (graph replay):
every kernel between two k_action launches with its start offset, duration and the gap
before it; medians over the later steps."""
import csv, glob, statistics, sys
from collections import defaultdict

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: (n.split("(")[0].replace("void ", "").replace("mjx::", "").replace("mjxt::", "")[:40])
steps, cur = [], None
for r in rows:
  n = short(r["Kernel_Name"])
  if n.startswith("k_action") or n.startswith("mjtr::k_action"):
    if cur:
      steps.append(cur)
    cur = []
  if cur is not None:
    cur.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
steps = steps[len(steps) // 4:]
agg = defaultdict(list)
tot = []
for s in steps:
  t0 = s[0][1]
  prev_end = t0
  for i, (n, a, b) in enumerate(s):
    agg[(i, n)].append((a - t0, b - a, a - prev_end))
    prev_end = max(prev_end, b)
  tot.append(prev_end - t0)
print(f"{len(steps)} steps, median span {statistics.median(tot)/1e3:.1f} us")
for (i, n), v in sorted(agg.items()):
  if len(v) < len(steps) // 2:
    continue
  m = lambda k: statistics.median(x[k] for x in v) / 1e3
  print(f"{i:3d} {n:40s} start {m(0):8.1f}  dur {m(1):7.1f}  gap {m(2):6.1f}")
