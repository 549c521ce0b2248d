"""Per-substep span of each row-class chain from a rocprofv3 kernel trace (rocpd SQLite or
kernel_trace.csv): for every classify_kernel launch, the time from its start to the end of
the last kernel of each queue before the next classify, plus the launches on that queue.
usage: chain_spans.py <trace dir> [max substeps]"""
import collections
import glob
import sqlite3
import statistics
import sys


def load(d):
  dbs = glob.glob(d + "/**/*.db", recursive=True)
  if dbs:
    c = sqlite3.connect(dbs[0])
    return [(n, s, e, q) for n, s, e, q in c.execute("select name,start,end,queue_id from kernels order by start")]
  import csv
  f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
  rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
  return [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "0")) for r in rows]


def short(n):
  if "step_phase" in n:
    return "P" + n.split("<")[1].split(",")[1].strip()
  if "step_newton_lat" in n:
    return "BL"
  return n.split("(")[0].replace("void ", "").split("::")[-1][:16]


rows = load(sys.argv[1])
cls = [i for i, r in enumerate(rows) if "classify_kernel" in r[0]]
maxn = int(sys.argv[2]) if len(sys.argv) > 2 else 10 ** 9
cls = cls[len(cls) // 4:][:maxn]  # skip warmup
spans = collections.defaultdict(list)
seqs = collections.Counter()
total = []
for a, b in zip(cls, cls[1:]):
  t0 = rows[a][1]
  per_q = collections.defaultdict(list)
  for r in rows[a + 1:b]:
    per_q[r[3]].append(r)
  if any("k_post" in r[0] for r in rows[a:b]):
    continue  # the env step's manager tail is not a substep
  for q, rs in per_q.items():
    key = " ".join(short(r[0]) for r in rs)
    seqs[(q, key)] += 1
    spans[(q, key)].append((rs[-1][2] - t0) / 1e3)
  total.append((rows[b][1] - t0) / 1e3)
print(f"substeps {len(total)}: classify-to-classify median {statistics.median(total):.1f} us")
for (q, key), v in sorted(spans.items(), key=lambda kv: -len(kv[1])):
  if len(v) < 3:
    continue
  print(f"  queue {q} [{key}] x{len(v)}: end median {statistics.median(v):.1f} us, p90 "
        f"{sorted(v)[int(0.9 * len(v))]:.1f}")
# per-kernel durations by queue
dur = collections.defaultdict(list)
for a, b in zip(cls, cls[1:]):
  for r in rows[a:b]:
    dur[(r[3], short(r[0]))].append((r[2] - r[1]) / 1e3)
for (q, n), v in sorted(dur.items()):
  if len(v) >= 3:
    print(f"  queue {q} {n}: median {statistics.median(v):.1f} us x{len(v)}")
