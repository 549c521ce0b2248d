"""Median per-substep phase timings from a rocprofv3 kernel trace of the bench:
phase A, the Newton span (all row classes), phase C and the whole substep."""
import csv, glob, statistics, sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
seq = []
for r in rows:
  n = r["Kernel_Name"]
  if "step_phase" in n:
    seq.append((n.split("<")[1].split(",")[1].strip(), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
A, B, C, T, G = [], [], [], [], []
i = 0
while i < len(seq):
  if seq[i][0] != "0":
    i += 1
    continue
  a, j, bs = seq[i], i + 1, []
  while j < len(seq) and seq[j][0] == "1":
    bs.append(seq[j]); j += 1
  if j < len(seq) and seq[j][0] == "2" and bs:
    c = seq[j]
    A.append(a[2] - a[1]); C.append(c[2] - c[1])
    B.append(max(b[2] for b in bs) - min(b[1] for b in bs)); T.append(c[2] - a[1])
    G.append((min(b[1] for b in bs) - a[2]) + (c[1] - max(b[2] for b in bs)))
  i = j
# skip the first quarter (warm-up, resets)
k = len(T) // 4
med = lambda v: statistics.median(v[k:]) / 1e3
print(f"{sys.argv[1]}: n={len(T)-k} A {med(A):.1f}  B-span {med(B):.1f}  C {med(C):.1f}  gaps {med(G):.1f}  substep {med(T):.1f} us")
