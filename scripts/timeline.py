"""Print the kernel timeline (start/end in us relative to the first kernel shown) of a few
consecutive env steps from a rocprofv3 kernel trace: which launches overlap, and the gaps.
usage: timeline.py <trace dir> [first kernel index] [count]"""
import csv, glob, sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
i0 = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows) // 2
cnt = int(sys.argv[3]) if len(sys.argv) > 3 else 60
t0 = int(rows[i0]["Start_Timestamp"])
prev_end = t0
for r in rows[i0:i0 + cnt]:
  s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
  name = r["Kernel_Name"]
  if "step_phase" in name:
    name = "phase" + name.split("<")[1].split(",")[1].strip()
  else:
    name = name.split("(")[0].replace("void ", "")[:48]
  gap = (s - prev_end) / 1e3
  print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  gap {gap:7.1f}  {name}")
  prev_end = max(prev_end, e)
