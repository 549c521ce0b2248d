"""One env step's kernel timeline from a rocprofv3 kernel trace (kernel_trace.csv): start, end
and duration of every dispatch between two k_post launches, relative to the first, with its
queue.  usage: step_timeline.py <trace dir> [which env step from the end, default 2]"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
kp = [i for i, r in enumerate(rows) if "k_post" in r["Kernel_Name"]]
i0, i1 = kp[-back - 1], kp[-back]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1 + 1]:
  s = (int(r["Start_Timestamp"]) - t0) / 1e3
  e = (int(r["End_Timestamp"]) - t0) / 1e3
  name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1][:34]
  print(f"{s:8.1f} {e:8.1f} {e - s:7.1f} q{r.get('Queue_Id', '?')} {name}")
