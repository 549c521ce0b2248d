"""Sum SQ counters per step phase over every dispatch, per world-substep (phase A
dispatches count the substeps)."""
import sys
sys.path.insert(0, __import__("os").path.dirname(__file__))
from profile_summary import _find, counters

src, nenv = sys.argv[1], int(sys.argv[2])
c = counters(_find(src, "*counter_collection.csv"))
nsub = None
for k in sorted(c):
  if ", 0," in k:
    nsub = len(next(iter(c[k].values())))
for k in sorted(c):
  print(k, "dispatches", len(next(iter(c[k].values()))))
  for name, v in sorted(c[k].items()):
    print(f"   {name:22s} per world-substep {sum(v) / nsub / nenv:10.1f}")
