"""Turn the rocprofv3 CSVs of scripts/profile_round.sh into committed profile summaries.

usage: python scripts/profile_summary.py <gpurun_out/prof_tag> <round tag, e.g. r01> <task> <num_envs> <nv>

Writes profiles/<round>_<tag>_kernel_stats.csv (the rocprofv3 --stats file as is),
profiles/<round>_<tag>_hbm_traffic.json (per-dispatch medians of FETCH_SIZE x2 and
WRITE_SIZE per step phase, summed over one Simulation.step) and
profiles/<round>_<tag>_pmc_sq.txt (SQ counters per launch and per world-substep).
"""

import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _find(d, pat):
  hits = sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))
  if not hits:
    raise FileNotFoundError(f"{pat} under {d}")
  return hits[0]


def _phase(name):
  if "step_phase" not in name:
    return None
  return name.split("(")[0].replace("void ", "").strip()


def counters(path):
  """{kernel: {counter: [per-dispatch values]}} from a counter_collection.csv."""
  out = {}
  with open(path) as fh:
    for row in csv.DictReader(fh):
      k = _phase(row["Kernel_Name"])
      if k is None:
        continue
      d = out.setdefault(k, {}).setdefault(row["Counter_Name"], {})
      key = row.get("Dispatch_Id") or row.get("Correlation_Id")
      d[key] = d.get(key, 0.0) + float(row["Counter_Value"])
  return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in out.items()}


def main():
  src, rnd, task, nenv, nv = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
  tag = os.path.basename(src.rstrip("/")).replace("prof_", "")
  prof = os.path.join(ROOT, "profiles")
  shutil.copy(_find(os.path.join(src, "kt"), "*kernel_stats.csv"),
              os.path.join(prof, f"{rnd}_{tag}_kernel_stats.csv"))
  fetch = counters(_find(os.path.join(src, "fetch"), "*counter_collection.csv"))
  write = counters(_find(os.path.join(src, "write"), "*counter_collection.csv"))
  # per Simulation.step: every dispatch of each phase summed, over the number of phase-A
  # dispatches (the Newton phase launches once per work class)
  def per_step(c, name):
    nstep = max(len(v[name]) for k, v in c.items() if ", 0," in k)
    return {k: sum(v[name]) / nstep for k, v in c.items()}
  f_kb = per_step(fetch, "FETCH_SIZE")
  w_kb = per_step(write, "WRITE_SIZE")
  total = sum(2 * 1024 * v for v in f_kb.values()) + sum(1024 * v for v in w_kb.values())
  traffic = {
    "task": task, "num_envs": nenv, "nv": nv,
    "unit": "bytes per Simulation.step (phases A+B+C)",
    "fetch_size_kb_raw": f_kb, "write_size_kb_raw": w_kb,
    "traffic_bytes_per_launch": total,
    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
              "scripts/physics_loop.py; all dispatches of a phase summed per substep; FETCH_SIZE doubled per the gfx950 "
              "correction (MI355X_MICROARCH.md HBM section); includes the phase hand-off scratch.",
  }
  with open(os.path.join(prof, f"{rnd}_{tag}_hbm_traffic.json"), "w") as fh:
    json.dump(traffic, fh, indent=1)
  sq = counters(_find(os.path.join(src, "sq"), "*counter_collection.csv"))
  lines = [f"# SQ counters per step phase ({task}, {nenv} worlds): all dispatches of the phase",
           "# summed per substep, and per world-substep; rocprofv3 --pmc (one pass) over",
           "# scripts/physics_loop.py.  *_CYCLES / SQ_WAIT_* count quad-cycles (MI355X_MICROARCH.md)."]
  nstep = max(len(next(iter(v.values()))) for k, v in sq.items() if ", 0," in k)
  for k in sorted(sq):
    lines.append(f"[{k}]  dispatches per substep {len(next(iter(sq[k].values()))) / nstep:.0f}")
    tot = {c: sum(v) / nstep for c, v in sq[k].items()}
    for c in sorted(tot):
      lines.append(f"  {c:20s} {tot[c]:16.0f}   per world {tot[c] / nenv:12.1f}")
    if tot.get("SQ_WAVE_CYCLES"):
      lines.append(f"  wait_any/wave_cycles = {tot.get('SQ_WAIT_ANY', 0) / tot['SQ_WAVE_CYCLES']:.3f}")
  with open(os.path.join(prof, f"{rnd}_{tag}_pmc_sq.txt"), "w") as fh:
    fh.write("\n".join(lines) + "\n")
  print(json.dumps(traffic, indent=1))
  print("\n".join(lines))


if __name__ == "__main__":
  main()
