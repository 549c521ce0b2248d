"""Summarise rocprofv3 passes over bench.py itself (scripts/profile_round.sh) into the
committed profile files.

usage: python scripts/profile_bench.py <gpurun_out/prof_tag> <round, e.g. r03> <task> <num_envs> <nv> <steps>

bench.py brackets its timed region with the engine's marker kernel (mjx_marker, tags 1 and
2, enqueued outside the timing), so every pass attributes exactly the dispatches of the
`steps` timed env steps -- the HIP-graph-captured env step the bench line measures.

Writes
  profiles/<round>_<tag>_kernel_stats.csv   the rocprofv3 --stats file of the kernel-trace run;
  profiles/<round>_<tag>_timed_region.json  per env step: span of the timed dispatches
                                            (first start .. last end) / steps, per-kernel
                                            dispatch counts and summed durations;
  profiles/<round>_<tag>_hbm_traffic.json   FETCH_SIZE x2 + WRITE_SIZE per env step, per
                                            kernel (separate --pmc passes; gfx950 FETCH
                                            correction, MI355X_MICROARCH.md HBM section);
  profiles/<round>_<tag>_pmc_sq.txt         SQ counters per env step and per world.
"""

import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MFMA_F32_FLOPS = 2 * 16 * 16 * 4  # v_mfma_f32_16x16x4_f32


def _find(d, pat):
  hits = sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))
  if not hits:
    raise FileNotFoundError(f"{pat} under {d}")
  return hits[0]


def _short(name):
  n = name.split("(")[0].replace("void ", "").strip()
  return n[:120]


def _region(rows, key="Dispatch_Id"):
  """Rows strictly between the first two marker dispatches (tags 1, 2), by dispatch id."""
  marks = sorted(int(r[key]) for r in rows if "marker_kernel" in r["Kernel_Name"])
  marks = sorted(set(marks))
  if len(marks) < 2:
    raise RuntimeError(f"expected 2 marker dispatches, found {len(marks)}")
  lo, hi = marks[0], marks[1]
  return [r for r in rows if lo < int(r[key]) < hi]


def kernel_trace(path, steps):
  with open(path) as fh:
    rows = list(csv.DictReader(fh))
  reg = _region(rows)
  t0 = min(int(r["Start_Timestamp"]) for r in reg)
  t1 = max(int(r["End_Timestamp"]) for r in reg)
  per = {}
  for r in reg:
    k = _short(r["Kernel_Name"])
    d = per.setdefault(k, [0, 0])
    d[0] += 1
    d[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
  kern = {k: {"dispatches_per_step": v[0] / steps, "ns_per_step": v[1] / steps,
              "avg_ns": v[1] / max(v[0], 1)} for k, v in sorted(per.items(), key=lambda x: -x[1][1])}
  return {"span_ms_per_step": (t1 - t0) / 1e6 / steps,
          "kernel_ns_per_step_sum": sum(v[1] for v in per.values()) / steps,
          "dispatches_per_step": len(reg) / steps, "kernels": kern}


def counters(path, steps):
  """{counter: {kernel: value per env step}} over the timed dispatches."""
  with open(path) as fh:
    rows = list(csv.DictReader(fh))
  reg = _region(rows)
  out = {}
  for r in reg:
    d = out.setdefault(r["Counter_Name"], {})
    k = _short(r["Kernel_Name"])
    d[k] = d.get(k, 0.0) + float(r["Counter_Value"]) / steps
  return out


def main():
  src, rnd, task, nenv, nv, steps = (sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]),
                                     int(sys.argv[5]), int(sys.argv[6]))
  tag = os.path.basename(src.rstrip("/")).replace("prof_", "")
  prof = os.path.join(ROOT, "profiles")
  shutil.copy(_find(os.path.join(src, "kt"), "*kernel_stats.csv"),
              os.path.join(prof, f"{rnd}_{tag}_kernel_stats.csv"))
  kt = kernel_trace(_find(os.path.join(src, "kt"), "*kernel_trace.csv"), steps)
  bench_line = None
  try:
    with open(os.path.join(src, "bench_prof.log")) as fh:
      for ln in fh:
        if ln.startswith("{"):
          bench_line = json.loads(ln)
  except OSError:
    pass
  kt.update(task=task, num_envs=nenv, steps=steps,
            bench_launch_ms=(bench_line or {}).get("roofline", {}).get("launch_ms"),
            bench_ms_per_step=(bench_line or {}).get("ms_per_step"),
            method="rocprofv3 --kernel-trace --stats over bench.py; dispatches between the two "
                   "mjx_marker kernels that bracket the timed region")
  with open(os.path.join(prof, f"{rnd}_{tag}_timed_region.json"), "w") as fh:
    json.dump(kt, fh, indent=1)
  res = {"task": task, "num_envs": nenv, "nv": nv, "path": "env_step_graph",
         "unit": "bytes per env step (the captured env step: physics + fused managers)"}
  f = counters(_find(os.path.join(src, "fetch"), "*counter_collection.csv"), steps).get("FETCH_SIZE", {})
  w = counters(_find(os.path.join(src, "write"), "*counter_collection.csv"), steps).get("WRITE_SIZE", {})
  res["fetch_bytes_per_step"] = {k: 2 * 1024 * v for k, v in sorted(f.items(), key=lambda x: -x[1])}
  res["write_bytes_per_step"] = {k: 1024 * v for k, v in sorted(w.items(), key=lambda x: -x[1])}
  res["traffic_bytes_per_env_step"] = (sum(res["fetch_bytes_per_step"].values()) +
                                       sum(res["write_bytes_per_step"].values()))
  sq = {}
  for sub in ("sq", "sq2"):
    sq_path = os.path.join(src, sub)
    if os.path.isdir(sq_path):
      sq.update(counters(_find(sq_path, "*counter_collection.csv"), steps))
  mfma = sum(v for c, d in sq.items() if "MFMA" in c and "INSTS" in c for v in d.values())
  res["mfma_flops_per_env_step"] = mfma * MFMA_F32_FLOPS
  tot = {c: sum(d.values()) for c, d in sq.items()}
  if tot.get("SQ_INSTS_VALU"):
    # the VALU issue ceiling of the bench line (bench.py roofline.frac_valu_issue): wave64
    # VALU instructions per env step, and per kernel the share of wave-cycles spent waiting
    res["valu_insts_per_env_step"] = tot["SQ_INSTS_VALU"]
    wc = sq.get("SQ_WAVE_CYCLES", {})
    res["wait_share_per_kernel"] = {
      k: {"wait_inst_any": sq.get("SQ_WAIT_INST_ANY", {}).get(k, 0.0) / c,
          "wait_any": sq.get("SQ_WAIT_ANY", {}).get(k, 0.0) / c}
      for k, c in sorted(wc.items(), key=lambda x: -x[1]) if c > 0 and k.startswith("mjx")}
  if tot.get("SQ_WAVE_CYCLES"):
    res["limiter"] = ("latency/issue: wait_any/wave_cycles = %.2f, VALU instructions per world "
                      "step %.0f, VMEM %.0f" % (tot.get("SQ_WAIT_ANY", 0) / tot["SQ_WAVE_CYCLES"],
                                                tot.get("SQ_INSTS_VALU", 0) / nenv,
                                                tot.get("SQ_INSTS_VMEM", 0) / nenv))
  res["method"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                   "bench.py; the timed region's dispatches (between the marker kernels) summed "
                   "per env step; FETCH_SIZE doubled (gfx950 correction, MI355X_MICROARCH.md)")
  with open(os.path.join(prof, f"{rnd}_{tag}_hbm_traffic.json"), "w") as fh:
    json.dump(res, fh, indent=1)
  if sq:
    lines = [f"# SQ counters per env step ({task}, {nenv} worlds), timed region of bench.py",
             "# (dispatches between the marker kernels); *_CYCLES / SQ_WAIT_* count quad-cycles."]
    kernels = sorted({k for d in sq.values() for k in d})
    for k in kernels:
      lines.append(f"[{k}]")
      for c in sorted(sq):
        v = sq[c].get(k, 0.0)
        lines.append(f"  {c:28s} {v:16.0f}   per world {v / nenv:12.1f}")
    lines.append("[all kernels]")
    for c in sorted(tot):
      lines.append(f"  {c:28s} {tot[c]:16.0f}   per world {tot[c] / nenv:12.1f}")
    if tot.get("SQ_WAVE_CYCLES"):
      lines.append(f"  wait_any/wave_cycles = {tot.get('SQ_WAIT_ANY', 0) / tot['SQ_WAVE_CYCLES']:.3f}")
    with open(os.path.join(prof, f"{rnd}_{tag}_pmc_sq.txt"), "w") as fh:
      fh.write("\n".join(lines) + "\n")
  print(json.dumps({"timed_region": {k: kt[k] for k in ("span_ms_per_step", "dispatches_per_step",
                                                        "bench_launch_ms", "bench_ms_per_step")},
                    "traffic_bytes_per_env_step": res["traffic_bytes_per_env_step"],
                    "mfma_flops_per_env_step": res["mfma_flops_per_env_step"]}, indent=1))


if __name__ == "__main__":
  main()
