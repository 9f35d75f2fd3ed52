"""Summarise a tools/gpu.sh profile run into profiles/<tag>/ (tracked):
  kernel_stats.csv       rocprofv3 --stats summary of the bench command
  pmc_summary.json       per-kernel means of the PMC passes + derived HBM bytes, clock, VALU use
and update profiles/pmc_traffic.json, read by bench.py for the roofline (HBM bytes and wave64
VALU instructions per launch of the step kernel).  Each entry records the sha256 prefix of the
gol_kernels.hip it was measured on; bench.py ignores an entry whose hash differs.

    python tools/pmc_summary.py <tag> <bench key, e.g. weak:131072x1048576:k12:band> [--clock GHZ]

The shader clock of a dispatch is GRBM_GUI_ACTIVE / 8 / its duration (rocprofv3 sums the 8 XCDs),
which reads high on dispatches shorter than ~0.3 ms (MI355X_MICROARCH.md, 'DVFS give-back'): for
those the clock is taken only from --clock (the in-kernel s_memtime / s_memrealtime median of
tools/timeline.py clock), else left null.

HBM bytes per launch = FETCH_SIZE*2 + WRITE_SIZE (KiB -> bytes), the gfx950 correction of
MI355X_MICROARCH.md §HBM (FETCH_SIZE reports half of a wide streaming read)."""
import collections
import csv
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag, key = sys.argv[1], sys.argv[2]  # e.g. r01 weak:131072x1048576:n1:k16:cpl0 (bench.py load_pmc key)
CLOCK = float(sys.argv[sys.argv.index("--clock") + 1]) if "--clock" in sys.argv else None
SHORT_NS = 300e3  # below this the GRBM quotient is not a clock
src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
dst = os.path.join(ROOT, "profiles", tag)
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))

means = collections.defaultdict(dict)
for d in sorted(os.listdir(src)):
    f = os.path.join(src, d, "run_counter_collection.csv")
    if not d.startswith("pmc_") or not os.path.exists(f):
        continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        # one kernel can be launched with several grids (a step's interior and its edge rows):
        # dispatches are grouped by (kernel, grid size)
        acc[(f'{r["Kernel_Name"]} @grid {r["Grid_Size"]}', r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in acc.items():
        means[k][c] = sum(v) / len(v)

# mean duration per (kernel, grid) from the trace pass
durs = collections.defaultdict(list)
for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))):
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    durs[f'{r["Kernel_Name"]} @grid {g}'].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
# AverageNs: the steady second half of the dispatches (the GPU's clocks settle during the first
# ~0.1-0.2 s of load: bench.py's warmup); AverageNs_all: every dispatch (rocprof's --stats figure)
stats = {k: {"AverageNs": sum(v[len(v) // 2:]) / len(v[len(v) // 2:]), "AverageNs_all": sum(v) / len(v), "Calls": len(v),
             "TotalNs": sum(v)} for k, v in durs.items()}
json.dump(stats, open(os.path.join(dst, "kernel_grid_stats.json"), "w"), indent=1)
out = {}
for k, c in means.items():
    ns = float(stats[k]["AverageNs"]) if k in stats else None
    e = {"counters": c, "avg_ns_trace": ns}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        b = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
        e["hbm_bytes_per_launch"] = b
        if ns:
            e["hbm_GBs"] = b / ns
    if "GRBM_GUI_ACTIVE" in c and ns:
        e["grbm_clock_GHz"] = c["GRBM_GUI_ACTIVE"] / 8 / ns
        if CLOCK:
            e["clock_GHz"], e["clock_source"] = CLOCK, "in-kernel s_memtime / s_memrealtime (tools/timeline.py clock)"
        elif ns >= SHORT_NS:
            e["clock_GHz"], e["clock_source"] = e["grbm_clock_GHz"], "GRBM_GUI_ACTIVE / 8 / trace duration"
        else:
            e["clock_GHz"], e["clock_source"] = None, "dispatch < 0.3 ms: the GRBM quotient reads high; no in-kernel clock given"
        if "SQ_INSTS_VALU" in c and e["clock_GHz"]:
            e["valu_issue_frac"] = c["SQ_INSTS_VALU"] / (256 * 4 * 0.5 * e["clock_GHz"] * ns)
    out[k] = e
json.dump(out, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
if not out:
    sys.exit(f"no PMC counter rows under {src}")
main = max(out, key=lambda k: stats.get(k, {}).get("TotalNs", 0))
tp = os.path.join(ROOT, "profiles", "pmc_traffic.json")
t = json.load(open(tp)) if os.path.exists(tp) else {}
sys.path.insert(0, ROOT)
from bench import kernel_source_hash  # noqa: E402  (the kernel sources + Makefile, as bench.py checks)
src_hash = kernel_source_hash()
if "hbm_bytes_per_launch" in out[main]:
    t[key] = {"kernel": main, "kernel_src": src_hash, "trace_calls": stats[main]["Calls"], "bytes_per_launch": out[main]["hbm_bytes_per_launch"],
              "profile": f"profiles/{tag}", "avg_ns_trace": out[main]["avg_ns_trace"]}
    c = out[main]["counters"]
    if "SQ_INSTS_VALU" in c:
        t[key]["valu_insts_per_launch"] = c["SQ_INSTS_VALU"]
    if "SQ_INSTS_SALU" in c:
        t[key]["salu_insts_per_launch"] = c["SQ_INSTS_SALU"]
    if "valu_issue_frac" in out[main]:
        t[key]["valu_issue_frac_profile_clock"] = round(out[main]["valu_issue_frac"], 4)
    if "clock_GHz" in out[main]:
        ck = out[main]["clock_GHz"]
        t[key]["clock_GHz"] = round(ck, 3) if ck else None
        t[key]["clock_source"] = out[main]["clock_source"]
    json.dump(t, open(tp, "w"), indent=1)
print(json.dumps(out[main], indent=1))
