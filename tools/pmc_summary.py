"""Summarise tools/profile.sh output: mean per-dispatch PMC values of the search
kernel (mgj_search) and the kernel-trace average duration."""
import csv
import glob
import json
import sys
from collections import defaultdict

d, workload = sys.argv[1], sys.argv[2]
KERNEL = sys.argv[3] if len(sys.argv) > 3 else "mgj_search"
counters = defaultdict(list)
for f in glob.glob(f"{d}/pmc*/**/*counter_collection.csv", recursive=True):
    per_dispatch = defaultdict(lambda: defaultdict(float))
    for row in csv.DictReader(open(f)):
        if KERNEL not in row.get("Kernel_Name", ""):
            continue
        per_dispatch[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
        res = {k: row.get(k) for k in ("Grid_Size", "Workgroup_Size", "VGPR_Count", "Accum_VGPR_Count",
                                         "SGPR_Count", "Scratch_Size", "LDS_Block_Size")}
    # full-size launches only (bench --no-ttfm runs no early-exit searches; be safe anyway)
    ref = "SQ_INSTS_VALU" if any("SQ_INSTS_VALU" in d for d in per_dispatch.values()) else None
    top = max((d.get(ref, 0.0) for d in per_dispatch.values()), default=0.0) if ref else 0.0
    for disp in per_dispatch.values():
        if ref and disp.get(ref, 0.0) < 0.5 * top:
            continue
        for k, v in disp.items():
            counters[k].append(v)
stats = {}
for f in glob.glob(f"{d}/trace/**/*kernel_stats.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        stats[row["Name"]] = {"calls": int(row["Calls"]), "average_ns": float(row["AverageNs"]),
                              "percentage": float(row["Percentage"])}
mean = {k: sum(v) / len(v) for k, v in counters.items()}
# per-dispatch durations: bench.py also launches the kernel for its early-exit time-to-first-model
# search (a short launch that stops at the first hit); the timed steps are the full-count launches
full = []
for f in glob.glob(f"{d}/trace/**/*kernel_trace.csv", recursive=True):
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            for r in csv.DictReader(open(f)) if KERNEL in r["Kernel_Name"]]
    if durs:
        med = sorted(durs)[len(durs) // 2]
        full = [x for x in durs if x > 0.5 * med]
bench = json.loads(open(f"{d}/bench_under_trace.json").read())
C = bench["config"]["candidates_per_gpu_step"]
out = {"workload": workload, "kernel": KERNEL, "candidates_per_launch": C,
       "jit_source_sha16": bench["config"].get("jit_source_sha16"),
       "per_launch_counters": mean, "kernel_stats": stats}
try:
    out["resources"] = res
except NameError:
    pass
der = {}
if "SQ_INSTS_VALU" in mean:
    der["valu_wave_instructions_per_candidate"] = mean["SQ_INSTS_VALU"] * 64 / C
if "FETCH_SIZE" in mean:
    # gfx950 reports half of wide reads (MI355X_MICROARCH.md §HBM): doubled; units are KB
    der["hbm_bytes_per_launch"] = (2 * mean["FETCH_SIZE"] + mean.get("WRITE_SIZE", 0.0)) * 1024
k = [v for n, v in stats.items() if KERNEL in n]
if k:
    der["rocprof_kernel_avg_ms"] = k[0]["average_ns"] / 1e6
    der["bench_kernel_ms"] = bench["roofline"]["kernel_ms"]
    der["bench_value_under_trace"] = bench["value"]
    if full:
        der["rocprof_full_launch_avg_ms"] = sum(full) / len(full)
        der["rocprof_full_launch_last10_avg_ms"] = sum(full[-10:]) / len(full[-10:])
    if "SQ_INSTS_VALU" in mean:
        ms = der.get("rocprof_full_launch_last10_avg_ms", k[0]["average_ns"] / 1e6)
        der["measured_valu_lane_ops_per_s_T"] = mean["SQ_INSTS_VALU"] * 64 / (ms * 1e-3) / 1e12
        der["valu_frac_of_78.6T"] = der["measured_valu_lane_ops_per_s_T"] / (256 * 4 * 32 * 2.4e9 / 1e12)
    if "SQ_INSTS_SALU" in mean:
        der["salu_instructions_per_candidate"] = mean["SQ_INSTS_SALU"] * 64 / C
    if "GRBM_GUI_ACTIVE" in mean and full:
        der["effective_clock_ghz"] = mean["GRBM_GUI_ACTIVE"] / 8 / (sum(full[-10:]) / len(full[-10:]) * 1e-3) / 1e9
out["derived"] = der
print(json.dumps(out, indent=1))
