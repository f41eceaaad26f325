"""Collect a gpurun profiling batch (tools/gpu_profile.sh) into profiles/:
kernel-trace stats of the bench command, PMC summaries, and profiles/traffic.json (HBM bytes per
launch of the tracer kernel for the bench workload, corrected per MI355X_MICROARCH.md: FETCH_SIZE
and WRITE_SIZE are KB; gfx950 FETCH_SIZE counts half the bytes of wide streaming reads, so it is
doubled -- an upper bound for the tracer's narrow scalar loads)."""
import csv
import collections
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(ROOT, "gpurun_out", "prof")
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
dst = os.path.join(ROOT, "profiles")
os.makedirs(dst, exist_ok=True)


def pmc(name):
    path = os.path.join(src, name, "run_counter_collection.csv")
    agg = collections.defaultdict(float)
    calls = collections.Counter()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        calls[(k, r["Counter_Name"])] += 1
    return {f"{k}|{c}": {"sum": v, "dispatches": calls[(k, c)]} for (k, c), v in agg.items()}


shutil.copy(os.path.join(src, "kt", "bench_kernel_stats.csv"),
            os.path.join(dst, f"{tag}_bench_kernel_stats.csv"))
bench = json.load(open(os.path.join(src, "kt_bench.json")))
summary = {"bench_under_rocprof": {k: bench[k] for k in ("value", "ms_per_step", "roofline")}}
for name in ("pmc_fetch", "pmc_write", "pmc_sq1", "pmc_sq2"):
    if os.path.exists(os.path.join(src, name)):
        summary[name] = pmc(name)
with open(os.path.join(dst, f"{tag}_pmc_summary.json"), "w") as f:
    json.dump(summary, f, indent=1)

kernel = bench["roofline"]["kernel"]
fetch = summary["pmc_fetch"][f"{kernel}|FETCH_SIZE"]
write = summary["pmc_write"][f"{kernel}|WRITE_SIZE"]
per_launch = (2 * fetch["sum"] / fetch["dispatches"] + write["sum"] / write["dispatches"]) * 1024
cfg = bench["config"]
key = f"{cfg['scene']}_{cfg['width']}x{cfg['height']}_s{cfg['spp']}_d{cfg['max_depth']}_n1"
traffic_path = os.path.join(dst, "traffic.json")
traffic = json.load(open(traffic_path)) if os.path.exists(traffic_path) else {}
traffic[key] = {"hbm_bytes_per_launch": per_launch, "kernel": kernel, "fetch_kb": fetch["sum"] / fetch["dispatches"],
                "write_kb": write["sum"] / write["dispatches"], "round": tag,
                "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of tools/render_once.py "
                        "at the bench config; FETCH_SIZE doubled (gfx950 correction)"}
# VALUBusy / VALUUtilization (rocprofiler-sdk counter_defs.yaml, gfx950 rows):
#   100 * SQ_ACTIVE_INST_VALU / CU_NUM / max(GRBM_GUI_ACTIVE), max over the 8 XCDs = sum / 8
#   100 * SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU * 64)
sq1, sq2 = summary.get("pmc_sq1", {}), summary.get("pmc_sq2", {})
try:
    valu = sq2[f"{kernel}|SQ_ACTIVE_INST_VALU"]["sum"]
    thread = sq2[f"{kernel}|SQ_THREAD_CYCLES_VALU"]["sum"]
    gui = sq1[f"{kernel}|GRBM_GUI_ACTIVE"]["sum"] / 8
    traffic[key]["valu_busy_pct"] = round(100 * valu / 256 / gui, 1)
    traffic[key]["valu_utilization_pct"] = round(100 * thread / (valu * 64), 1)
    traffic[key]["valu_note"] = ("VALUBusy = 100 SQ_ACTIVE_INST_VALU / 256 CUs / (GRBM_GUI_ACTIVE / 8 "
                                 "XCDs); VALUUtilization = 100 SQ_THREAD_CYCLES_VALU / "
                                 "(SQ_ACTIVE_INST_VALU x 64): active lanes per VALU instruction")
except KeyError:
    pass
with open(traffic_path, "w") as f:
    json.dump(traffic, f, indent=1)
print(json.dumps(traffic[key]))
