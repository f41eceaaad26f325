"""Collect a gpurun profiling batch (tools/gpu_run.sh profile) into profiles/<tag>_*:
  <tag>_bench_{c4,c3,c2,c5}.json     the bench lines of the BASELINE configs, their roofline
                                     counters (traffic, VALU issue) merged from this batch's own
                                     PMC passes (the same build and workload; bench.py merges
                                     profiles/traffic.json the same way at run time)
  <tag>_bench_kernel_stats[_cfg].csv rocprofv3 --kernel-trace --stats of each bench command
  <tag>_pmc_summary.json             the PMC passes per config and kernel, and derived figures
  traffic.json                       per workload key: the tracer kernel's HBM bytes per launch
                                     and VALU figures, read by bench.py when its kernel matches

Derived figures (MI355X_MICROARCH.md rocprofv3 sections):
  hbm_bytes_per_launch = 2 * FETCH_SIZE + WRITE_SIZE (KB -> B; gfx950 FETCH_SIZE counts half
                         the bytes of wide streaming reads, doubled: an upper bound here)
  valu_issue_frac      = SQ_INSTS_VALU * 4 cycles / (1024 SIMDs * 2.4 GHz * kernel time): issue
                         SLOTS against one quad-cycle per instruction at the peak clock. Round 6
                         measured three VALU rates on gfx950 (fast add/sub/mul/mov/logic ~2.7
                         cycles, the rest ~4.5, sqrt/rcp 8.5: tools/microbench_classes.hip), so
                         this is a count, not the pipe's occupancy; the class-weighted pipe time
                         is in profiles/r06_cycle_attrib.txt (C4: 0.99 of the SIMD cycles)
  effective_clock_ghz  = GRBM_GUI_ACTIVE / 8 XCDs / kernel time
  valu_lane_util       = SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU * 64): active lanes per
                         VALU instruction
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(ROOT, "gpurun_out", "prof")
tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
dst = os.path.join(ROOT, "profiles")
os.makedirs(dst, exist_ok=True)

CFG_KEYS = {  # render_once arguments of the PMC passes (tools/gpu_run.sh profile)
    "c4": ("final", 1920, 1080, 1024, 10),
    "c3": ("final", 1920, 1080, 256, 10),
    "c2": ("three", 800, 450, 64, 8),
    "c5": ("stress4096", 3840, 2160, 4096, 50),
}


def pmc(name):
    """Counters of each kernel's last dispatch (the passes render two frames: the second is the
    steady state, e.g. after the cost order's measuring frame)."""
    path = os.path.join(src, name, "run_counter_collection.csv")
    last = {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        key = (k, r["Counter_Name"])
        d = int(r["Dispatch_Id"])  # one row per dispatch and counter
        if key not in last or d > last[key][0]:
            last[key] = (d, float(r["Counter_Value"]))
    return {f"{k}|{c}": v for (k, c), (_, v) in last.items()}


def run_stats(name):
    """The render_once JSON (profiled run) printed into the pass's log: its last frame."""
    for line in open(os.path.join(src, name + ".log")):
        if line.startswith("{") or line.startswith("["):
            st = json.loads(line)
            return st[-1] if isinstance(st, list) else st
    raise ValueError(name)


def kernel_name(st):
    return st["kernel"]  # vcrt_stats.kernel: the symbol the profiled frame launched


for cfg in ("c4", "c3", "c2", "c5"):
    p = os.path.join(src, f"bench_{cfg}.err")
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, f"{tag}_bench_{cfg}.err"))
    kt = os.path.join(src, f"kt_{cfg}", "bench_kernel_stats.csv")
    if os.path.exists(kt):
        shutil.copy(kt, os.path.join(dst, f"{tag}_bench_kernel_stats"
                                          f"{'' if cfg == 'c4' else '_' + cfg}.csv"))
        shutil.copy(os.path.join(src, f"kt_{cfg}.json"),
                    os.path.join(dst, f"{tag}_bench_under_rocprof_{cfg}.json"))

summary = {}
traffic_path = os.path.join(dst, "traffic.json")
traffic = json.load(open(traffic_path)) if os.path.exists(traffic_path) else {}
for cfg, (scene, w, h, spp, depth) in CFG_KEYS.items():
    if not os.path.exists(os.path.join(src, f"{cfg}_sq1")):
        continue
    passes = {}
    for p in ("fetch", "write", "sq1", "sq2"):
        passes.update(pmc(f"{cfg}_{p}"))
    st = run_stats(f"{cfg}_sq1")
    kernel = kernel_name(st)
    t = st["kernel_ms"] * 1e-3
    c = {k.split("|")[1]: v for k, v in passes.items() if k.startswith(kernel + "|")}
    derived = {
        "kernel": kernel,
        "kernel_ms_profiled": st["kernel_ms"],
        "hbm_bytes_per_launch": (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024,
        "fetch_kb": c["FETCH_SIZE"], "write_kb": c["WRITE_SIZE"],
        "valu_issue_frac": round(c["SQ_INSTS_VALU"] * 4 / (1024 * 2.4e9 * t), 4),
        "effective_clock_ghz": round(c["GRBM_GUI_ACTIVE"] / 8 / t / 1e9, 3),
        "valu_lane_util": round(c["SQ_THREAD_CYCLES_VALU"] / (c["SQ_ACTIVE_INST_VALU"] * 64), 4),
        "salu_per_valu": round(c["SQ_INSTS_SALU"] / c["SQ_INSTS_VALU"], 4),
        "segments": st["segments"],
        "valu_instr_per_segment_wave": round(c["SQ_INSTS_VALU"] * 64 / st["segments"], 1),
    }
    summary[cfg] = {"render": {k: st[k] for k in ("kernel_ms", "segments", "group_tests",
                                                    "bound_tests", "kernel_variant",
                                                    "tables_in_lds", "block_threads",
                                                    "grid_blocks", "accumulate_chunk")},
                    "counters_per_dispatch": passes, "derived": derived}
    key = f"{scene}_{w}x{h}_s{spp}_d{depth}_n1"
    traffic[key] = dict(derived, source=f"profiles/{tag}_pmc_summary.json [{cfg}]",
                        round=tag)
# the bench lines with this batch's counters (bench.py's own merge, redone with the fresh file)
for cfg, (scene, w, h, spp, depth) in CFG_KEYS.items():
    p = os.path.join(src, f"bench_{cfg}.json")
    if not os.path.exists(p):
        continue
    line = json.loads([ln for ln in open(p) if ln.startswith("{")][-1])
    prof = traffic.get(f"{scene}_{w}x{h}_s{spp}_d{depth}_n1", {})
    if cfg in summary and prof.get("kernel") == line["roofline"]["kernel"]:
        rf = line["roofline"]
        rf["traffic"] = prof["hbm_bytes_per_launch"]
        for k in ("valu_issue_frac", "valu_lane_util", "effective_clock_ghz"):
            rf[k] = prof[k]
        rf["profile"] = prof["source"]
    with open(os.path.join(dst, f"{tag}_bench_{cfg}.json"), "w") as f:
        f.write(json.dumps(line) + "\n")
with open(os.path.join(dst, f"{tag}_pmc_summary.json"), "w") as f:
    json.dump(summary, f, indent=1)
with open(traffic_path, "w") as f:
    json.dump(traffic, f, indent=1)
for cfg, s in summary.items():
    print(cfg, json.dumps(s["derived"]))
