"""Summarise tools/gpu_pmc_ab.sh: per tag, the trace kernel's instruction counters per frame and
the derived issue figures (VALU issue = SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x 2.4 GHz x time)).

  python tools/pmc_ab_summary.py [gpurun_out/pmcab]
"""
import collections
import csv
import glob
import json
import os
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcab"


def counters(d):
    agg = collections.defaultdict(float)
    calls = collections.Counter()
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        k = r["Kernel_Name"].split("(")[0]
        if not k.startswith("vcrt_trace"):
            continue
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        calls[(k, r["Counter_Name"])] += 1
    return {c: v / calls[(k, c)] for (k, c), v in agg.items()}, sorted({k for k, _ in agg})


def stats(log):
    for line in open(log):
        if line.startswith("[") or line.startswith("{"):
            st = json.loads(line)
            return st[-1] if isinstance(st, list) else st
    return None


tags = sorted({os.path.basename(p)[:-2] for p in glob.glob(os.path.join(src, "*_1"))})
for t in tags:
    c1, k1 = counters(os.path.join(src, t + "_1"))
    c2, _ = counters(os.path.join(src, t + "_2"))
    c = {**c1, **c2}
    st = stats(os.path.join(src, t + "_1.log")) or {}
    ms = st.get("kernel_ms", float("nan"))
    v = c.get("SQ_INSTS_VALU", 0.0)
    segs = st.get("segments", 0)
    line = {
        "kernel": k1,
        "kernel_ms": round(ms, 3),
        "valu_G": round(v / 1e9, 3),
        "salu_G": round(c.get("SQ_INSTS_SALU", 0) / 1e9, 3),
        "lds_G": round(c.get("SQ_INSTS_LDS", 0) / 1e9, 3),
        "smem_G": round(c.get("SQ_INSTS_SMEM", 0) / 1e9, 3),
        "vmem_G": round(c.get("SQ_INSTS_VMEM", 0) / 1e9, 3),
        "valu_issue": round(v * 4 / (1024 * 2.4e9 * ms * 1e-3), 4) if ms == ms else None,
        "lane_util": round(c.get("SQ_THREAD_CYCLES_VALU", 0) /
                           max(1.0, c.get("SQ_ACTIVE_INST_VALU", 0) * 64), 4),
        "valu_per_wave_segment": round(v / max(1, segs / 64), 1),
        "wait_inst_any/active_any": round(c.get("SQ_WAIT_INST_ANY", 0) /
                                          max(1.0, c.get("SQ_ACTIVE_INST_ANY", 0)), 3),
    }
    print(t, json.dumps(line))
