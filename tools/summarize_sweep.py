"""Summarize gpurun_out/sweep.jsonl (render_once results, optional diagnostics counters)."""
import json
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sweep.jsonl"
for line in open(path):
    d = json.loads(line)
    if d.get("failed"):
        print(d["name"], "FAILED")
        continue
    r = d["r"][-1] if isinstance(d["r"], list) else d["r"]
    dbg = r["debug"]
    extra = ""
    if dbg[0]:
        util = dbg[1] / (64 * dbg[0])
        span = (dbg[4] - dbg[5]) / 100e6 * 1e3
        mean_end = (dbg[6] * 256 / dbg[7] - dbg[5]) / 100e6 * 1e3 if dbg[7] else 0
        extra = " util %.3f hitgrp/iter %.3f wave-end spread %.1f ms (mean %.1f)" % (
            util, dbg[2] / dbg[0], span, mean_end)
    tf = r["sphere_tests"] * 23 / (r["kernel_ms"] * 1e-3) / 1e12
    print("%-11s %-22s %7.1f ms (+%.2f resolve) %7.1f Msps %.3e tests/s %.1f TF grid %d%s" % (
        d["name"], d["env"], r["kernel_ms"], r.get("resolve_ms", 0), r["msamples_per_s"],
        r["tests_per_s"], tf, r["grid_blocks"], extra))
