"""Where the flat scan's wave time goes: the report of a stats-build frame (VCRT_DEBUG_STATS=1,
s_memtime per phase; tools/gpu_run.sh phases)."""
import json
import sys
st = json.load(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/phases.json"))
d = st["debug"]
wi = d[0]
tot = d[14]
print("kernel_ms %.2f wave-iters %d waves %d" % (st["kernel_ms"], wi, d[7]))
for name, k in (("scan", 8), ("big list", 15), ("levels", 9), ("node pushes", 16),
                ("node passes", 10), ("group passes", 11), ("cand passes", 12),
                ("shade+sky", 17), ("block fetch", 18), ("camera trace", 23)):
    print("%-13s %5.1f%% of wave time, %8.1f ticks per wave-iter" % (name, 100 * d[k] / tot, d[k] / wi))
if d[3]:
    print("  of which shading %5.1f%% of wave time, %8.1f ticks per wave-iter" % (100 * d[3] / tot, d[3] / wi))
print("cand passes per wave-iter %.2f; node %.2f group %.2f (from counters)" % (
    d[13] / wi, (st["bound_tests"] / wi), st["group_tests"] / wi))
print("total ticks per wave-iter %.1f" % (tot / wi))
if len(d) > 31 and d[24]:
    print("camera trace: entries per wave-iter %.2f, camera lanes %.1f of %.1f live; listed loop "
          "%.2f trips for %.2f groups per camera lane (util %.2f); root loop %.2f trips for %.2f "
          "candidates per camera lane (util %.2f)" % (
              d[24] / wi, d[25] / d[24], d[26] / d[24], d[27] / d[24], d[28] / d[25],
              d[28] / max(1, d[27] * 64), d[29] / d[24], d[30] / d[25], d[30] / max(1, d[29] * 64)))
    print("live lanes per wave-iter %.1f; main-scan hit lanes per wave-iter %.1f" % (d[1] / wi, d[31] / wi))
if len(d) > 22 and d[22]:
    print("flat passes per wave-iter %.2f, partial %.2f; entries per live lane %.3f" % (
        d[22] / wi, d[21] / wi, d[19] / d[20]))
if len(d) > 39 and d[33]:
    print("loop top: retire %.1f%% of wave time (%.1f ticks per wave-iter), run in %.2f of "
          "wave-iters, %.2f quanta per wave-iter" % (100 * d[32] / tot, d[32] / wi, d[38] / wi,
                                                     d[39] / wi))
    print("fetch loop in %.2f of wave-iters; blocks %.4f, items started %.3f, next items %.3f, "
          "switches %.3f per wave-iter" % (d[33] / wi, d[34] / wi, d[35] / wi, d[36] / wi,
                                           d[37] / wi))
