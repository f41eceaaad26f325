"""Cycle attribution of the flat tracer kernel (verdict r05 item 2): the measured instruction
attribution (tools/valu_regions.py: every instruction of the product code object in its counted
region x the region's entries in a stats frame of the same workload) weighted by the issue cost
of each instruction's class, measured by tools/microbench_classes.hip on the same GPU.

Costs are SIMD cycles per wave64 instruction, from GRBM_GUI_ACTIVE of the microbenchmark's
dispatches (clock-independent), at 5 waves per SIMD (the flat kernel's occupancy; 8 independent
chains per wave) and at 1 wave per SIMD (one wave's own issue interval). gfx950 measured three
VALU rates: "fast" (v_add/sub/mul_f32, v_mov_b32, v_and/or/xor_b32, v_add_u32 with vector or
literal operands: ~2.7 cycles), "normal" (everything else: fma, min/max, compares, selects,
packed, f64, shifts, lane ops, and a fast op with a scalar operand: ~4.5 cycles) and
transcendental (v_sqrt/v_rcp_f32 ~8.5, v_rcp_f64 ~16.6); scalar instructions ~4.6 per SIMD.

  python tools/cycle_attrib.py --stats STATS.json --micro-grbm GRBM.csv [--pmc PMC.json]
                               [--out profiles/r06_cycle_attrib.txt]
"""
import argparse
import collections
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import valu_attrib as V  # noqa: E402
import valu_regions as R  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# double-rate VALU operations on gfx950 (microbench_classes: ~2.7 cycles per wave64 instruction at
# 5 waves per SIMD against ~4.5), when no operand is a scalar register
FAST = {"v_add_f32", "v_sub_f32", "v_subrev_f32", "v_mul_f32", "v_mov_b32", "v_and_b32",
        "v_or_b32", "v_xor_b32", "v_add_u32", "v_sub_u32", "v_subrev_u32"}
TRANS = re.compile(r"^v_(sqrt|rcp|rsq|rcp_iflag|exp|log|sin|cos)_f32")
TRANS64 = re.compile(r"^v_(rcp|sqrt|rsq)_f64")
SCALAR_OPERAND = re.compile(r"(^|[\s,\[-])(s\d+|s\[\d+:\d+\]|vcc(_lo|_hi)?|exec(_lo|_hi)?|m0|ttmp)")
# the microbenchmark kernel whose cycles stand for each class
KERNEL = {"fast": "k_mul", "normal": "k_fma", "trans": "k_sqrt", "trans64": "k_rcp64",
          "salu": "k_salu"}
# sub-labels of the normal class, for the report
SUBCLASS = [("packed", r"^v_pk_"), ("f64", r"_f64"), ("cmp", r"^v_cmpx?_"),
            ("cndmask", r"^v_cndmask"), ("minmax", r"^v_(max|min|med)"),
            ("fma", r"^v_(fma|fmac|mad)"), ("lane", r"^v_(readlane|readfirstlane|writelane)"),
            ("dpp", r"_dpp$"), ("div", r"^v_div_"), ("int", r"^v_")]


def base(mn):
    return re.sub(r"_e(32|64)$", "", mn)


def klass(mn, ops):
    """(class, sub-label) of one instruction, or None if it is neither VALU nor SALU."""
    if R.is_salu(mn):
        return "salu", "salu"
    if not V.is_valu(mn):
        return None
    b = base(mn)
    if TRANS64.match(b):
        return "trans64", "trans64"
    if TRANS.match(b):
        return "trans", "trans"
    operands = ops.split(" ", 1)[1] if " " in ops.strip() else ""
    if b in FAST and not SCALAR_OPERAND.search(operands):
        return "fast", "fast"
    if b in FAST:
        return "normal", "fast op, scalar operand"
    for lab, pat in SUBCLASS:
        if re.search(pat, b):
            return "normal", lab
    return "normal", "other"


def grbm_costs(path):
    """Cycles per wave64 instruction per microbenchmark kernel at 1 / 5 / 8 waves per SIMD: each
    kernel ran 3 configurations (1, 8, 5 waves per SIMD) x (1 warm-up + 5 timed) dispatches."""
    per = collections.defaultdict(dict)
    for row in csv.DictReader(open(path)):
        d = int(row["Dispatch_Id"])
        per[d]["k"] = row["Kernel_Name"].split("(")[0].strip()
        if row["Counter_Name"] == "GRBM_GUI_ACTIVE":
            per[d]["g"] = per[d].get("g", 0.0) + float(row["Counter_Value"])
    byk = collections.defaultdict(list)
    for d in sorted(per):
        byk[per[d]["k"]].append(per[d]["g"])
    out = {}
    insts = 2048 * 8  # ITERS x 8 per wave

    def mean(xs):  # GRBM_GUI_ACTIVE sums the 8 XCDs
        return sum(xs) / len(xs) / 8.0

    for k, g in byk.items():
        if len(g) < 18:
            continue
        out[k] = {"w1": mean(g[1:6]) / insts, "w8": mean(g[7:12]) / (8 * insts),
                  "w5": mean(g[13:18]) / (5 * insts)}
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--stats", required=True, help="stats-build render_once JSON (region counts)")
    p.add_argument("--micro-grbm", required=True,
                   help="rocprofv3 counter_collection.csv (GRBM_GUI_ACTIVE) of microbench_classes")
    p.add_argument("--pmc", default=None,
                   help="JSON of the product frame's counters {name: value per dispatch}")
    p.add_argument("--hsaco", default=None)
    p.add_argument("--kernel", default="vcrt_trace_cull_flat")
    p.add_argument("--out", default=None)
    a = p.parse_args()
    product = os.path.join(ROOT, "vulkancomputeraytracing_amd", "lib", "vcrt_tracer.hsaco")
    insts, label, _ = R.assign_regions(a.hsaco, product, a.kernel)
    st = json.load(open(a.stats))
    st = st[-1] if isinstance(st, list) else st
    d = st["debug"]
    waves = d[7]

    def entries(r):
        return waves if r < 0 else d[R.REGION_DEBUG_BASE + r]

    mc = grbm_costs(a.micro_grbm)
    cost5 = {c: mc[k]["w5"] for c, k in KERNEL.items()}
    dyn = collections.Counter()
    sub = collections.Counter()
    mnem = collections.Counter()
    reg = collections.defaultdict(collections.Counter)
    for _, mn, ops, r in insts:
        kc = klass(mn, ops)
        if kc is None:
            continue
        c, lab = kc
        n = entries(r)
        dyn[c] += n
        sub[(c, lab)] += n
        mnem[(mn, c)] += n
        reg[r][c] += n
    valu = sum(v for c, v in dyn.items() if c != "salu")
    pipe = {c: v * cost5[c] for c, v in dyn.items()}
    valu_cyc = sum(v for c, v in pipe.items() if c != "salu")
    nan = float("nan")
    L = []
    w = L.append
    w("Cycle attribution of %s at C4 (tools/cycle_attrib.py)" % a.kernel)
    w("stats frame: %d segments, %d wave-iterations, %d waves" % (st["segments"], d[0], waves))
    w("")
    w("Issue costs measured on the GPU (tools/microbench_classes.hip, GRBM_GUI_ACTIVE per")
    w("dispatch): SIMD cycles per wave64 instruction, 8 independent chains per wave:")
    w("  %-8s %-10s %10s %10s %10s" % ("class", "kernel", "1 wave", "5 waves", "8 waves"))
    for c, k in KERNEL.items():
        w("  %-8s %-10s %10.2f %10.2f %10.2f" % (c, k, mc[k]["w1"], mc[k]["w5"], mc[k]["w8"]))
    w("  every form at 5 waves per SIMD:")
    items = sorted(mc.items(), key=lambda kv: kv[1]["w5"])
    for i in range(0, len(items), 6):
        w("    " + ", ".join("%s %.2f" % (k, v["w5"]) for k, v in items[i:i + 6]))
    w("")
    w("Dynamic instruction mix of one C4 frame (wave64 instructions, from the attribution):")
    w("  %-34s %14s %8s %16s %7s" % ("class / kind", "instructions", "of VALU", "VALU cycles",
                                      "share"))
    for (c, lab), v in sorted(sub.items(), key=lambda kv: -kv[1]):
        cy = v * cost5[c]
        is_v = c != "salu"
        w("  %-34s %14.4g %7.1f%% %16.4g %6.1f%%" % (
            c + " / " + lab, v, 100.0 * v / valu if is_v else nan, cy if is_v else nan,
            100.0 * cy / valu_cyc if is_v else nan))
    w("  VALU: %.4g instructions, %.4g SIMD cycles at the 5-wave costs (%.2f per instruction);"
      % (valu, valu_cyc, valu_cyc / valu))
    w("  SALU: %.4g instructions, %.4g cycles of the scalar unit" % (dyn["salu"],
                                                                    pipe.get("salu", 0.0)))
    w("")
    w("The most frequent instructions (dynamic, class):")
    for (mn, c), v in mnem.most_common(24):
        w("  %14.4g  %-28s %s" % (v, mn, c))
    w("")
    w("Regions by VALU cycles (5-wave costs):")
    rows = []
    for r, cc in reg.items():
        cy = sum(v * cost5[c] for c, v in cc.items() if c != "salu")
        rows.append((cy, r, cc))
    rows.sort(key=lambda t: -t[0])
    for cy, r, cc in rows[:28]:
        mix = ", ".join("%s %.3g" % (c, v) for c, v in cc.most_common(4))
        w("  %12.4g %5.1f%%  %-34s %s" % (cy, 100.0 * cy / valu_cyc, label(r), mix))
    if a.pmc:
        pm = json.load(open(a.pmc))
        simd_cycles = 1024 * pm["GRBM_GUI_ACTIVE"] / 8.0
        w("")
        w("Against the product frame (PMC per dispatch, %s):" % os.path.basename(a.pmc))
        w("  GRBM_GUI_ACTIVE / 8 = %.4g cycles per XCD; x 1024 SIMDs = %.4g SIMD cycles" % (
            pm["GRBM_GUI_ACTIVE"] / 8.0, simd_cycles))
        w("  SQ_INSTS_VALU %.4g (attributed %.4g, ratio %.4f); SQ_INSTS_SALU %.4g (attributed"
          " %.4g, ratio %.4f)" % (pm["SQ_INSTS_VALU"], valu, valu / pm["SQ_INSTS_VALU"],
                                  pm["SQ_INSTS_SALU"], dyn["salu"],
                                  dyn["salu"] / pm["SQ_INSTS_SALU"]))
        w("  SQ_ACTIVE_INST_VALU %.4g quad-cycles = %.4g cycles = %.3f of the SIMD cycles: the"
          % (pm["SQ_ACTIVE_INST_VALU"], 4 * pm["SQ_ACTIVE_INST_VALU"],
             4 * pm["SQ_ACTIVE_INST_VALU"] / simd_cycles))
        w("    counter gives one quad-cycle to each instruction of the fast and normal classes"
          " alike (microbenchmark: SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU = 1.00 for both, 2.00 for")
        w("    v_sqrt / v_rcp, 4.00 for v_rcp_f64), so it cannot tell the double-rate forms apart")
        w("  VALU cycles by the measured class costs: %.4g = %.3f of the SIMD cycles" % (
            valu_cyc, valu_cyc / simd_cycles))
        sa = pipe.get("salu", 0.0)
        w("  SALU cycles by the measured scalar cost: %.4g = %.3f of the SIMD cycles" % (
            sa, sa / simd_cycles))
        ref = 4 * (pm["SQ_ACTIVE_INST_VALU"] + pm["SQ_INSTS_SALU"])
        w("  class-weighted VALU + SALU = %.4g cycles against (SQ_ACTIVE_INST_VALU + SQ_INSTS_SALU)"
          " x 4 = %.4g: ratio %.4f" % (valu_cyc + sa, ref, (valu_cyc + sa) / ref))
        if "SQ_WAVE_CYCLES" in pm:
            w("  per wave: %.4g cycles alive; waiting on dependencies (SQ_WAIT_INST_ANY) %.3f,"
              " issuing (SQ_ACTIVE_INST_ANY) %.3f of its life" % (
                  4 * pm["SQ_WAVE_CYCLES"] / pm["SQ_WAVES"],
                  pm.get("SQ_WAIT_INST_ANY", 0) / pm["SQ_WAVE_CYCLES"],
                  pm.get("SQ_ACTIVE_INST_ANY", 0) / pm["SQ_WAVE_CYCLES"]))
    text = "\n".join(L)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
