"""Cycle attribution of the flat tracer kernel (verdict r05 item 2): the measured instruction
attribution (tools/valu_regions.py: every instruction of the product code object in its counted
region x the region's entries in a stats frame of the same workload) weighted by the issue cost
of each instruction's class, measured by tools/microbench_classes.hip on the same GPU.

Per class two costs, both relative to v_mul_f32 (one quad-cycle of a SIMD's VALU per wave
instruction):
  pipe   -- the SIMD's VALU throughput cost (8 waves per SIMD, independent chains), and the
            counter's own weighting SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU of the form (PMC run);
  issue  -- one wave's issue interval (1 wave per SIMD), i.e. what the form costs the wave's own
            instruction stream (SALU included: a scalar instruction takes the wave's issue slot).
The weighted sums are compared with the product frame's SQ_ACTIVE_INST_VALU (+ the SALU issue,
SQ_INSTS_SALU) and with the SIMDs' quad-cycles in the frame (1024 SIMDs x GRBM_GUI_ACTIVE / 4 ...).

  python tools/cycle_attrib.py --stats STATS.json --micro MICRO.json [--micro-pmc CSV]
                               [--pmc PMC.json] [--out profiles/r06_cycle_attrib.txt]
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

CLASSES = [  # (class, pattern on the full mnemonic, encoding suffix included), first match wins
    ("dpp", r".*_dpp$"),
    ("sdwa", r".*_sdwa$"),
    ("packed", r"^v_pk_"),
    ("trans64", r"^v_(rcp|sqrt|rsq)_f64"),
    ("trans", r"^v_(sqrt|rcp|rsq|rcp_iflag|exp|log|sin|cos)_f32"),
    ("div", r"^v_div_(scale|fmas|fixup)_f(32|64)"),
    ("cvt64", r"^v_cvt_.*f64|^v_cvt_f64"),
    ("f64", r"^v_.*_f64"),
    ("mul32", r"^v_(mul_lo_u32|mul_hi_u32|mul_hi_i32|mad_u64_u32|mad_i64_i32|mul_lo_i32)"),
    ("int64", r"^v_(lshl_add_u64|lshlrev_b64|lshrrev_b64|ashrrev_i64|mov_b64)"),
    ("lane", r"^v_(readlane|readfirstlane|writelane)_b32"),
    ("cndmask_vcc", r"^v_cndmask_b32_e32$"),
    ("cndmask_sgpr", r"^v_cndmask_b32_e64$"),
    ("cmp", r"^v_cmpx?_"),
    ("vop2", r"^v_.*_e32$"),   # VOP1 / VOP2 encodings (4-byte, no modifiers)
    ("vop3", r"^v_"),          # VOP3 encodings (8-byte: _e64 and VOP3-only forms)
]
# the microbenchmark form that stands for each class
FORM = {"vop2": "v_mul_f32", "vop3": "v_fma_f32", "cmp": "v_cmp_lt_f32",
        "cndmask_vcc": "v_cndmask_b32", "cndmask_sgpr": "v_cndmask_b32_e64_sgpr",
        "packed": "v_pk_fma_f32", "f64": "v_fma_f64", "cvt64": "v_cvt_f64_f32",
        "trans": "v_sqrt_f32", "trans64": "v_rcp_f64", "div": "v_div_scale_f32",
        "mul32": "v_mul_lo_u32", "int64": "v_lshl_add_u64", "lane": "v_readfirstlane_b32",
        "dpp": "v_add_u32_dpp", "sdwa": "v_fma_f32", "salu": "s_add_u32"}


def klass(mn):
    if R.is_salu(mn):
        return "salu"
    if not V.is_valu(mn):
        return None
    for c, pat in CLASSES:
        if re.match(pat, mn):
            return c
    return None


def micro_costs(micro, micro_pmc):
    forms = {f["form"]: f for f in micro["forms"]}
    ref = forms["v_mul_f32"]
    out = {}
    for f, d in forms.items():
        out[f] = {"pipe": d["ms_8waves"] / ref["ms_8waves"], "issue": d["ms_1wave"] / ref["ms_1wave"]}
    # the counter's own weighting: SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU per form (per dispatch)
    if micro_pmc:
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        for path in micro_pmc:
            for row in csv.DictReader(open(path)):
                k = row["Kernel_Name"].split("(")[0].strip()
                acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
        kname = {"v_mul_f32": "k_mul", "v_fma_f32": "k_fma", "v_mov_b32": "k_mov",
                 "v_cndmask_b32": "k_cnd", "v_add_u32": "k_addu", "v_max3_f32": "k_max3",
                 "v_cmp_lt_f32": "k_cmp", "v_sqrt_f32": "k_sqrt", "v_rcp_f32": "k_rcp",
                 "v_div_scale_f32": "k_dsc", "v_div_fmas_f32": "k_dfm",
                 "v_div_fixup_f32": "k_dfx", "v_mul_lo_u32": "k_mullo",
                 "v_mul_hi_u32": "k_mulhi", "v_add_u32_dpp": "k_dpp",
                 "v_mbcnt_lo_u32_b32": "k_mbcnt", "v_bfe_u32": "k_bfe", "v_fma_f64": "k_fma64",
                 "v_mul_f64": "k_mul64", "v_add_f64": "k_add64", "v_lshl_add_u64": "k_lshl64",
                 "v_rcp_f64": "k_rcp64", "v_pk_fma_f32": "k_pkfma", "v_pk_mul_f32": "k_pkmul",
                 "v_pk_add_f32": "k_pkadd", "v_cvt_f64_f32": "k_cvt64",
                 "v_readfirstlane_b32": "k_rfl", "s_add_u32": "k_salu", "mix_v_mul_s_add": "k_mix",
                 "v_fmac_f32": "k_fmac", "v_max_f32": "k_max", "v_and_b32": "k_and",
                 "v_lshlrev_b32": "k_lshl", "v_alignbit_b32": "k_align",
                 "v_mul_f32_e64": "k_mule64", "v_sub_f32": "k_sub",
                 "v_cndmask_b32_e64_sgpr": "k_cnds", "v_mul_f32_sgpr": "k_muls"}
        for f, k in kname.items():
            c = acc.get(k)
            if f in out and c and c.get("SQ_INSTS_VALU"):
                out[f]["counter_qc"] = c.get("SQ_ACTIVE_INST_VALU", 0) / c["SQ_INSTS_VALU"]
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--stats", required=True, help="stats-build render_once JSON (region counts)")
    p.add_argument("--micro", required=True, help="tools/microbench_classes JSON")
    p.add_argument("--micro-pmc", action="append", default=[],
                   help="rocprofv3 counter_collection.csv of the microbenchmark (any number)")
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

    costs = micro_costs(json.load(open(a.micro)), a.micro_pmc)
    dyn = collections.Counter()      # class -> dynamic wave-instructions
    mnem = collections.Counter()     # mnemonic -> dynamic wave-instructions
    reg_dyn = collections.defaultdict(collections.Counter)  # region -> class -> dynamic
    for _, mn, _, r in insts:
        c = klass(mn)
        if c is None:
            continue
        n = entries(r)
        dyn[c] += n
        mnem[mn] += n
        reg_dyn[r][c] += n
    lines = []
    out = lines.append
    out("Cycle attribution of %s (tools/cycle_attrib.py)" % a.kernel)
    out("stats frame: %d segments, %d wave-iterations" % (st["segments"], d[0]))
    out("")
    out("Issue costs per class (tools/microbench_classes.hip, relative to v_mul_f32):")
    out("  %-8s %-20s %6s %6s %8s" % ("class", "form", "pipe", "issue", "counter"))
    for c in sorted(dyn, key=lambda c: -dyn[c]):
        f = FORM[c]
        k = costs.get(f, {})
        out("  %-8s %-20s %6.2f %6.2f %8s" % (c, f, k.get("pipe", float("nan")),
                                             k.get("issue", float("nan")),
                                             "%.2f" % k["counter_qc"] if "counter_qc" in k
                                             else "-"))
    for f in ("v_mov_b32", "v_add_u32", "v_fmac_f32", "v_max_f32", "v_and_b32", "v_lshlrev_b32",
              "v_sub_f32", "v_mul_f32_sgpr", "v_mul_f32_e64", "v_max3_f32", "v_alignbit_b32",
              "v_rcp_f32", "v_div_fmas_f32", "v_div_fixup_f32", "v_mul_hi_u32",
              "v_mbcnt_lo_u32_b32", "v_bfe_u32", "v_mul_f64", "v_add_f64", "v_pk_mul_f32",
              "v_pk_add_f32", "mix_v_mul_s_add"):
        if f in costs:
            k = costs[f]
            out("  %-8s %-20s %6.2f %6.2f %8s" % ("", f, k["pipe"], k["issue"],
                                                 "%.2f" % k["counter_qc"] if "counter_qc" in k
                                                 else "-"))
    out("")
    tot_i = sum(v for c, v in dyn.items() if c != "salu")
    tot_pipe = sum(v * costs[FORM[c]]["pipe"] for c, v in dyn.items() if c != "salu")
    tot_cnt = sum(v * costs[FORM[c]].get("counter_qc", costs[FORM[c]]["pipe"])
                  for c, v in dyn.items() if c != "salu")
    tot_issue = sum(v * costs[FORM[c]]["issue"] for c, v in dyn.items())
    out("Dynamic mix of the frame (wave-instructions, from the attribution):")
    out("  %-8s %14s %7s %16s %7s %16s %7s" % ("class", "instructions", "share", "pipe qcycles",
                                              "share", "issue slots", "share"))
    for c in sorted(dyn, key=lambda c: -dyn[c]):
        v = dyn[c]
        pc = 0.0 if c == "salu" else v * costs[FORM[c]]["pipe"]
        ic = v * costs[FORM[c]]["issue"]
        out("  %-8s %14.4g %6.1f%% %16.4g %6.1f%% %16.4g %6.1f%%" % (
            c, v, 100 * v / (tot_i + dyn["salu"]), pc, 100 * pc / tot_pipe, ic,
            100 * ic / tot_issue))
    out("  VALU total %.4g wave-instructions; pipe-weighted %.4g quad-cycles (x%.3f); "
        "counter-weighted %.4g; issue-weighted incl. SALU %.4g slots" % (
            tot_i, tot_pipe, tot_pipe / tot_i, tot_cnt, tot_issue))
    out("")
    out("The most frequent mnemonics (dynamic):")
    for m, v in mnem.most_common(25):
        out("  %14.4g  %s" % (v, m))
    out("")
    out("Regions by issue-weighted slots (VALU by class cost + SALU):")
    rows = []
    for r, cc in reg_dyn.items():
        slots = sum(v * costs[FORM[c]]["issue"] for c, v in cc.items())
        pipe = sum(v * costs[FORM[c]]["pipe"] for c, v in cc.items() if c != "salu")
        rows.append((slots, pipe, r, cc))
    rows.sort(reverse=True)
    for slots, pipe, r, cc in rows[:30]:
        top = ", ".join("%s %.3g" % (c, v) for c, v in cc.most_common(4))
        out("  %12.4g %5.1f%%  pipe %12.4g  %-34s %s" % (slots, 100 * slots / tot_issue, pipe,
                                                     label(r), top))
    if a.pmc:
        pm = json.load(open(a.pmc))
        out("")
        out("Against the product frame's counters (%s):" % a.pmc)
        for k in sorted(pm):
            out("  %-22s %.4g" % (k, pm[k]))
        if "SQ_INSTS_VALU" in pm:
            out("  attributed VALU / SQ_INSTS_VALU = %.4f" % (tot_i / pm["SQ_INSTS_VALU"]))
        if "SQ_ACTIVE_INST_VALU" in pm:
            out("  pipe-weighted / SQ_ACTIVE_INST_VALU = %.4f; counter-weighted / "
                "SQ_ACTIVE_INST_VALU = %.4f" % (tot_pipe / pm["SQ_ACTIVE_INST_VALU"],
                                                tot_cnt / pm["SQ_ACTIVE_INST_VALU"]))
        if "SQ_ACTIVE_INST_VALU" in pm and "SQ_INSTS_SALU" in pm:
            out("  issue-weighted (VALU + SALU) / (SQ_ACTIVE_INST_VALU + SQ_INSTS_SALU) = %.4f" %
                (tot_issue / (pm["SQ_ACTIVE_INST_VALU"] + pm["SQ_INSTS_SALU"])))
    text = "\n".join(lines)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
