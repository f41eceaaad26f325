"""Measured VALU attribution of the flat tracer kernel: the product code object's static VALU
instructions per counted region (tracer.hip reg::*) times the number of times a wave executed
that region in a stats-build frame of the same workload (VCRT_DEBUG_STATS=1: region counters in
vcrt_stats.debug[40..127]), against the product's SQ_INSTS_VALU of the same frame.

How an instruction gets its region: the -gline-tables-only build (identical instruction stream to
the product, checked) symbolizes every instruction with its inline chain; walking the chain from
the innermost frame out, the first tracer.hip line that lies inside the block of a region(...)
marker (innermost block wins) names the region; a marker whose region is relative to its call
site (rb + ... in the shading lambda and the big-list helpers) takes the base from the call
site's reg:: argument. Code inside no marker block belongs to the loop iteration (kIter), or to
the kernel's prologue / epilogue (once per wave). The stats build counts a region each time the
wave reaches its marker with some lane active; the hardware issues a VALU instruction whenever
the wave reaches it, even with no lane active when the compiler put no exec-skip branch around
it, so small unguarded blocks are under-counted: the comparison with SQ_INSTS_VALU bounds that.

  python tools/valu_regions.py --stats STATS.json --sq-valu TOTAL [--hsaco LT.hsaco]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import valu_attrib as V  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRACER = os.path.join(ROOT, "vulkancomputeraytracing_amd", "csrc", "tracer.hip")
REGION_DEBUG_BASE = 40
SIN3_FALLBACK = 0  # vcrt_math.h: sin3's fallback loop starts after this line


def enum_values(src):
    body = re.search(r"namespace reg \{\s*enum : uint32_t \{(.*?)\};", src, re.S).group(1)
    vals, nxt = {}, 0
    for tok in re.sub(r"//[^\n]*", "", body).replace("\n", " ").split(","):
        tok = tok.strip()
        if not tok:
            continue
        if "=" in tok:
            name, v = [t.strip() for t in tok.split("=")]
            nxt = int(v)
        else:
            name = tok
        vals[name] = nxt
        nxt += 1
    return vals


def blocks(lines):
    """For every region(...) marker: (line, expr, block_open, block_close) (1-based lines)."""
    text = "\n".join(lines)
    # brace positions -> line numbers
    line_of = []
    for i, ln in enumerate(lines):
        line_of.extend([i + 1] * (len(ln) + 1))
    stack, match = [], {}
    for pos, ch in enumerate(text):
        if ch == "{":
            stack.append(pos)
        elif ch == "}" and stack:
            match[stack.pop()] = pos
    opens = sorted(match)
    out = []
    for m in re.finditer(r"\bregion\(rrow, ([^;]*?)\);", text):
        if "void region(" in text[max(0, m.start() - 40):m.start()]:
            continue
        # the innermost block that holds the marker
        op = max((o for o in opens if o < m.start() and match[o] > m.start()), default=None)
        if op is None:
            continue
        out.append((line_of[m.start()], m.group(1).strip(), line_of[op], line_of[match[op]]))
    return out


# SQ_INSTS_SALU counts the scalar ALU instructions and the branches (checked: C4's attributed
# total is 0.97 of it with branches, 0.75 without), not memory, waits or nops
_NOT_SALU = ("s_load", "s_buffer_load", "s_store", "s_buffer_store", "s_waitcnt", "s_nop",
             "s_setprio", "s_barrier", "s_endpgm", "s_sleep", "s_memtime", "s_memrealtime",
             "s_dcache", "s_sendmsg", "s_trap", "s_icache", "s_atomic", "s_scratch")


def is_salu(mn):
    return mn.startswith("s_") and not mn.startswith(_NOT_SALU)


def assign_regions(hsaco, product, kernel):
    """Every instruction of `kernel` in the product code object with the region that holds it:
    ([(address, mnemonic, operands, region)], label(region) -> name). hsaco: the
    -gline-tables-only build (None: built by tools/mkab.sh lt)."""
    class A:
        pass
    a = A()
    a.hsaco, a.product, a.kernel = hsaco, product, kernel
    if a.hsaco is None:
        a.hsaco = subprocess.run(["bash", os.path.join(ROOT, "tools", "mkab.sh"), "lt"],
                                 env=dict(os.environ, EXTRA="-gline-tables-only"),
                                 capture_output=True, text=True, check=True).stdout.strip()
    src = open(TRACER).read()
    math_lines = open(os.path.join(os.path.dirname(TRACER), "vcrt_math.h")).read().split("\n")
    global SIN3_FALLBACK
    SIN3_FALLBACK = next(i + 1 for i, ln in enumerate(math_lines)
                         if "if (fell_back) *fell_back = !ok;" in ln)
    lines = src.split("\n")
    ev = enum_values(src)
    # the global regions, and the shading's offsets from its call site's base (kSh*)
    is_sh = lambda k: k.startswith("kSh") and not k.startswith("kShade")  # noqa: E731
    names = {v: k for k, v in ev.items() if not is_sh(k) and k != "kCount"}
    sh_names = {v: k for k, v in ev.items() if is_sh(k)}
    marks = blocks(lines)
    insts = V.disasm(a.hsaco, a.kernel)
    prod = V.disasm(a.product, a.kernel)
    same = V.normalized(insts) == V.normalized(prod)
    print(f"{a.kernel}: {len(insts)} instructions; line-table build identical to the product: {same}")
    if not same:
        sys.exit("the line-table build differs from the product code object")
    chains = V.symbolize(a.hsaco, [ad for ad, _, _ in insts])
    loop_line = next(i + 1 for i, ln in enumerate(lines) if ln.startswith("    for (;;) {")
                     and i > next(j for j, l2 in enumerate(lines) if "void trace_impl(" in l2))
    loop_end = next(i + 1 for i, ln in enumerate(lines) if "VCRT_WAVE_END_TIMES  // diagnostics" in ln)

    def reg_token(ln, span=3):
        """The last reg:: value named on source lines ln .. ln + span - 1 (a call site)."""
        toks = re.findall(r"reg::(k\w+)", " ".join(lines[ln - 1:ln - 1 + span]))
        return ev[toks[-1]] if toks else None

    def lam_base(chain):
        """The shading lambda's region base: the reg::kShadeBase* of its call site."""
        for f, fl, ln in chain:
            if fl == "tracer.hip" and "shade_and_advance(" in " ".join(lines[ln - 1:ln + 1]):
                b = reg_token(ln, 2)
                if b is not None and b >= ev["kShadeBase0"]:
                    return b
        return None

    def marker_at(ln):
        """The marker of the innermost block holding line ln (among markers of that block, the
        last one at or before ln), or None."""
        inside = [m for m in marks if m[2] <= ln <= m[3]]
        if not inside:
            return None
        op = max(m[2] for m in inside)
        same = sorted((m for m in inside if m[2] == op), key=lambda m: m[0])
        before = [m for m in same if m[0] <= ln]
        return before[-1] if before else same[0]

    def region_of(chain):
        fns = " | ".join(f for f, _, _ in chain)
        if any(k in fns for k in ("sin_canonical", "ksin", "kcos", "reduce_large")) or \
                any(fl == "vcrt_math.h" and "sin3" in f and ln >= SIN3_FALLBACK
                    for f, fl, ln in chain):
            b = lam_base(chain)
            if b is not None:
                return b + ev["kShSinFallback"]
        for k, (f, fl, ln) in enumerate(chain):
            if fl != "tracer.hip":
                continue
            m = marker_at(ln)
            if m is None:
                continue
            expr = m[1]
            if expr.startswith("reg::"):
                return ev[expr[5:]]
            mm = re.fullmatch(r"rb(?: \+ (?:reg::(k\w+)|(\d+)))?", expr)
            if not mm:
                raise ValueError(expr)
            off = ev[mm.group(1)] if mm.group(1) else int(mm.group(2) or 0)
            if "rb + reg::kSh" in expr or expr == "rb + reg::kShEntry":
                base = lam_base(chain)
            else:  # the big-list helpers: the call site's reg::kCamBig / kMainBig
                base = next((reg_token(ln2) for f2, fl2, ln2 in chain[k + 1:]
                             if fl2 == "tracer.hip" and reg_token(ln2) is not None), None)
            if base is None:
                raise ValueError(f"no call-site base for {expr} at line {ln}: {chain}")
            return base + off
        impl = [ln for f, fl, ln in chain if f.startswith("trace_impl") and fl == "tracer.hip"]
        if impl and loop_line <= impl[-1] < loop_end:
            return ev["kIter"]
        return -1  # prologue / epilogue: once per wave


    def label(r):
        if r < 0:
            return "prologue/epilogue"
        if r in names:
            return names[r]
        if ev["kShadeBase1"] <= r < ev["kShadeBase1"] + 16:
            return "shade(sky after scan)." + sh_names.get(r - ev["kShadeBase1"], "?")
        if ev["kShadeBase0"] <= r < ev["kShadeBase0"] + 16:
            return "shade(camera phase)." + sh_names.get(r - ev["kShadeBase0"], "?")
        return str(r)
    return [(ad, mn, ops, region_of(chains[ad])) for ad, mn, ops in insts], label, chains


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--hsaco", default=None)
    p.add_argument("--product", default=os.path.join(ROOT, "vulkancomputeraytracing_amd", "lib",
                                                     "vcrt_tracer.hsaco"))
    p.add_argument("--kernel", default="vcrt_trace_cull_flat")
    p.add_argument("--stats", required=True, help="stats-build render_once JSON (one frame)")
    p.add_argument("--sq-valu", type=float, required=True,
                   help="SQ_INSTS_VALU of the product frame (instructions, per dispatch)")
    p.add_argument("--json", default=None)
    p.add_argument("--kind", choices=("valu", "salu"), default="valu",
                   help="salu: scalar ALU and branch instructions (s_* but memory, waits, "
                        "nops), against SQ_INSTS_SALU given as --sq-valu")
    p.add_argument("--detail", action="append", default=[],
                   help="region name: also list its static VALU per innermost source line")
    a = p.parse_args()
    insts_r, label, chains = assign_regions(a.hsaco, a.product, a.kernel)
    static = collections.Counter()
    where = collections.defaultdict(collections.Counter)
    for ad, mn, _, r in insts_r:
        if (V.is_valu(mn) if a.kind == "valu" else is_salu(mn)):
            static[r] += 1
            f, fl, ln = chains[ad][0]
            where[r][(fl, ln, f.split("(")[0][:40])] += 1
    st = json.load(open(a.stats))
    st = st[-1] if isinstance(st, list) else st
    d = st["debug"]
    waves = d[7]
    total = 0.0
    rows = []
    for r, n in static.items():
        cnt = waves if r < 0 else d[REGION_DEBUG_BASE + r]
        dyn = n * cnt
        total += dyn
        rows.append((dyn, r, n, cnt))
    rows.sort(reverse=True)

    print(f"stats frame: {st['segments']} segments, {waves} waves, {d[0]} wave-iterations")
    K = a.kind.upper()
    print(f"{'dynamic ' + K:>14} {'share':>6} {'static':>6} {'entries':>12}  region")
    for dyn, r, n, cnt in rows:
        name = label(r)
        print(f"{dyn:14.4g} {100 * dyn / total:5.1f}% {n:6d} {cnt:12d}  {name}")
    for want in a.detail:
        for r in static:
            if label(r) == want:
                print(f"-- {want}: static {K} by innermost source line")
                for (fl, ln, f), n in sorted(where[r].items()):
                    print(f"   {n:4d}  {fl}:{ln}  {f}")
    print(f"attributed total {total:.4g} {K} instructions; SQ_INSTS_{K} {a.sq_valu:.4g}: "
          f"ratio {total / a.sq_valu:.4f}")
    if a.json:
        json.dump({"kernel": a.kernel, "attributed": total, "sq_insts_valu": a.sq_valu,
                   "ratio": total / a.sq_valu,
                   "regions": [{"region": label(r),
                                "index": r, "static": n, "entries": cnt, "dynamic": dyn}
                               for dyn, r, n, cnt in rows]},
                  open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
