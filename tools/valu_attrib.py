"""VALU attribution of the flat tracer kernel by phase (static instruction counts beside the
stats build's measured phase shares).

Static part: every instruction of a kernel in a line-table build of the code object
(-gline-tables-only, whose instruction stream this tool checks is identical to the product code
object's) is symbolized with its inline chain (llvm-symbolizer --inlining) and assigned to a
phase of trace_impl (camera fast trace: big list / listed spheres / roots; main scan: ray set-up,
big list, node level, passes by kind; shading: sines / normal and scatter / sky / next camera
ray; retire; fetch; loop control). Rare fallback code (the canonical sine, hipcc's full sqrt and
division sequences, the linear scan of unguarded waves) is listed under its own phase.

With --phases (the JSON of a stats-build frame, VCRT_DEBUG_STATS=1 tools/render_once.py: wave
clock per phase, pass and loop trip counts) and --sq-valu (SQ_INSTS_VALU per wave-segment of the
product at the same workload, profiles/traffic.json), it prints the measured time shares beside
the static counts. This is an estimate: PC sampling is not available on the GPU pool, and the
product kernel is not instrumented; the stats build's clocks include memory waits.

  python tools/valu_attrib.py --hsaco LINE_TABLE.hsaco [--kernel vcrt_trace_cull_flat]
      [--phases gpurun_out/phases.json] [--sq-valu 753.2]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRACER = os.path.join(ROOT, "vulkancomputeraytracing_amd", "csrc", "tracer.hip")


def disasm(hsaco, kernel):
    """[(address, mnemonic, text)] of one kernel."""
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", hsaco],
                         capture_output=True, text=True, check=True).stdout
    insts, cur = [], None
    for line in out.splitlines():
        m = re.match(r"^([0-9a-f]+) <(\w+)>:", line)
        if m:
            cur = m.group(2)
            continue
        if cur != kernel:
            continue
        m = re.match(r"^\s+(\S+)(.*?)//\s*([0-9A-F]+):", line)
        if m:
            insts.append((int(m.group(3), 16), m.group(1), (m.group(1) + m.group(2)).strip()))
    return insts


def normalized(insts):
    return [re.sub(r"0x[0-9a-f]+", "X", t) for _, _, t in insts]


def symbolize(hsaco, addrs):
    """address -> [(function, line)] innermost first."""
    inp = "\n".join(hex(a) for a in addrs) + "\n"
    out = subprocess.run([f"{LLVM}/llvm-symbolizer", f"--obj={hsaco}", "--inlining",
                          "--functions=linkage", "--demangle"], input=inp, capture_output=True,
                         text=True, check=True).stdout
    chains = []
    for block in out.strip("\n").split("\n\n"):
        lines = block.split("\n")
        frames = []
        for i in range(0, len(lines) - 1, 2):
            fn = lines[i]
            m = re.match(r"(.*):(\d+):(\d+)$", lines[i + 1])
            frames.append((fn, os.path.basename(m.group(1)) if m else "?",
                           int(m.group(2)) if m else 0))
        chains.append(frames)
    assert len(chains) == len(addrs), (len(chains), len(addrs))
    return dict(zip(addrs, chains))


def marker_lines():
    """tracer.hip line numbers of trace_impl's region markers (found by text, so the tool
    follows edits of the source)."""
    src = open(TRACER).read().split("\n")

    def find(text, start=0):
        for i in range(start, len(src)):
            if text in src[i]:
                return i + 1
        raise KeyError(text)
    m = {}
    m["impl"] = find("__device__ __forceinline__ void trace_impl(")
    m["lam"] = find("auto shade_and_advance", m["impl"])
    m["lam_sky"] = find("const float len = sqrt_fast(dot(d, d));", m["lam"])
    m["lam_end"] = find("if (ended) {", m["lam_sky"])
    m["loop"] = find("    for (;;) {", m["impl"])
    m["retire"] = find("// ---- retire the finished", m["loop"])
    m["fetch"] = find("// ---- lanes whose item is finished", m["retire"])
    m["cam"] = find("// ---- flat scan: a camera ray not yet traced", m["fetch"])
    m["cam_list"] = find("the quarter's listed spheres", m["cam"])
    m["cam_roots"] = find("...then the candidates' roots", m["cam_list"])
    m["cam_tally"] = find("issued work: the big list and the loop's passes", m["cam_roots"])
    m["cam_shade"] = find("One shading for the camera rays", m["cam_tally"])
    m["scan"] = find("// ---- one segment: scan the whole sphere list", m["cam_shade"])
    m["shade"] = find("// ---- shade (textures.glsl)", m["scan"])
    m["end"] = find("VCRT_WAVE_END_TIMES", m["shade"])
    # the real branches of the rare fallbacks (asm volatile(""): not if-converted)
    m["rare"] = {find("const float full = __builtin_sqrtf(x);"),
                 find("const float full = __builtin_sqrtf(disc);"),
                 find("normal = divs(pcv, cr.w);")}
    return m


def phase(chain, mk):
    """The phase of one instruction from its inline chain (innermost first)."""
    fns = [f for f, _, _ in chain]
    text = " | ".join(fns)
    if any(k in text for k in ("sin_canonical", "ksin", "kcos", "reduce_large")):
        return "rare: canonical sine (fallback of the fast sine)"
    if any(fl == "tracer.hip" and ln in mk["rare"] for _, fl, ln in chain):
        return "rare: full sqrt / division (fallbacks)"
    impl = [(f, fl, ln) for f, fl, ln in chain if f.startswith("trace_impl")]
    line = impl[0][2] if impl else 0
    # shade_and_advance (its body lies between its definition and the loop; the other lambda,
    # pixel_corner, counts where it is called)
    lam = [ln for f, _, ln in chain if f == "operator()" and mk["lam"] <= ln < mk["loop"]]
    if lam:  # shade_and_advance (the lambda)
        if any(k in text for k in ("sin3", "sin_fast_try")):
            return "shading: the three sines (fast path)"
        ln = lam[0]
        if mk["lam_sky"] <= ln < mk["lam_end"]:
            return "shading: sky"
        if ln >= mk["lam_end"]:
            return "shading: sample end, next camera ray"
        return "shading: normal, scatter"
    if "flat_pass<0" in text:
        return "scan: candidate passes"
    if "flat_pass<1" in text:
        return "scan: group passes"
    if "flat_pass<2" in text:
        return "scan: node passes"
    if "flat_pass<3" in text:
        return "scan: chunk passes"
    if "flat_drain" in text:
        return "scan: pass selection"
    if "scan_culled_flat" in text:
        if "exact_group_uniform" in text:
            return "scan: big list"
        if "box_ray" in text or "recip_a" in text:
            return "scan: ray set-up (box ray)"
        if "push_bound_pair_nf" in text or "near_far_addr" in text:
            return "scan: node level (chunk's 8 node boxes)"
        return "scan: set-up, lists, pushes, key"
    if "scan_spheres" in text:
        return "rare: linear scan (waves outside the guarded range)"
    if not impl:
        return "other"
    if "exact_group_uniform_cam" in text:
        return "camera: big list"
    if mk["cam_list"] <= line < mk["cam_roots"]:
        return "camera: listed spheres"
    if mk["cam_roots"] <= line < mk["cam_tally"]:
        return "camera: candidate roots"
    if mk["cam"] <= line < mk["cam_shade"]:
        return "camera: set-up and tallies"
    if mk["retire"] <= line < mk["fetch"]:
        return "retire (quantize, ring add)"
    if mk["fetch"] <= line < mk["cam"]:
        return "fetch (blocks, slots, first camera ray)"
    if mk["cam_shade"] <= line < mk["scan"]:
        return "shading: hand-over (pending hits)"
    if mk["scan"] <= line < mk["shade"]:
        return "scan: guard, dispatch"
    if mk["shade"] <= line < mk["end"]:
        return "shading: hand-over (pending hits)"
    if mk["loop"] <= line:
        return "loop control"
    return "kernel prologue / epilogue"


def is_valu(mn):
    return mn.startswith("v_")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--hsaco", default=None, help="-gline-tables-only build of tracer.hip "
                   "(default: built now from the current source into ab_objs/lt.hsaco)")
    p.add_argument("--product", default=os.path.join(ROOT, "vulkancomputeraytracing_amd", "lib",
                                                     "vcrt_tracer.hsaco"))
    p.add_argument("--kernel", default="vcrt_trace_cull_flat")
    p.add_argument("--phases", default=None)
    p.add_argument("--sq-valu", type=float, default=None)
    p.add_argument("--json", default=None)
    a = p.parse_args()
    if a.hsaco is None:  # the line tables must come from the source the markers are read from
        a.hsaco = subprocess.run(["bash", os.path.join(ROOT, "tools", "mkab.sh"), "lt"],
                                 env=dict(os.environ, EXTRA="-gline-tables-only"),
                                 capture_output=True, text=True, check=True).stdout.strip()
    insts = disasm(a.hsaco, a.kernel)
    prod = disasm(a.product, a.kernel)
    same = normalized(insts) == normalized(prod)
    print(f"{a.kernel}: {len(insts)} instructions, line-table build identical to the product: "
          f"{same}")
    if not same:
        sys.exit("the line-table build differs from the product code object")
    mk = marker_lines()
    chains = symbolize(a.hsaco, [ad for ad, _, _ in insts])
    static = collections.Counter()
    ph_of = {}
    for ad, mn, _ in insts:
        ph = phase(chains[ad], mk)
        ph_of[ad] = ph
        if is_valu(mn):
            static[ph] += 1
    res = {"kernel": a.kernel, "instructions": len(insts),
           "static_valu": dict(static.most_common())}
    print("static VALU instructions by phase:")
    for ph, n in static.most_common():
        print(f"  {n:5d}  {ph}")
    if a.phases:
        st = json.load(open(a.phases))
        d = st["debug"]
        wi, tot = d[0], d[14]
        shares = [("camera fast trace (shading excluded)", d[23] - d[3]),
                  ("camera-phase shading", d[3]), ("main scan: big list", d[15]),
                  ("main scan: node level", d[9]), ("main scan: node pushes", d[16]),
                  ("main scan: node passes", d[10]), ("main scan: group passes", d[11]),
                  ("main scan: candidate passes", d[12]),
                  ("main scan: rest (ray set-up, lists, key, drain)",
                   d[8] - d[15] - d[9] - d[16] - d[10] - d[11] - d[12]),
                  ("main-scan sky shading", d[17]), ("fetch", d[18])]
        rest = tot - sum(v for _, v in shares)
        shares.append(("loop, retire, hand-over", rest))
        print(f"stats build: {wi} wave-iterations, {st['segments']} segments, "
              f"{st['segments'] / 64 / wi:.2f} wave-segments per wave-iteration")
        print("measured wave-time shares (stats build, s_memtime per phase):")
        res["time_share"] = {}
        for name, v in shares:
            print(f"  {100.0 * v / tot:5.1f}%  {name}")
            res["time_share"][name] = v / tot
        res["wave_iterations"] = wi
        res["segments"] = st["segments"]
        if a.sq_valu:
            per_iter = a.sq_valu * st["segments"] / 64 / wi
            print(f"product VALU per wave-iteration (SQ_INSTS_VALU {a.sq_valu} per wave-segment): "
                  f"{per_iter:.0f}; by time share:")
            for name, v in shares:
                print(f"  {per_iter * v / tot:6.0f}  {name}")
            res["valu_per_iteration"] = per_iter
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
