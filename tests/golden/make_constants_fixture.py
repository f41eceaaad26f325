"""Regenerates tests/golden/reference_constants.json: the reference's configuration constants and
the shader literals the hot path uses, parsed as DATA from the reference files themselves.

Run in the build container (it reads /root/reference, which the GPU box does not have):
    python tests/golden/make_constants_fixture.py

Parsed (file:line as of the reference commit the survey studied; the parser finds them by
pattern, not by line number, and records the line each came from):
  shaders/include/globals.glsl:9-26   SAMPLES_PER_PIXEL (the `#if 0` resolved: its #else branch,
                                      1), MAX_RECURSION_LEVEL, IMAGE_WIDTH/HEIGHT, the camera
                                      (lookfrom, lookat, vup, vfov) and `infinity` (max_t)
  include/Common.hpp:23-25            WINDOW_WIDTH/HEIGHT (the dispatch size), RENDER_ITERATION
  shaders/include/functions.glsl:11   rand's dot coefficients and scale
  shaders/include/functions.glsl:76   min_t
  shaders/include/functions.glsl:87-88 the sky blend: 0.5 * (y + 1.0), mix(vec3(1), vec3(.5,.7,1))
  shaders/shader.comp:48              the jitter offset -0.5
  shaders/shader.comp:14              the 16x16 workgroup (the dispatch truncation)
Numeric literals are converted with C strtof, as a GLSL fp32 literal converts; each float is
stored with its IEEE bit pattern so tests compare bits.
"""
import ctypes
import json
import os
import re
import struct

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("VCRT_REFERENCE", "/root/reference")

_libc = ctypes.CDLL(None)
_libc.strtof.restype = ctypes.c_float
_libc.strtof.argtypes = [ctypes.c_char_p, ctypes.c_void_p]

NUM = r"[-+]?(?:[0-9]+\.?[0-9]*|\.[0-9]+)(?:[eE][-+]?[0-9]+)?"


def f32(text):
    t = text.strip()
    if not re.fullmatch(NUM, t):
        raise ValueError(f"not a numeric literal: {t!r}")
    return float(_libc.strtof(t.encode(), None))


def bits(x):
    return "0x%08x" % struct.unpack("<I", struct.pack("<f", x))[0]


def entry(values, path, line):
    vals = values if isinstance(values, list) else [values]
    return {"value": vals if isinstance(values, list) else vals[0],
            "f32_bits": [bits(v) for v in vals] if isinstance(values, list) else bits(vals[0]),
            "source": f"{path}:{line}"}


def active_lines(path):
    """(line number, text) of the lines a C/GLSL preprocessor keeps, for `#if 0` / `#if 1` /
    `#else` / `#endif` (all this file uses); other directives pass through."""
    keep = [True]
    out = []
    for i, text in enumerate(open(os.path.join(REF, path)), 1):
        s = text.strip()
        m = re.match(r"#\s*if\s+(\d+)\s*$", s)
        if m:
            keep.append(keep[-1] and m.group(1) != "0")
            continue
        if re.match(r"#\s*(if|ifdef|ifndef)\b", s):  # guards, platform switches: both kept
            keep.append(keep[-1])
            continue
        if re.match(r"#\s*else\b", s):
            parent = keep[-2] if len(keep) > 1 else True
            keep[-1] = parent and not keep[-1]
            continue
        if re.match(r"#\s*endif\b", s):
            keep.pop()
            continue
        if keep[-1]:
            out.append((i, text.split("//")[0]))
    return out


def find(lines, pattern, path):
    hits = [(i, m) for i, t in lines for m in [re.search(pattern, t)] if m]
    if len(hits) != 1:
        raise ValueError(f"{path}: {len(hits)} matches of {pattern!r}")
    return hits[0]


def main():
    c = {}
    g = "shaders/include/globals.glsl"
    gl = active_lines(g)
    for name in ("SAMPLES_PER_PIXEL", "MAX_RECURSION_LEVEL", "IMAGE_WIDTH", "IMAGE_HEIGHT"):
        i, m = find(gl, r"#\s*define\s+%s\s+(\d+)\s*$" % name, g)
        c[name] = {"value": int(m.group(1)), "source": f"{g}:{i}"}
    for name in ("lookfrom", "lookat", "vup"):
        i, m = find(gl, r"vec3\s+camera_%s\s*=\s*vec3\(([^)]*)\)" % name, g)
        c["camera_" + name] = entry([f32(v) for v in m.group(1).split(",")], g, i)
    i, m = find(gl, r"float\s+camera_vfov\s*=\s*(%s)\s*;" % NUM, g)
    c["camera_vfov"] = entry(f32(m.group(1)), g, i)
    i, m = find(gl, r"const\s+float\s+infinity\s*=\s*(%s)\s*;" % NUM, g)
    c["infinity"] = entry(f32(m.group(1)), g, i)

    h = "include/Common.hpp"
    hl = active_lines(h)
    for name in ("WINDOW_WIDTH", "WINDOW_HEIGHT", "RENDER_ITERATION"):
        i, m = find(hl, r"constexpr\s+auto\s+%s\s*=\s*(\d+)\s*;" % name, h)
        c[name] = {"value": int(m.group(1)), "source": f"{h}:{i}"}

    f = "shaders/include/functions.glsl"
    fl = active_lines(f)
    i, m = find(fl, r"fract\(sin\(dot\(co\.xy\s*,\s*vec2\((%s)\s*,\s*(%s)\)\)\)\s*\*\s*(%s)\)"
                % (NUM, NUM, NUM), f)
    c["rand_dot"] = entry([f32(m.group(1)), f32(m.group(2))], f, i)
    c["rand_scale"] = entry(f32(m.group(3)), f, i)
    i, m = find(fl, r"global_hit_record\.min_t\s*=\s*(%s)\s*;" % NUM, f)
    c["min_t"] = entry(f32(m.group(1)), f, i)
    at = [i for i, t in fl if re.search(r"global_hit_record\.max_t\s*=\s*infinity\s*;\s*$", t)]
    assert at, "max_t = infinity"  # before the bounce loop and again every pass
    c["max_t_is_infinity"] = {"value": True, "source": ", ".join(f"{f}:{i}" for i in at)}
    i, m = find(fl, r"float\s+a\s*=\s*(%s)\s*\*\s*\(unit_direction\.y\s*\+\s*(%s)\)\s*;" % (NUM, NUM), f)
    c["sky_blend"] = entry([f32(m.group(1)), f32(m.group(2))], f, i)
    i, m = find(fl, r"mix\(vec3\(([^)]*)\)\s*,\s*vec3\(([^)]*)\)\s*,\s*a\)", f)
    lo = [f32(v) for v in m.group(1).split(",")]
    c["sky_bottom"] = entry(lo * 3 if len(lo) == 1 else lo, f, i)  # vec3(1) splats
    c["sky_top"] = entry([f32(v) for v in m.group(2).split(",")], f, i)

    s = "shaders/shader.comp"
    sl = active_lines(s)
    i, m = find(sl, r"\((%s)\+rand\(vec2\(i,i\)\)\)\*pixel_delta_u\s*\+\s*\((%s)\+rand\(vec2\(i\+1,i\+1\)\)\)"
                % (NUM, NUM), s)
    c["jitter_offset"] = entry([f32(m.group(1)), f32(m.group(2))], s, i)
    i, m = find(sl, r"local_size_x\s*=\s*(\d+)\s*,\s*local_size_y\s*=\s*(\d+)", s)
    c["local_size"] = {"value": [int(m.group(1)), int(m.group(2))], "source": f"{s}:{i}"}

    out = {"reference": "fhh200000/VulkanComputeRayTracing (/root/reference)",
           "literal_parse": "C strtof (GLSL fp32 literal); f32_bits = IEEE-754 binary32",
           "constants": c}
    with open(os.path.join(HERE, "reference_constants.json"), "w") as fh:
        json.dump(out, fh, indent=1)
        fh.write("\n")
    print("wrote", len(c), "constants")


if __name__ == "__main__":
    main()
