"""Regenerates tests/golden/world_globals_glsl.{npy,json}: the reference's compile-time scene
table `const sphere world[]` (shaders/include/globals.glsl:29-518), parsed as DATA.

Run in the build container (it reads /root/reference, which the GPU box does not have):
    python tests/golden/make_world_fixture.py

Every `sphere(vec3(cx,cy,cz), r, vec3(R,G,B), vec3(TEXTURE_*, param, z))` initializer of the
array, in source order, becomes one float32 row [cx, cy, cz, r, R, G, B, material id, param, z]
(the field order of structures.glsl:10-16). Numeric literals are parsed with C strtof, as a GLSL
fp32 literal converts; TEXTURE_* take the values of textures.glsl:10-12. That covers the 481
SceneGenerator lines (globals.glsl:31-511), the three big spheres (:513-515) and the hand-added
ground (:517), so the whole table -- values and order (ties go to the lower index,
functions.glsl:27-29, 77) -- is pinned against the reference file itself, not a restatement.
The JSON records the source lines each row came from and a SHA-256 of the table.
"""
import ctypes
import hashlib
import json
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("VCRT_REFERENCE", "/root/reference")
GLOBALS = os.path.join(REF, "shaders", "include", "globals.glsl")
TEXTURES = os.path.join(REF, "shaders", "include", "textures.glsl")

SPHERE = re.compile(r"sphere\(\s*vec3\(([^)]*)\)\s*,\s*([^,]+?)\s*,\s*vec3\(([^)]*)\)\s*,\s*"
                    r"vec3\(([^)]*)\)\s*\)")

_libc = ctypes.CDLL(None)
_libc.strtof.restype = ctypes.c_float
_libc.strtof.argtypes = [ctypes.c_char_p, ctypes.c_void_p]


def f32(text: str) -> float:
    t = text.strip()
    if not re.fullmatch(r"[-+]?[0-9]*\.?[0-9]+(e[-+]?[0-9]+)?", t):
        raise ValueError(f"not a numeric literal: {t!r}")
    return _libc.strtof(t.encode(), None)


def texture_ids(path: str) -> dict:
    ids = {}
    for line in open(path):
        m = re.match(r"\s*#define\s+(TEXTURE_\w+)\s+(\d+)\s*$", line)
        if m:
            ids[m.group(1)] = float(m.group(2))
    return ids


def parse_world(path: str, ids: dict):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.search(r"const\s+sphere\s+world\[\]", l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith("};"))
    rows, where = [], []
    for i in range(start, end + 1):
        line = lines[i].split("//")[0]
        for m in SPHERE.finditer(line):
            c = [f32(v) for v in m.group(1).split(",")]
            col = [f32(v) for v in m.group(3).split(",")]
            tex = [v.strip() for v in m.group(4).split(",")]
            mat = ids[tex[0]] if tex[0] in ids else f32(tex[0])
            row = c + [f32(m.group(2))] + col + [mat, f32(tex[1]), f32(tex[2])]
            assert len(row) == 10, (i + 1, line)
            rows.append(row)
            where.append(i + 1)
    return np.array(rows, dtype=np.float32), (start + 1, end + 1), where


def main():
    ids = texture_ids(TEXTURES)
    assert ids == {"TEXTURE_LAMBERTIAN": 1.0, "TEXTURE_METAL": 2.0, "TEXTURE_GLASS": 3.0}, ids
    table, span, where = parse_world(GLOBALS, ids)
    np.save(os.path.join(HERE, "world_globals_glsl.npy"), table)
    meta = {
        "source": "shaders/include/globals.glsl (reference), const sphere world[]",
        "array_lines": list(span),
        "rows": int(len(table)),
        "row_source_lines": {"first": where[0], "generated_last": where[480],
                             "big_three": where[481:484], "ground": where[484]}
        if len(where) == 485 else where,
        "columns": ["cx", "cy", "cz", "radius", "r", "g", "b", "material", "param", "z"],
        "materials": ids,
        "literal_parse": "C strtof (GLSL fp32 literal)",
        "table_sha256": hashlib.sha256(table.tobytes()).hexdigest(),
    }
    with open(os.path.join(HERE, "world_globals_glsl.json"), "w") as f:
        json.dump(meta, f, indent=1)
        f.write("\n")
    print("wrote world fixture:", meta["rows"], "rows from lines", span)


if __name__ == "__main__":
    main()
