"""Regenerates the committed fixtures in tests/golden/ (run in the build container).

1. scene_generator.*: output of the REFERENCE's own SceneGenerator.cpp, compiled from
   /root/reference by oracle/Makefile into oracle/_ref/SceneGenerator (never copied).
   Stored as data, not text: the SHA-256 + length of its stdout and the parsed sphere table
   (float32 [481, 10]: center xyz, radius, colour rgb, material id, param, 0), where each
   printed decimal is parsed with C strtof exactly as a GLSL fp32 literal.
2. oracle_images.npz: small renders of the CPU oracle (oracle/vcrt_oracle.c), pinning the
   oracle against regressions and giving the GPU tests fixed expected images.

Usage: python tests/golden/make_golden.py
"""
import ctypes
import hashlib
import json
import os
import re
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from tests import oracle_py  # noqa: E402

MATERIALS = {"TEXTURE_LAMBERTIAN": 1, "TEXTURE_METAL": 2, "TEXTURE_GLASS": 3}
LINE = re.compile(r"sphere\(vec3\(([^)]*)\),\s*([-0-9.]+),\s*vec3\(([^)]*)\),\s*"
                  r"vec3\((TEXTURE_\w+),([^,]+),([^)]+)\)\),")

_libc = ctypes.CDLL(None)
_libc.strtof.restype = ctypes.c_float
_libc.strtof.argtypes = [ctypes.c_char_p, ctypes.c_void_p]


def f32(text: str) -> float:
    return _libc.strtof(text.strip().encode(), None)


def parse_spheres(text: str) -> np.ndarray:
    rows = []
    for m in LINE.finditer(text):
        c = [f32(v) for v in m.group(1).split(",")]
        col = [f32(v) for v in m.group(3).split(",")]
        rows.append(c + [f32(m.group(2))] + col +
                    [float(MATERIALS[m.group(4)]), f32(m.group(5)), f32(m.group(6))])
    return np.array(rows, dtype=np.float32)


# Small oracle renders: (name, scene, width, height, spp, depth)
IMAGES = [
    ("red_64x36_s1_d1", "red", 64, 36, 1, 1),
    ("three_80x45_s4_d8", "three", 80, 45, 4, 8),
    ("final_48x27_s2_d10", "final", 48, 27, 2, 10),
]


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all", "ref"], check=True)
    out = subprocess.run([oracle_py.REF_SCENEGEN], capture_output=True, check=True).stdout
    generated = out.split(b"\n\n")[0].decode()  # the 481 generated lines
    spheres = parse_spheres(generated)
    np.save(os.path.join(HERE, "scene_generator_spheres.npy"), spheres)
    meta = {"sha256": hashlib.sha256(out).hexdigest(), "bytes": len(out),
            "generated_spheres": int(len(spheres)),
            "source": "reference SceneGenerator.cpp compiled with g++ -O2 -std=c++20"}
    with open(os.path.join(HERE, "scene_generator_stdout.json"), "w") as f:
        json.dump(meta, f, indent=1)
        f.write("\n")

    o = oracle_py.load()
    images = {}
    for name, scene, w, h, spp, depth in IMAGES:
        img, segs = o.render(o.config(w, h, spp, depth), o.scene(scene))
        images[name] = img
        images[name + "__segments"] = np.array([segs], dtype=np.uint64)
    np.savez_compressed(os.path.join(HERE, "oracle_images.npz"), **images)
    print("wrote fixtures:", meta, list(images))


if __name__ == "__main__":
    main()
