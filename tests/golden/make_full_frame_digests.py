"""Whole-frame oracle digests of the BASELINE configs C3 and C4 (and full-width rows of C5).

Runs the CPU oracle (oracle/vcrt_oracle.c, a linear scan restating shader.comp:42-57 and
functions.glsl:65-92 over every pixel) in THIS build container and commits, per config:
  - sha256 of the whole frame's float32 bits ([H][W][4], row 0 = top, little-endian),
  - a 16-hex-digit sha256 prefix per row (so a failing GPU test names its rows),
  - the segment total (ray segments traced, the GPU's in-kernel count must equal it),
  - the whole-frame per-channel RMS of the accumulated image against the reference's
    sequential fp32 sum / spp (north_star's 1e-4 bar), both from the same oracle pass.
The accumulation is the renderer's own default: quantum G = vcrt_work_quantum(desc) (4 for C3
and C4, 8 for C5's 4096 spp) and the per-pixel scale rule (32 for these scenes, whose radiance is
<= 1 per sample). tests/test_gpu_configs.py renders the default frames on the GPU and asserts
these digests bit for bit. The fixture is data (digests and counts); the script is committed so
it can be re-run: ~25 min for C4 on 8 cores, ~6 min for C3; rows are checkpointed in /tmp.

    python tests/golden/make_full_frame_digests.py c3 c4 c5rows
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tests import oracle_py  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "full_frame_digests.json")

CONFIGS = {  # name: (scene, W, H, spp, depth, quantum, rows or None for the whole frame)
    "c3": ("final", 1920, 1080, 256, 10, 4, None),
    "c4": ("final", 1920, 1080, 1024, 10, 4, None),
    # C5: eight full 3840-wide rows at full spp (4096) and depth (50): sky, sphere field, ground
    "c5rows": ("stress4096", 3840, 2160, 4096, 50, 8, [120, 400, 700, 1000, 1300, 1600, 1900, 2150]),
}


def row_digest(row: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(row, dtype="<f4").tobytes()).hexdigest()[:16]


def run(name: str, band: int = 32, threads: int = 0) -> dict:
    scene, w, h, spp, depth, quantum, rows = CONFIGS[name]
    o = oracle_py.load()
    sp = o.scene(scene)
    cfg = o.config(w, h, spp, depth, quantum=quantum)
    want = list(range(h)) if rows is None else list(rows)
    tmp = f"/tmp/vcrt_full_{name}"
    img_path, seq_path, prog_path = tmp + "_img.npy", tmp + "_seq.npy", tmp + "_progress.json"
    mode = "r+" if os.path.exists(prog_path) else "w+"
    img = np.lib.format.open_memmap(img_path, mode=mode, dtype=np.float32,
                                    shape=(len(want), w, 4))
    seq = np.lib.format.open_memmap(seq_path, mode=mode, dtype=np.float32,
                                    shape=(len(want), w, 4))
    prog = json.load(open(prog_path)) if mode == "r+" else {"done": 0, "segments": 0}
    t0 = time.time()
    while prog["done"] < len(want):
        i0 = prog["done"]
        i1 = min(len(want), i0 + band) if rows is None else i0 + 1
        if rows is None:
            a, s, segs = o.render_seq(cfg, sp, rows=range(want[i0], want[i1 - 1] + 1),
                                      threads=threads)
            img[i0:i1] = a[want[i0]:want[i1 - 1] + 1]
            seq[i0:i1] = s[want[i0]:want[i1 - 1] + 1]
        else:  # one full row as a pixel list, so every thread takes part
            xy = [(x, want[i0]) for x in range(w)]
            a, s, segs = o.render_pixels_seq(cfg, sp, xy, threads=threads)
            img[i0] = a
            seq[i0] = s
        img.flush()
        seq.flush()
        prog["done"] = i1
        prog["segments"] += int(segs)
        json.dump(prog, open(prog_path, "w"))
        el = time.time() - t0
        print(f"{name}: rows {i1}/{len(want)}  {el:.0f} s", flush=True)
    d = (img.astype(np.float64) - seq.astype(np.float64))[..., :3].reshape(-1, 3)
    res = {
        "scene": scene, "width": w, "height": h, "spp": spp, "max_depth": depth,
        "quantum": quantum, "scale_log2": 32,
        "rows": None if rows is None else want,
        "frame_sha256": hashlib.sha256(np.ascontiguousarray(img, dtype="<f4").tobytes()).hexdigest(),
        "row_sha256_16": [row_digest(img[i]) for i in range(len(want))],
        "segments": prog["segments"],
        "rms_vs_sequential": [float(v) for v in np.sqrt((d ** 2).mean(axis=0))],
        "max_abs_vs_sequential": float(np.abs(d).max()),
        "finite": bool(np.isfinite(img).all()),
        "max_value": float(img[..., :3].max()),
        # eight pixels' float bits (x, y, r, g, b, a), so a CPU test can re-render a few pixels
        "sample_pixels": [[int(x), int(want[i])] + [int(v) for v in img[i, x].view(np.uint32)]
                          for i, x in zip(np.linspace(0, len(want) - 1, 8).astype(int),
                                          np.linspace(0, w - 1, 8).astype(int))],
    }
    return res


def main(names):
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    out["_about"] = ("oracle/vcrt_oracle.c over whole frames (or the listed full-width rows) "
                     "of BASELINE C3/C4/C5 at full spp and depth, made by "
                     "tests/golden/make_full_frame_digests.py")
    for n in names:
        out[n] = run(n)
        json.dump(out, open(OUT, "w"), indent=1)
        print(n, {k: v for k, v in out[n].items() if k != "row_sha256_16"}, flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or ["c3", "c4", "c5rows"])
