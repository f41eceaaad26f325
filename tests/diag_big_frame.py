"""Diagnostic (test infrastructure: the oracle is its checker): where a large frame departs
from the oracle. Renders W x H once per setting
(--settings: env assignments per run, e.g. "none" "VCRT_PRIMARY_LISTS=0" "VCRT_ACCUM_RING=0")
and compares every --step-th row with the oracle's pixels, printing the rows that differ, the
first of them and a few pixels of it.

  python tests/diag_big_frame.py --width 8192 --height 8192 --spp 8 --depth 3 --step 256
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import vulkancomputeraytracing_amd as vc  # noqa: E402
from tests import oracle_py  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--width", type=int, default=8192)
p.add_argument("--height", type=int, default=8192)
p.add_argument("--spp", type=int, default=8)
p.add_argument("--depth", type=int, default=3)
p.add_argument("--step", type=int, default=256)
p.add_argument("--variant", type=int, default=0)
p.add_argument("--settings", nargs="*", default=["none"])
a = p.parse_args()
o = oracle_py.load()
sc = o.scene("final")
rows = sorted(set(range(0, a.height, a.step)) | {a.height - 1})
want_rows = {}
for setting in a.settings:
    env = {}
    if setting != "none":
        for kv in setting.split(","):
            k, v = kv.split("=")
            env[k] = v
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    desc = vc.RenderDesc(width=a.width, height=a.height, samples_per_pixel=a.spp,
                         max_depth=a.depth, device=0, kernel_variant=a.variant)
    with vc.Renderer(desc, "final") as r:
        r.draw_next_frame()
        got, st = r.read_framebuffer(), r.stats()
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    cfg = o.config(a.width, a.height, a.spp, a.depth, **o.partition(st))
    bad = []
    for y in rows:
        if y not in want_rows:
            xy = np.stack([np.arange(a.width), np.full(a.width, y)], axis=1)
            want_rows[y] = o.render_pixels(cfg, sc, xy)[0]
        g = got[y]
        nd = int((g.view(np.uint32) != want_rows[y].view(np.uint32)).any(axis=1).sum())
        if nd:
            bad.append((y, nd))
    print(f"[{setting}] kernel {st['kernel']} ring {st['ring_entries']} chunk "
          f"{st['accumulate_chunk']} q {st['accumulate_quantum']}: {len(bad)} of {len(rows)} rows "
          f"differ {bad[:12]}", flush=True)
    if bad:
        y = bad[0][0]
        idx = np.nonzero((got[y].view(np.uint32) != want_rows[y].view(np.uint32)).any(axis=1))[0]
        for x in idx[:4]:
            print(f"   ({x},{y}) gpu {got[y][x].tolist()} oracle {want_rows[y][x].tolist()}")
