"""Wave-union vs per-lane group need for the culled scan (statistics only, float64 geometry):
reuses cull_potential.py's path sampler, the real group bounds from vcrt_cull_tables, and
reports per wave-iteration: union of needed groups, max over lanes, mean per lane; for the
line test alone and with the t-interval test at the final hit distance (ideal ordering)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools.sim import cull_potential as cp  # noqa: E402
from vulkancomputeraytracing_amd import scene as S  # noqa: E402

t = S.cull_tables(S.builtin_scene("final"))
b = t["bound"]
G = 2 * b.shape[0]
col = lambda k: np.stack([b[:, k], b[:, k + 1]], 1).reshape(G).astype(np.float64)  # noqa: E731
Cc = np.stack([col(0), col(2), col(4)], 1)
Rr = col(6)
real = (t["index"] >= 0).any(1)

rng = np.random.default_rng(2)
tot = {k: 0.0 for k in ("union", "max", "mean", "union_t", "max_t", "mean_t")}
n_it = 0
for _ in range(30):
    tx, ty = rng.integers(0, cp.W // 8), rng.integers(0, cp.H // 8)
    streams = []
    for i in range(64):
        x, y = tx * 8 + i % 8, ty * 8 + i // 8
        st = []
        for s in range(4):
            st += cp.path(x, y, s)
        streams.append(st)
    L = max(len(s) for s in streams)
    for it in range(min(L, 12)):
        rays = [s[it] for s in streams if it < len(s)]
        need = np.zeros((len(rays), G), bool)
        need_t = np.zeros((len(rays), G), bool)
        for li, (org, d) in enumerate(rays):
            oc = org[None, :] - Cc
            a = d @ d
            hb = oc @ d
            dist2 = (oc * oc).sum(1) - hb * hb / a
            H = Rr + 0.03
            line = dist2 <= H ** 2
            _, tb = cp.hit(org, d)
            tc = -hb / a
            h = H / np.sqrt(a)
            inrange = (tc + h > 0) & (tc - h < tb)
            need[li] = line & real
            need_t[li] = line & inrange & real
        for k, m in (("", need), ("_t", need_t)):
            tot["union" + k] += m.any(0).sum()
            tot["max" + k] += m.sum(1).max()
            tot["mean" + k] += m.sum(1).mean()
        n_it += 1
print({k: round(v / n_it, 1) for k, v in tot.items()}, "groups", int(real.sum()))
