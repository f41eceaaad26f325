"""Estimate wave-level cluster culling for the final scene: simulate paths (float64, approximate
RTIOW math; statistics only), emulate the persistent kernel's lane streams (each lane runs its
pixel's samples back to back), and count for every wave-iteration the fraction of sphere
clusters that at least one lane's ray line may hit (line distance <= R + margin)."""
import sys
import os
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests import oracle_py  # noqa: E402

o = oracle_py.load()
S = o.scene("final")
C = S["center"].astype(np.float64); R = S["radius"].astype(np.float64)
COL = S["colour"].astype(np.float64); TYP = S["texture"][:, 0].astype(int); PAR = S["texture"][:, 1]
W, H = 1920, 1080
cam = o.camera(o.config(W, H, 1, 10)).astype(np.float64)
p00, du, dv, ctr = cam[0:3], cam[3:6], cam[6:9], cam[9:12]
rng = np.random.default_rng(1)


def hit(o_, d_):
    oc = o_[None, :] - C
    a = d_ @ d_
    hb = oc @ d_
    cc = (oc * oc).sum(1) - R * R
    disc = hb * hb - a * cc
    best, bt = -1, 1e5
    for j in np.nonzero(disc >= 0)[0]:
        sq = np.sqrt(disc[j])
        for t in ((-hb[j] - sq) / a, (-hb[j] + sq) / a):
            if 0.001 < t < bt:
                bt, best = t, j
                break
    return best, bt


def path(x, y, s):
    jx, jy = rng.uniform(-0.5, 0.5, 2)
    d = (p00 + x * du + y * dv + jx * du + jy * dv) - ctr
    org = ctr.copy()
    segs = []
    for depth in range(10):
        segs.append((org.copy(), d.copy()))
        j, t = hit(org, d)
        if j < 0:
            break
        p = org + t * d
        n = (p - C[j]) / R[j]
        u = rng.uniform(0, 1, 3); u /= np.linalg.norm(u)
        if TYP[j] == 1:
            d = n + u
        elif TYP[j] == 2:
            d = d - 2 * (n @ d) * n + PAR[j] * u
        else:
            d = d - 2 * (n @ d) * n if rng.uniform() < 0.5 else d  # crude glass
        org = p
    return segs


# clusters: generated spheres by grid cell blocks of BxB cells, big/ground singletons
def clusters(block):
    gen = np.arange(481)
    key = (np.floor((C[gen, 0] + 11) / block) * 100 + np.floor((C[gen, 2] + 11) / block)).astype(int)
    out = []
    for k in np.unique(key):
        m = gen[key == k]
        out.append(m)
    for j in range(481, 485):
        out.append(np.array([j]))
    cen, rad = [], []
    for m in out:
        c = C[m].mean(0)
        cen.append(c)
        rad.append(max(np.linalg.norm(C[j] - c) + R[j] for j in m))
    return out, np.array(cen), np.array(rad)


if __name__ == "__main__":
    tiles = [(rng.integers(0, W // 8), rng.integers(0, H // 8)) for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 40)]
    for block in (1, 2, 3, 4):
        cl, cc_, rr = clusters(block)
        sizes = np.array([len(m) for m in cl])
        work_full, work_cull = 0.0, 0.0
        for tx, ty in tiles:
            streams = []
            for i in range(64):
                x, y = tx * 8 + i % 8, ty * 8 + i // 8
                st = []
                for s in range(4):
                    st += path(x, y, s)
                streams.append(st)
            L = max(len(s) for s in streams)
            for it in range(min(L, 12)):
                rays = [s[it] for s in streams if it < len(s)]
                if not rays:
                    break
                need = np.zeros(len(cl), bool)
                for org, d in rays:
                    oc = org[None, :] - cc_
                    a = d @ d
                    hb = oc @ d
                    dist2 = (oc * oc).sum(1) - hb * hb / a
                    margin = rr + 0.03 + 2e-3 * np.sqrt((oc * oc).sum(1))
                    need |= dist2 <= margin ** 2
                work_full += 485
                work_cull += sizes[need].sum() + len(cl) * 16 / 9.5 / 4  # + cluster tests
        print(f"block {block}x{block}: {len(cl)} clusters, mean size {sizes[:-4].mean():.1f}; "
              f"scan work with culling = {work_cull / work_full:.3f} of full")
