"""Per-rank cost balance of tile-ownership maps on a measured cost map (segments per pixel,
tools/cost_map.py): max / mean of the ranks' summed segments for N GPUs. The product assigns
8x8 tile (tx, ty) to rank (tx + slope * ty) % N (vcrt_math.h owner_of, kTileSlope).
  python tools/balance_study.py COST.npy [--worlds 2,4,8]"""
import argparse

import numpy as np

a = argparse.ArgumentParser()
a.add_argument("cost")
a.add_argument("--worlds", default="2,4,8")
args = a.parse_args()
c = np.load(args.cost).astype(np.float64)
h, w = c.shape
ty, tx = np.mgrid[0:h, 0:w] // 8
for world in [int(x) for x in args.worlds.split(",")]:
    out = []
    for name, rank in [(f"slope {s}", (tx + s * ty) % world) for s in range(1, world, 2)] + \
                      [("slope 1, period shift", (tx + ty + (ty // world)) % world),
                       ("4x4 cells, slope 1", (np.mgrid[0:h, 0:w][1] // 4 + np.mgrid[0:h, 0:w][0] // 4) % world)]:
        per = np.bincount(rank.ravel(), weights=c.ravel(), minlength=world)
        out.append(f"{name}: {per.max() / per.mean():.4f}")
    print(f"N={world}: " + "; ".join(out))
