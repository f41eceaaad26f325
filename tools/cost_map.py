"""Segments per pixel of a frame (diagnostics code object built with -DVCRT_COST_MAP: the tracer
counts each pixel's segments into its sums' unused fourth channel, the resolve writes them to
alpha), saved as a float32 [H, W] .npy for offline balance studies (tools/balance_study.py).
  python tools/cost_map.py CODE_OBJECT OUT.npy [--spp 64]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vulkancomputeraytracing_amd as vc  # noqa: E402

a = argparse.ArgumentParser()
a.add_argument("code_object")
a.add_argument("out")
a.add_argument("--spp", type=int, default=64)
a.add_argument("--scene", default="final")
a.add_argument("--width", type=int, default=1920)
a.add_argument("--height", type=int, default=1080)
a.add_argument("--depth", type=int, default=10)
args = a.parse_args()
desc = vc.RenderDesc(width=args.width, height=args.height, samples_per_pixel=args.spp,
                     max_depth=args.depth, device=0, code_object_path=args.code_object)
with vc.Renderer(desc, args.scene) as r:
    r.draw_next_frame()
    img = r.read_framebuffer()
    st = r.stats()
cost = img[..., 3].astype(np.float32)
print(f"segments {st['segments']} map sum {cost.sum():.0f}")
np.save(args.out, cost)
