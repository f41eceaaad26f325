"""Render N frames of one configuration through the C ABI and print the stats as JSON
(profiling driver: rocprofv3 ... -- python tools/render_once.py ...)."""
import argparse
import json
import os
import sys

# VCRT_PKG_ROOT: the package (and its libvcrt.so) of another tree (tools/mkab_tree.sh), for A/B
sys.path.insert(0, os.environ.get("VCRT_PKG_ROOT",
                                  os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import vulkancomputeraytracing_amd as vc  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--spp", type=int, default=64)
    p.add_argument("--depth", type=int, default=10)
    p.add_argument("--scene", default="final")
    p.add_argument("--variant", type=int, default=0)
    p.add_argument("--blocks-per-cu", type=int, default=0)
    p.add_argument("--frames", type=int, default=1)
    p.add_argument("--code-object", default=None)
    p.add_argument("--chunk", type=int, default=0)
    p.add_argument("--rank", type=int, default=0)
    p.add_argument("--world", type=int, default=1)
    p.add_argument("--tail", type=int, default=0, help="accumulate_tail (0 = rule, -1 = none)")
    p.add_argument("--tail-chunk", type=int, default=0)
    p.add_argument("--quantum", type=int, default=0, help="accumulate_quantum (0 = rule)")
    a = p.parse_args()
    desc = vc.RenderDesc(width=a.width, height=a.height, samples_per_pixel=a.spp,
                         max_depth=a.depth, kernel_variant=a.variant,
                         blocks_per_cu=a.blocks_per_cu, device=0,
                         code_object_path=a.code_object, accumulate_chunk=a.chunk,
                         rank=a.rank, world_size=a.world, accumulate_tail=a.tail,
                         accumulate_tail_chunk=a.tail_chunk)
    if a.quantum:
        desc.accumulate_quantum = a.quantum
    with vc.Renderer(desc, a.scene) as r:
        out = []
        for _ in range(a.frames):
            r.draw_next_frame()
            st = r.stats()
            st["msamples_per_s"] = st["samples"] / (st["kernel_ms"] * 1e3)
            st["tests_per_s"] = st["sphere_tests"] / (st["kernel_ms"] * 1e-3)
            out.append(st)
    print(json.dumps(out[-1] if len(out) == 1 else out))


if __name__ == "__main__":
    main()
