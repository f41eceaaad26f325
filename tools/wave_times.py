"""Wave start / queue-drained / end times of the product kernel (diagnostics code object built
with -DVCRT_WAVE_END_TIMES, run with VCRT_DEBUG_STATS=2): how long the frame's waves keep
running after the queue empties, per rank of an N-way shard (default C4; --scene / --width /
--height / --spp / --depth for the other configs, e.g. C2: three 800 450 64 8).
  VCRT_DEBUG_STATS=2 python tools/wave_times.py CODE_OBJECT [--chunk K] [--worlds 1,8]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vulkancomputeraytracing_amd as vc  # noqa: E402

a = argparse.ArgumentParser()
a.add_argument("code_object")
a.add_argument("--chunk", type=int, default=0)
a.add_argument("--worlds", default="1,8")
a.add_argument("--ranks", type=int, default=2)
a.add_argument("--tail", type=int, default=0)
a.add_argument("--tail-chunk", type=int, default=0)
a.add_argument("--scene", default="final")
a.add_argument("--width", type=int, default=1920)
a.add_argument("--height", type=int, default=1080)
a.add_argument("--spp", type=int, default=1024)
a.add_argument("--depth", type=int, default=10)
a.add_argument("--blocks-per-cu", type=int, default=0)
args = a.parse_args()
for world in [int(w) for w in args.worlds.split(",")]:
    for rank in range(min(world, args.ranks)):
        desc = vc.RenderDesc(width=args.width, height=args.height, samples_per_pixel=args.spp,
                             max_depth=args.depth, blocks_per_cu=args.blocks_per_cu,
                             device=0, rank=rank, world_size=world, accumulate_chunk=args.chunk,
                             accumulate_tail=args.tail, accumulate_tail_chunk=args.tail_chunk,
                             code_object_path=args.code_object)
        with vc.Renderer(desc, args.scene) as r:
            r.draw_next_frame()
            r.draw_next_frame()
            st = r.stats()
        d = st["debug"]
        waves = d[7]
        t0 = d[9]
        ms = lambda t: round((t - t0) / 1e5, 3)  # 100 MHz ticks -> ms after the first start
        print(json.dumps({"world": world, "rank": rank, "chunk": st["accumulate_chunk"],
                          "tail": [st["accumulate_tail"], st["accumulate_tail_chunk"]],
                          "kernel_ms": round(st["kernel_ms"], 3), "waves": waves,
                          "first_drained_ms": ms(d[10]),
                          "mean_drained_ms": ms(d[11] * 256 / waves),
                          "first_end_ms": ms(d[5]), "mean_end_ms": ms(d[6] * 256 / waves),
                          "last_end_ms": ms(d[4]),
                          "lifetime_hist_0.1ms": d[12:28], "after_drain_hist": d[28:32]}))
