"""Where a frame's time goes at its ends (stats build, VCRT_DEBUG_STATS=1): kernel time, the
spread of the waves' end times (first / mean / last, s_memrealtime at 100 MHz) -- the drain --
for the full C4 frame and for one rank of an N-way shard."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["VCRT_DEBUG_STATS"] = "1"
import vulkancomputeraytracing_amd as vc  # noqa: E402

out = {}
for world, chunk in ((1, 0), (8, 0), (8, 8)):
    desc = vc.RenderDesc(width=1920, height=1080, samples_per_pixel=1024, max_depth=10, device=0,
                         rank=0, world_size=world, accumulate_chunk=chunk)
    with vc.Renderer(desc, "final") as r:
        r.draw_next_frame()
        r.draw_next_frame()
        st = r.stats()
    d = st["debug"]
    waves = d[7]
    first, last, mean = d[5], d[4], d[6] * 256 / waves
    out[f"n{world}_k{st['accumulate_chunk']}"] = {
        "kernel_ms": round(st["kernel_ms"], 3),
        "drain_last_minus_first_ms": round((last - first) / 1e5, 3),
        "drain_last_minus_mean_ms": round((last - mean) / 1e5, 3),
        "waves": waves, "iters_per_wave": round(d[0] / waves, 1),
        "active_lanes_per_iter": round(d[1] / max(1, d[0]), 2)}
print(json.dumps(out, indent=1))
