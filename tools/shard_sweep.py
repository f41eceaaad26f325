"""Per-rank kernel time of an N-way tile-sharded frame, all ranks rendered one after another on
this GPU: max over ranks is what strong scaling sees; sum vs the unsharded frame shows the
per-rank fixed costs (launch, drain).

Each renderer draws --frames frames back to back and reports the mean kernel time of the last
half. The GPU's clock follows its load: a lone 12-ms shard frame after host work runs at ~2.29 GHz
(GRBM_GUI_ACTIVE, profiles/r05_clock.txt) where the 90-ms full frame's second frame runs at
~2.38 GHz, so the round-4 method (the second frame of each renderer) charged the shards ~3.5% of
clock. On an 8-GPU node every GPU renders its shard frame after frame; the sustained frames are
that steady state. --frames 2 --last 1 is the round-4 method."""
import argparse
import json
import os
import sys

# VCRT_PKG_ROOT: the package (and its libvcrt.so) of another tree (tools/mkab_tree.sh), for A/B
sys.path.insert(0, os.environ.get("VCRT_PKG_ROOT",
                                  os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import vulkancomputeraytracing_amd as vc  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--spp", type=int, default=1024)
p.add_argument("--worlds", default="2,4,8")
p.add_argument("--chunk", type=int, default=0)
p.add_argument("--variant", type=int, default=0)
p.add_argument("--code-object", default=None)
p.add_argument("--tail", type=int, default=0, help="accumulate_tail (0 = rule, -1 = none)")
p.add_argument("--tail-chunk", type=int, default=0)
p.add_argument("--quantum", type=int, default=0, help="accumulate_quantum (0 = the rule)")
p.add_argument("--frames", type=int, default=8, help="frames per renderer, back to back")
p.add_argument("--last", type=int, default=0, help="frames averaged at the end (0: half)")
a = p.parse_args()
last = a.last or max(1, a.frames // 2)


def timed(desc):
    """Kernel ms of a renderer's last `last` of `frames` frames, and its last stats."""
    with vc.Renderer(desc, "final") as r:
        ms = []
        for _ in range(a.frames):
            r.draw_next_frame()
            ms.append(r.stats()["kernel_ms"])
        return sum(ms[-last:]) / last, r.stats()


base = dict(width=1920, height=1080, samples_per_pixel=a.spp, max_depth=10, device=0,
            accumulate_chunk=a.chunk, kernel_variant=a.variant, code_object_path=a.code_object,
            accumulate_tail=a.tail, accumulate_tail_chunk=a.tail_chunk,
            accumulate_quantum=a.quantum)
full, st = timed(vc.RenderDesc(**base))
res = {"full_ms": full, "spp": a.spp, "chunk_arg": a.chunk, "variant": a.variant,
       "frames": a.frames, "last": last,
       "full_partition": [st["accumulate_chunk"], st["accumulate_tail"],
                          st["accumulate_tail_chunk"]]}
for world in [int(x) for x in a.worlds.split(",")]:
    per, work = [], []
    for rank in range(world):
        ms, st = timed(vc.RenderDesc(rank=rank, world_size=world, **base))
        per.append(ms)
        work.append([st["segments"], st["group_tests"], st["bound_tests"]])
    res[f"world{world}"] = {"per_rank_ms": [round(x, 2) for x in per], "max_ms": max(per),
                            "per_rank_segments_groups_bounds": work,
                            "sum_ms": sum(per), "chunk": st["accumulate_chunk"],
                            "tail": [st["accumulate_tail"], st["accumulate_tail_chunk"]],
                            "ideal_efficiency": full / (world * max(per))}
    print(world, json.dumps(res[f"world{world}"]), file=sys.stderr)
print(json.dumps(res))
