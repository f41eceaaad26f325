"""Per-rank kernel time (second frame) of an N-way tile-sharded frame, all ranks rendered one
after another on this GPU: max over ranks is what strong scaling sees; sum vs the unsharded frame shows the
per-rank fixed costs (launch, drain)."""
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
a = p.parse_args()
base = dict(width=1920, height=1080, samples_per_pixel=a.spp, max_depth=10, device=0,
            accumulate_chunk=a.chunk, kernel_variant=a.variant, code_object_path=a.code_object,
            accumulate_tail=a.tail, accumulate_tail_chunk=a.tail_chunk,
            accumulate_quantum=a.quantum)
# steady state: the second frame of each renderer (the first after Begin runs ~5% slower)
with vc.Renderer(vc.RenderDesc(**base), "final") as r:
    r.draw_next_frame()
    r.draw_next_frame()
    st = r.stats()
    full = st["kernel_ms"]
res = {"full_ms": full, "spp": a.spp, "chunk_arg": a.chunk, "variant": a.variant,
       "full_partition": [st["accumulate_chunk"], st["accumulate_tail"],
                          st["accumulate_tail_chunk"]]}
for world in [int(x) for x in a.worlds.split(",")]:
    per = []
    for rank in range(world):
        with vc.Renderer(vc.RenderDesc(rank=rank, world_size=world, **base), "final") as r:
            r.draw_next_frame()
            r.draw_next_frame()
            st = r.stats()
            per.append(st["kernel_ms"])
    res[f"world{world}"] = {"per_rank_ms": [round(x, 2) for x in per], "max_ms": max(per),
                            "sum_ms": sum(per), "chunk": st["accumulate_chunk"],
                            "tail": [st["accumulate_tail"], st["accumulate_tail_chunk"]],
                            "ideal_efficiency": full / (world * max(per))}
    print(world, json.dumps(res[f"world{world}"]), file=sys.stderr)
print(json.dumps(res))
