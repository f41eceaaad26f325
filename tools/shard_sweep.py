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
p.add_argument("--gather", action="store_true",
               help="also time what rank 0 adds at each N: vcrt_assemble of the N-way packed "
                    "buffer and the receives of the N - 1 peers' tiles (a local device copy of "
                    "the same bytes as a lower bound, and the xGMI link model)")
p.add_argument("--link-gbs", type=float, default=76.8,
               help="xGMI GB/s per link and direction (MI355X: 7 links x ~153.6 GB/s "
                    "bidirectional; each peer sends over its own link)")
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


def rank0_extra(world, reps=50):
    """What rank 0 adds after its own shard at N = world (capi.cpp gather_frame): receiving the
    N - 1 peers' packed tiles (pad x 64 x 16 B each, padded to the largest rank) and
    vcrt_assemble re-interleaving all N into the [H][W] frame. Timed on this GPU: the assemble
    by the host wall time of back-to-back vcrt_assemble_tiles calls, each of which waits for its
    kernel (it runs on the renderer's stream, which torch's events do not see: launch and wait
    included, an upper bound), the receives as
    a device-to-device copy of the same bytes (a lower bound: xGMI is slower than HBM) and as
    the link model (each peer over its own link at --link-gbs, all at once)."""
    import time
    import torch
    from vulkancomputeraytracing_amd import distributed as D
    w, h = 1920, 1080
    pad = D.tiles_per_rank(w, h, world)
    per_rank_bytes = pad * 64 * 16
    gathered = torch.zeros((world * pad * 64, 4), dtype=torch.float32, device="cuda:0")
    frame = torch.empty((h, w, 4), dtype=torch.float32, device="cuda:0")
    with vc.Renderer(vc.RenderDesc(width=w, height=h, world_size=world, device=0)) as r:
        for _ in range(5):
            r.assemble_tiles(gathered.data_ptr(), frame.data_ptr(), pad)
        t0 = time.perf_counter()
        for _ in range(reps):
            r.assemble_tiles(gathered.data_ptr(), frame.data_ptr(), pad)
        assemble_ms = (time.perf_counter() - t0) * 1e3 / reps
    src = torch.empty(((world - 1) * pad * 64, 4), dtype=torch.float32, device="cuda:0")
    dst = torch.empty_like(src)
    for _ in range(5):
        dst.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize()
    return {"per_rank_bytes": per_rank_bytes, "peers": world - 1,
            "assemble_ms": assemble_ms, "recv_copy_ms": e0.elapsed_time(e1) / reps,
            "recv_link_model_ms": per_rank_bytes / (a.link_gbs * 1e9) * 1e3}


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
    extra = rank0_extra(world) if a.gather else None
    res[f"world{world}"] = {"per_rank_ms": [round(x, 2) for x in per], "max_ms": max(per),
                            "per_rank_segments_groups_bounds": work,
                            "sum_ms": sum(per), "chunk": st["accumulate_chunk"],
                            "tail": [st["accumulate_tail"], st["accumulate_tail_chunk"]],
                            "ideal_efficiency": full / (world * max(per))}
    if extra is not None:  # the frame ends when rank 0 has received and assembled every shard
        w = res[f"world{world}"]
        w["rank0_gather"] = extra
        w["efficiency_with_gather_copy_bound"] = full / (
            world * (max(per) + extra["recv_copy_ms"] + extra["assemble_ms"]))
        w["efficiency_with_gather_link_model"] = full / (
            world * (max(per) + extra["recv_link_model_ms"] + extra["assemble_ms"]))
    print(world, json.dumps(res[f"world{world}"]), file=sys.stderr)
print(json.dumps(res))
