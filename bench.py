"""Headline benchmark: Msamples/s (pixels x spp / s) rendering the RTIOW final scene at
1920x1080, 1024 spp, max depth 10 (BASELINE.json metric, configs[3]) on N MI355X GPUs.

One step = one DrawNextFrame of the whole frame: on every rank the gfx950 tracer renders the
rank's 8x8 tiles (tile (tx, ty) belongs to rank (tx + ty) % N), then (N > 1) the packed rank
framebuffers are all-gathered over RCCL and rank 0 re-interleaves the frame. The frame is fixed
as N grows (strong scaling).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_TFLOPS = 157.3        # MI355X FP32 vector, MI355X_MICROARCH.md chip table
FLOPS_PER_SPHERE_TEST = 23      # functions.glsl:15-19 as written
FLOPS_PER_BOUND_TEST = 26       # tracer.hip box_gap, per box: 6 fma 12, per-axis min/max 6,
                                # tnear/tfar 4, gap sub + add + fma 4
KERNEL_NAMES = {1: "vcrt_trace_lds", 2: "vcrt_trace_smem", 3: "vcrt_trace_cull",
                4: "vcrt_trace_cull_lane", 5: "vcrt_trace_cull_flat"}
PROFILE_TRAFFIC = os.path.join(ROOT, "profiles", "traffic.json")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# BASELINE.json configs; c4 (the headline metric's workload) is the default.
# c1 is the reference's CPU plumbing case (tests/), not a bench line.
CONFIGS = {
    "c2": {"scene": "three", "width": 800, "height": 450, "spp": 64, "depth": 8},
    "c3": {"scene": "final", "width": 1920, "height": 1080, "spp": 256, "depth": 10},
    "c4": {"scene": "final", "width": 1920, "height": 1080, "spp": 1024, "depth": 10},
    "c5": {"scene": "stress4096", "width": 3840, "height": 2160, "spp": 4096, "depth": 50},
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--config", choices=sorted(CONFIGS), default="c4",
                   help="BASELINE.json workload (c4: the headline metric; c5: the stress scene)")
    p.add_argument("--width", type=int, default=None)
    p.add_argument("--height", type=int, default=None)
    p.add_argument("--spp", type=int, default=None)
    p.add_argument("--depth", type=int, default=None)
    p.add_argument("--scene", default=None)
    p.add_argument("--variant", type=int, default=0)
    p.add_argument("--blocks-per-cu", type=int, default=0)
    p.add_argument("--chunk", type=int, default=0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--validate", action="store_true",
                   help="rank 0 re-renders the frame on one GPU after the timed steps and checks "
                        "the gathered frame bit for bit (use with an explicit --chunk)")
    p.add_argument("--cpu-seconds", type=float, default=15.0,
                   help="target CPU work for the cpu_baseline sample")
    a = p.parse_args()
    for k, v in CONFIGS[a.config].items():  # explicit flags override the preset
        if getattr(a, k) is None:
            setattr(a, k, v)
    return a


def cpu_baseline(args):
    """The CPU oracle (C restatement of shader.comp) on a bounded sample of the same workload:
    full-width rows y = 0, k, 2k, ... at the first s samples, on the host's cores."""
    from tests import oracle_py
    o = oracle_py.load()
    threads = min(16, os.cpu_count() or 1)
    scene = o.scene(args.scene)
    # calibrate on a tiny sample, then size the real one for ~cpu_seconds of work
    # (34 rows spread over the frame: sky, spheres and ground in frame proportion)
    probe_rows, probe_spp = range(0, args.height, max(1, args.height // 32)), 2
    t0 = time.perf_counter()
    o.render(o.config(args.width, args.height, probe_spp, args.depth), scene, rows=probe_rows,
             threads=threads)
    dt = max(time.perf_counter() - t0, 1e-3)
    rate = len(probe_rows) * args.width * probe_spp / dt  # samples/s
    target = rate * args.cpu_seconds
    frame = args.width * args.height
    if target >= 4 * frame:  # whole frame at the first spp samples
        spp = max(4, min(args.spp, int(target // frame)))
        rows = range(0, args.height)
        step = 1
    else:                    # every step-th row at 4 spp
        spp = min(args.spp, 4)
        nrows = max(1, int(target / (args.width * spp)))
        step = max(1, args.height // nrows)
        rows = range(0, args.height, step)
    t0 = time.perf_counter()
    o.render(o.config(args.width, args.height, spp, args.depth), scene, rows=rows, threads=threads)
    dt = time.perf_counter() - t0
    samples = len(rows) * args.width * spp
    return {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"oracle/vcrt_oracle.c -O3, {threads} threads: rows y%{step}==0 "
                      f"({len(rows)} rows x {args.width}) at spp {spp} of the same "
                      f"{args.scene} scene/camera/depth {args.depth}; {samples} samples "
                      f"in {dt:.2f} s",
            "seconds": round(dt, 3)}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import vulkancomputeraytracing_amd as vc
    from vulkancomputeraytracing_amd import distributed as D

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    # one process per GPU; VCRT_DIST_BACKEND=gloo rehearses the N > 1 flow with several ranks
    # sharing the GPUs of a smaller box (RCCL needs one GPU per rank)
    backend = os.environ.get("VCRT_DIST_BACKEND", "nccl")
    device = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)

    desc = vc.RenderDesc(width=args.width, height=args.height, samples_per_pixel=args.spp,
                         max_depth=args.depth, device=device, rank=rank, world_size=world,
                         kernel_variant=args.variant,
                         blocks_per_cu=args.blocks_per_cu, accumulate_chunk=args.chunk)
    dev = torch.device("cuda", device)
    tiles_pad = D.tiles_per_rank(args.width, args.height, world)
    local_elems = args.width * args.height if world == 1 else tiles_pad * 64
    local = torch.zeros((local_elems, 4), dtype=torch.float32, device=dev)
    frame = None
    if world > 1 and rank == 0:
        frame = torch.empty((args.height, args.width, 4), dtype=torch.float32, device=dev)

    r = vc.Renderer(desc, args.scene)
    r.set_framebuffer_device(local.data_ptr(), local.numel() * 4)
    nspheres = len(vc.builtin_scene(args.scene))

    def step():
        r.draw_next_frame()  # returns when the rank's rows are complete
        if world > 1:
            gathered = D.gather_tiles(local, tiles_pad)
            if rank == 0:
                torch.cuda.current_stream().synchronize()
                D.assemble_frame(r, gathered, frame, tiles_pad)

    for i in range(args.warmup):
        step()
        log(f"[rank {rank}] warmup {i}: frame {r.stats()['frame_ms']:.1f} ms")

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    kernel_ms, segments = [], []
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
        st = r.stats()
        kernel_ms.append(st["kernel_ms"])
        segments.append(st["segments"])
        log(f"[rank {rank}] step {i}: frame {st['frame_ms']:.1f} ms, kernel "
            f"{st['kernel_ms']:.1f} ms, {st['segments']} segments")
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    st = r.stats()
    r.close()
    validated = None
    if args.validate and rank == 0:
        import numpy as np
        got = (frame if world > 1 else local.view(args.height, args.width, 4)).cpu().numpy()
        # the reference render sums in the ranks' chunks (the default chunk follows the largest
        # rank's share, so it is the same on every rank)
        ref_desc = vc.RenderDesc(width=args.width, height=args.height, samples_per_pixel=args.spp,
                                 max_depth=args.depth, device=device, kernel_variant=args.variant,
                                 accumulate_chunk=st["accumulate_chunk"])
        with vc.Renderer(ref_desc, args.scene) as ref:
            ref.draw_next_frame()
            want = ref.read_framebuffer()
        validated = bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
        log(f"validate: gathered frame bit-identical to a 1-GPU render: {validated}")

    if rank == 0:
        samples = args.width * args.height * args.spp * args.steps
        value = samples / elapsed / 1e6
        k_ms = sum(kernel_ms) / len(kernel_ms)
        seg = sum(segments) / len(segments)
        # Algorithmic work: the reference's linear scan tests every sphere on
        # every segment, 23 flops each (functions.glsl:15-19).
        flops = seg * nspheres * FLOPS_PER_SPHERE_TEST
        # Issued work: the culled scans skip most of those tests (same bits): every lane of each
        # wave-level group test (4 spheres x 23) and box test (26); the linear scans issue all.
        executed = flops
        if st["kernel_variant"] in (3, 4, 5):
            executed = (st["group_tests"] * 64 * 4 * FLOPS_PER_SPHERE_TEST
                        + st["bound_tests"] * 64 * FLOPS_PER_BOUND_TEST)
        kernel = KERNEL_NAMES.get(st["kernel_variant"], "?")
        if st["kernel_variant"] == 4 and st["tables_in_lds"]:
            kernel += "_lds_wide" if st["block_threads"] == 1024 else "_lds"
        if st["kernel_variant"] == 5 and not st["tables_in_lds"]:
            kernel += "_global"
        achieved = flops / (k_ms * 1e-3) / 1e12
        issued = executed / (k_ms * 1e-3) / 1e12
        # HBM bytes and VALU busy of the same kernel at this config, from the committed
        # rocprofv3 PMC passes (tools/gpu_profile.sh -> profiles/traffic.json)
        key = f"{args.scene}_{args.width}x{args.height}_s{args.spp}_d{args.depth}_n{world}"
        prof = {}
        if os.path.exists(PROFILE_TRAFFIC):
            try:
                prof = json.load(open(PROFILE_TRAFFIC)).get(key, {})
            except (OSError, ValueError):
                prof = {}
        cfg_name = next((n for n, c in CONFIGS.items()
                         if all(getattr(args, k) == v for k, v in c.items())), "custom")
        metric = ("Msamples/sec (pixels×spp/s) at 1920×1080, 1024spp, RTIOW final scene"
                  if cfg_name == "c4" else
                  f"Msamples/sec (pixels×spp/s) at {args.width}×{args.height}, {args.spp}spp, "
                  f"{args.scene} scene")
        out = {
            "metric": metric,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (deterministic RTIOW scene from SceneGenerator seed 5489)",
            "config": {"workload": f"{cfg_name}: rtiow_{args.scene}_{args.width}x{args.height}_"
                                   f"{args.spp}spp_d{args.depth}",
                       "scene": args.scene, "spheres": nspheres, "width": args.width,
                       "height": args.height, "spp": args.spp, "max_depth": args.depth,
                       "parallelism": f"tiles8x8-diagonal-x{world}",
                       "accumulate_chunk": st["accumulate_chunk"],
                       "kernel_variant": st["kernel_variant"],
                       "grid_blocks": st["grid_blocks"]},
            # fp32 VALU-bound (no MFMA); achieved = algorithmic flops per
            # launch (segments x spheres x 23, the reference's hit_sphere scan of every
            # segment this launch traced) / the kernel's HIP-event time. The exact culled
            # scan skips most of those tests with bit-identical results, so frac exceeds 1;
            # what the kernel issued is beside it, and the hardware view is VALU busy.
            "roofline": {"bound": "valu", "achieved": round(achieved, 3),
                         "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                         "traffic": prof.get("hbm_bytes_per_launch"),
                         "kernel": kernel, "kernel_ms": round(k_ms, 3),
                         "numerator": "SURVEY.md 8(d): segments x spheres x 23 flops per launch "
                                      "(functions.glsl:15-19 for every sphere of every segment)",
                         "flops_per_launch": flops,
                         "segments_per_launch": int(seg),
                         "issued_flops_per_launch": executed,
                         "issued_tflops": round(issued, 3),
                         "issued_frac": round(issued / PEAK_FP32_TFLOPS, 4),
                         "issued_numerator": "wave-level group tests x 64 x 4 x 23 + bound tests "
                                             "x 64 x 26 (DESIGN.md 5)",
                         "valu_busy_pct": prof.get("valu_busy_pct"),
                         "valu_utilization_pct": prof.get("valu_utilization_pct")},
        }
        if validated is not None:
            out["validated_bitwise_vs_1gpu"] = validated
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(args)
            except Exception as e:  # reported, never fatal to the GPU number
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
