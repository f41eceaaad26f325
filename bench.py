"""Headline benchmark: Msamples/s (pixels x spp / s) rendering the RTIOW final scene at
1920x1080, 1024 spp, max depth 10 (BASELINE.json metric, configs[3]) on N MI355X GPUs.

One step = one DrawNextFrame of the whole frame. On every rank the gfx950 tracer renders the
rank's 8x8 tiles (tile (tx, ty) belongs to rank (tx + ty) % N). For N > 1 the same
vcrt_draw_next_frame then gathers every rank's packed tiles to rank 0 over RCCL, inside
libvcrt.so (vcrt_comm_init; one grouped send/recv), and rank 0 re-interleaves the frame. The
frame is fixed as N grows (strong scaling). torch.distributed (gloo) is only the control plane:
the communicator id, barriers and the max-over-ranks time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]
       torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_TFLOPS = 157.3        # MI355X FP32 vector (packed FMA), MI355X_MICROARCH.md chip table
PEAK_FP32_NONFMA_TFLOPS = 78.65  # the same issue rate without FMA (1 flop per lane-op of a packed
                                 # add/mul): the ceiling of the exact sphere test, which parity
                                 # keeps free of contraction
FLOPS_PER_SPHERE_TEST = 23      # functions.glsl:15-19 as written
FLOPS_PER_BOUND_TEST = 27       # tracer.hip box_gap, per box: 6 fma 12, per-axis min/max 6,
                                # tnear/tfar 4, the near end's clamp at 0 (fact (4)) 1,
                                # gap sub + add + fma 4
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
    p.add_argument("--min-warmup-seconds", type=float, default=3.0,
                   help="after the W warmup steps, further untimed steps until the warmup has "
                        "kept the GPU busy this long: the shader clock follows the load (a lone "
                        "12-ms shard frame runs at ~2.15-2.30 GHz, sustained frames at ~2.38: "
                        "profiles/r05_clock.txt), and the timed steps measure the steady state; "
                        "3 s also keeps the GPU busy across a once-per-5-s utilisation sampler's "
                        "tick before the CPU baseline starts. Reported as warmup_extra; 0 turns "
                        "it off")
    p.add_argument("--max-warmup-steps", type=int, default=200,
                   help="upper bound on those extra steps")
    p.add_argument("--validate", action="store_true",
                   help="(the default) after the timed steps, rank 0 checks its frame: bit for "
                        "bit against the CPU oracle on pixels of a few full-width rows at full "
                        "spp and depth, and (N > 1) against a 1-GPU render of the whole frame; "
                        "--no-validate turns it off")
    p.add_argument("--no-validate", action="store_true")
    p.add_argument("--validate-rows", type=int, default=2)
    p.add_argument("--validate-budget", type=float, default=1e10,
                   help="oracle sphere tests the row check may cost (~2 s on 16 threads): wider "
                        "or deeper workloads check every k-th pixel of the rows")
    p.add_argument("--cpu-seconds", type=float, default=15.0,
                   help="target CPU work for the cpu_baseline sample")
    a = p.parse_args()
    for k, v in CONFIGS[a.config].items():  # explicit flags override the preset
        if getattr(a, k) is None:
            setattr(a, k, v)
    return a


# ---- host description (cpu_baseline) ---------------------------------------------------------

def cpu_quota():
    """CPUs this process may use: its affinity set, capped by a cgroup v2/v1 CPU quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(period))))
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                n = min(n, max(1, q // period))
        except (OSError, ValueError):
            pass
    return n


def host_cpu():
    """Model name and physical core count of the host (all sockets), from /proc/cpuinfo."""
    model, cores = platform.processor() or "?", set()
    phys = core = None
    try:
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name":
                model = v
            elif k == "physical id":
                phys = v
            elif k == "core id":
                core = v
            elif not k and phys is not None and core is not None:
                cores.add((phys, core))
                phys = core = None
    except OSError:
        pass
    return model, (len(cores) or None)


def cpu_baseline(args):
    """The CPU oracle (C restatement of shader.comp, oracle/vcrt_oracle.c -O3) on a bounded
    sample of the same workload: full-width rows y = 0, k, 2k, ... (or the whole frame at the
    first s samples), on every CPU this process may use."""
    from tests import oracle_py
    o = oracle_py.load()
    threads = cpu_quota()
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
    model, phys = host_cpu()
    return {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "threads": threads, "host_logical_cpus": os.cpu_count(),
            "host_physical_cores": phys, "cpu_model": model,
            "sample": f"oracle/vcrt_oracle.c -O3 (linear hit_sphere scan, the reference's "
                      f"algorithm), {threads} threads = every CPU this job may use (affinity "
                      f"and cgroup quota; the host has {os.cpu_count()} logical CPUs): rows "
                      f"y%{step}==0 ({len(rows)} rows x {args.width}) at spp {spp} of the same "
                      f"{args.scene} scene/camera/depth {args.depth}; {samples} samples in "
                      f"{dt:.2f} s",
            "seconds": round(dt, 3)}


# ---- validation (outside the timed region) ---------------------------------------------------

def validate(args, got, st, device, world):
    """Rank 0's frame against the CPU oracle on the pixels of a few full-width rows at full spp
    and depth (bit for bit, same accumulation quantum and scale; every k-th pixel of the rows when
    the whole rows would cost the oracle more than --validate-budget sphere tests), and for N > 1
    against a default 1-GPU render of the whole frame: the image depends on the quantum and the
    scene's scale alone, neither of which depends on N. Runs outside the timed region."""
    import numpy as np
    from tests import oracle_py
    import vulkancomputeraytracing_amd as vc
    o = oracle_py.load()
    out = {}
    rows = list(range(args.height // (2 * args.validate_rows), args.height,
                      max(1, args.height // args.validate_rows)))[:args.validate_rows]
    scene = o.scene(args.scene)
    # ~4 segments per sample on the reference scenes' mix of sky, ground and spheres
    per_pixel = float(args.spp) * 4.0 * len(scene)
    stride = max(1, int(np.ceil(len(rows) * args.width * per_pixel / args.validate_budget)))
    xy = np.array([(x, y) for y in rows for x in range(stride // 2, args.width, stride)],
                  dtype=np.int32)
    cfg = o.config(args.width, args.height, args.spp, args.depth, **o.partition(st))
    t0 = time.perf_counter()
    want, _ = o.render_pixels(cfg, scene, xy, threads=cpu_quota())
    out["rows_vs_oracle"] = rows
    out["pixels_vs_oracle"] = int(len(xy))
    out["pixel_stride"] = stride
    out["oracle_seconds"] = round(time.perf_counter() - t0, 2)
    out["bitwise_vs_oracle"] = bool(np.array_equal(got[xy[:, 1], xy[:, 0]].view(np.uint32),
                                                   want.view(np.uint32)))
    out["accumulate_scale_log2"] = st["accumulate_scale_log2"]
    if world > 1:
        # the default 1-GPU frame (its own work items): equal bit for bit when the gather is right
        ref_desc = vc.RenderDesc(width=args.width, height=args.height, samples_per_pixel=args.spp,
                                 max_depth=args.depth, device=device, kernel_variant=args.variant)
        with vc.Renderer(ref_desc, args.scene) as ref:
            ref.draw_next_frame()
            one = ref.read_framebuffer()
            q1 = ref.stats()["accumulate_quantum"]
        out["quantum"] = [st["accumulate_quantum"], q1]
        out["bitwise_vs_1gpu"] = bool(np.array_equal(got.view(np.uint32), one.view(np.uint32)))
    log(f"validate: {out}")
    return out


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
    # One process per GPU. The frame gather runs over RCCL inside libvcrt (vcrt_comm_init).
    # VCRT_DIST_BACKEND=gloo rehearses the N > 1 flow with several ranks sharing the GPUs of a
    # smaller box (RCCL needs one GPU per rank): the gather then goes through gloo.
    backend = os.environ.get("VCRT_DIST_BACKEND", "nccl")
    device = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("gloo")  # control plane: comm id, barriers, max time

    desc = vc.RenderDesc(width=args.width, height=args.height, samples_per_pixel=args.spp,
                         max_depth=args.depth, device=device, rank=rank, world_size=world,
                         kernel_variant=args.variant,
                         blocks_per_cu=args.blocks_per_cu, accumulate_chunk=args.chunk)
    r = vc.Renderer(desc, args.scene)
    nspheres = len(vc.builtin_scene(args.scene))
    gather = None
    frame = local = None
    if world > 1 and backend == "nccl":
        ids = [vc.renderer.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(ids, src=0)
        ok = 1
        try:
            r.comm_init(ids[0])
        except vc.VcrtError as e:  # vcrt_comm_init released whatever it had set up
            log(f"[rank {rank}] vcrt_comm_init failed: {e}")
            ok = 0
        # every rank learns whether all joined; if one did not, all gather through gloo so the
        # job still measures the frame (the JSON's config.gather names the path that ran)
        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if flag.item() == 1:
            gather = "rccl in libvcrt (vcrt_draw_next_frame: grouped send/recv to rank 0)"
        else:
            log(f"[rank {rank}] RCCL gather unavailable on some rank: gloo gather instead")
            r.close()  # a fresh renderer without a communicator (vcrt_end drops it if held)
            r = vc.Renderer(desc, args.scene)
            backend = "gloo-fallback"
    if world > 1 and backend != "nccl":
        dev = torch.device("cuda", device)
        tiles_pad = D.tiles_per_rank(args.width, args.height, world)
        local = torch.zeros((tiles_pad * 64, 4), dtype=torch.float32, device=dev)
        r.set_framebuffer_device(local.data_ptr(), local.numel() * 4)
        if rank == 0:
            frame = torch.empty((args.height, args.width, 4), dtype=torch.float32, device=dev)
        gather = ("gloo fallback after vcrt_comm_init failed" if backend == "gloo-fallback" else
                  "gloo rehearsal") + " (torch.distributed.gather of host copies)"

    def step():
        r.draw_next_frame()  # N > 1 (RCCL): returns on rank 0 with the gathered frame
        if local is not None:
            gathered = D.gather_tiles(local, tiles_pad)
            if rank == 0:
                torch.cuda.current_stream().synchronize()
                D.assemble_frame(r, gathered, frame, tiles_pad)

    t_w = time.perf_counter()
    for i in range(args.warmup):
        step()
        log(f"[rank {rank}] warmup {i}: frame {r.stats()['frame_ms']:.1f} ms")
    # extra warmup until the GPU has been busy for min_warmup_seconds (every rank runs the same
    # count: rank 0 decides, so the collective draws stay matched)
    extra = 0
    if args.warmup > 0 and args.min_warmup_seconds > 0:
        torch.cuda.synchronize()
        frame_s = max(1e-4, (time.perf_counter() - t_w) / args.warmup)
        extra = max(0, int((args.min_warmup_seconds - args.warmup * frame_s) / frame_s + 0.999))
        extra = min(extra, args.max_warmup_steps)
        if world > 1:
            t = torch.tensor([extra], dtype=torch.int64)
            dist.broadcast(t, src=0)
            extra = int(t.item())
        for i in range(extra):
            step()
        if extra:
            log(f"[rank {rank}] {extra} more warmup steps ({args.min_warmup_seconds} s of load)")

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    kernel_ms, segments, gather_ms = [], [], []
    barrier()
    t0 = time.perf_counter()
    frame_ms = []
    for i in range(args.steps):  # per-frame bookkeeping kept light; logged after the timing
        step()
        k, sg, gm, fm = r.frame_times()
        kernel_ms.append(k)
        segments.append(sg)
        gather_ms.append(gm)
        frame_ms.append(fm)
    barrier()
    elapsed = time.perf_counter() - t0
    for i in range(args.steps):
        log(f"[rank {rank}] step {i}: frame {frame_ms[i]:.1f} ms, kernel {kernel_ms[i]:.1f} ms, "
            f"gather {gather_ms[i]:.2f} ms, {segments[i]} segments")
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    st = r.stats()
    # per-rank kernel times (the balance of the shards) for the JSON line
    k_mean = sum(kernel_ms) / len(kernel_ms)
    rank_ms = [k_mean]
    if world > 1:
        rank_ms = [None] * world
        dist.all_gather_object(rank_ms, k_mean)
    # every line proves its own frame (outside the timed region) unless --no-validate
    do_validate = not args.no_validate
    got = None
    if do_validate and rank == 0:  # a host copy, before the renderer closes
        got = frame.cpu().numpy() if frame is not None else r.read_framebuffer()
    # close before validate(): libvcrt keeps one renderer per process, and validate() opens
    # its own (a second vcrt_begin would end this one, communicator included)
    r.close()
    validated = validate(args, got, st, device, world) if got is not None else None

    if rank == 0:
        samples = args.width * args.height * args.spp * args.steps
        value = samples / elapsed / 1e6
        k_ms = sum(kernel_ms) / len(kernel_ms)
        seg = sum(segments) / len(segments)
        kernel = st["kernel"]  # the symbol the timed frames launched (vcrt_stats.kernel)
        # Issued work of the timed kernel (the roofline numerator): every lane of each
        # wave-level exact group test (4 spheres x 23 flops, functions.glsl:15-19) and box test
        # (27 flops, FLOPS_PER_BOUND_TEST), counted by in-kernel per-wave counters; the linear
        # scans issue the reference's whole scan.
        ref_flops = seg * nspheres * FLOPS_PER_SPHERE_TEST  # brute-force scan, SURVEY.md 8(d)
        issued = ref_flops
        if st["kernel_variant"] in (3, 4, 5):
            issued = (st["group_tests"] * 64 * 4 * FLOPS_PER_SPHERE_TEST
                      + st["bound_tests"] * 64 * FLOPS_PER_BOUND_TEST)
        achieved = issued / (k_ms * 1e-3) / 1e12
        # HBM bytes and VALU counters of this kernel at this workload, from the committed
        # rocprofv3 PMC passes (tools/gpu_profile.sh -> profiles/traffic.json); used only when
        # the profiled kernel is the one this run launched
        key = f"{args.scene}_{args.width}x{args.height}_s{args.spp}_d{args.depth}_n{world}"
        prof = {}
        if os.path.exists(PROFILE_TRAFFIC):
            try:
                prof = json.load(open(PROFILE_TRAFFIC)).get(key, {})
            except (OSError, ValueError):
                prof = {}
        if prof.get("kernel") != kernel:
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
            "warmup_extra": extra,
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
                       "gather": gather,
                       "accumulate_quantum": st["accumulate_quantum"],
                       "accumulate_chunk": st["accumulate_chunk"],
                       "accumulate_tail": [st["accumulate_tail"], st["accumulate_tail_chunk"]],
                       "kernel_variant": st["kernel_variant"],
                       "grid_blocks": st["grid_blocks"],
                       "cost_order": st.get("cost_order", 0)},
            # fp32 VALU-bound (no MFMA). achieved = the fp32 work the timed
            # kernel issued (exact sphere tests and box tests, per-wave counters) / its
            # HIP-event time, so frac <= 1 is a roofline fraction. The brute-force equivalent
            # (segments x spheres x 23: the reference's linear scan of every segment this
            # launch traced) is reported as a speed-up beside it.
            "roofline": {"bound": "valu", "achieved": round(achieved, 3),
                         "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                         "peak_nonfma": PEAK_FP32_NONFMA_TFLOPS,
                         "frac_nonfma": round(achieved / PEAK_FP32_NONFMA_TFLOPS, 4),
                         "traffic": prof.get("hbm_bytes_per_launch"),
                         "kernel": kernel, "kernel_ms": round(k_ms, 3),
                         "numerator": "issued fp32 work per launch: wave-level exact group "
                                      "tests x 64 lanes x 4 x 23 + box tests x 64 x 27 "
                                      "(in-kernel counters; DESIGN.md 7)",
                         "issued_flops_per_launch": issued,
                         "segments_per_launch": int(seg),
                         "bruteforce_flops_per_launch": ref_flops,
                         "speedup_vs_bruteforce_at_peak": round(
                             ref_flops / (PEAK_FP32_TFLOPS * 1e12) / (k_ms * 1e-3), 3),
                         "valu_issue_frac": prof.get("valu_issue_frac"),
                         "valu_lane_util": prof.get("valu_lane_util"),
                         "effective_clock_ghz": prof.get("effective_clock_ghz"),
                         "profile": prof.get("source")},
            "gather_ms": round(sum(gather_ms) / len(gather_ms), 3),
            "per_rank_kernel_ms": {"min": round(min(rank_ms), 3), "max": round(max(rank_ms), 3),
                                   "ranks": [round(v, 3) for v in rank_ms]},
        }
        if validated is not None:
            out["validated"] = validated
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
