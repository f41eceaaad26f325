"""Seeded random configurations, bit for bit against the oracle (GPU).

Each case draws a scene (clusters with nested, duplicate and hollow spheres, RTIOW-style grids,
spheres on a line, scenes scaled far from unit size, a camera inside a glass sphere), a camera,
a ragged frame size, spp, depth, kernel variant, work partition / quantum, an optional rank of a
sharded frame and an optional second progressive frame. The product path (through the C ABI)
must give the oracle's bits for every pixel it renders, and its segment count on one GPU. The
reference loop these restate is shader.comp:42-57 over functions.glsl:65-92; the cases only
widen the inputs the fixed-configuration tests (test_gpu_parity.py) cover.
"""
import os

import numpy as np
import pytest

import vulkancomputeraytracing_amd as vc
from vulkancomputeraytracing_amd import _native as N

from tests.test_gpu_parity import assert_bitwise

pytestmark = pytest.mark.gpu

VARIANTS = [vc.KERNEL_AUTO, vc.KERNEL_LDS, vc.KERNEL_SMEM, vc.KERNEL_CULL, vc.KERNEL_CULL_LANE,
            vc.KERNEL_CULL_FLAT]


def _material(rng):
    m = int(rng.integers(1, 4))
    param = {1: rng.uniform(0.0, 1.2), 2: rng.uniform(0.0, 1.0), 3: rng.uniform(1.1, 2.4)}[m]
    return m, float(param)


def _cluster(rng, n, spread):
    rows = [((0.0, -1000.0, 0.0), 1000.0, (0.5, 0.5, 0.5), 1, 1.0)]
    for i in range(n - 1):
        c = tuple(float(v) for v in rng.uniform(-spread, spread, 3))
        r = float(np.exp(rng.uniform(np.log(1e-3), np.log(0.3 * spread + 0.1))))
        m, p = _material(rng)
        rows.append((c, r, tuple(float(v) for v in rng.uniform(0, 1, 3)), m, p))
        if i % 7 == 3:  # exact duplicate, other material: the lower index must win ties
            rows.append((c, r, (1.0, 0.0, 0.0), 1 + m % 3, 0.5))
        if i % 11 == 5:  # hollow glass shell inside it
            rows.append((c, -0.8 * r, (1.0, 1.0, 1.0), 3, 1.5))
    return rows


def _line(rng, n):
    # every centre on one line: degenerate (flat) hierarchy boxes
    return [((float(x), 0.5, 0.0), float(rng.uniform(0.05, 0.45)),
             tuple(float(v) for v in rng.uniform(0, 1, 3)), *_material(rng))
            for x in np.linspace(-6, 6, n)]


def make_case(oracle, seed, bright=False, big=False):
    rng = np.random.default_rng((3000 if big else 2000 if bright else 1000) + seed)
    kind = "big" if big else ["cluster", "cluster", "grid", "line", "scaled", "inside"][seed % 6]
    look = (0.0, 0.5, 0.0)
    if kind == "big":  # many hierarchy chunks; tables beyond LDS (boxes-only and global kernels)
        rows = _cluster(rng, int(rng.integers(600, 5000)), 20.0)
        eye = tuple(float(v) for v in rng.uniform(-25, 25, 3))
        eye = (eye[0], abs(eye[1]) + 0.5, eye[2])
        look = tuple(float(v) for v in rng.uniform(-5, 5, 3))
    elif kind == "cluster":
        rows = _cluster(rng, int(rng.integers(3, 400)), 3.0)
        eye = tuple(float(v) for v in rng.uniform(-10, 10, 3))
        eye = (eye[0], abs(eye[1]) + 0.5, eye[2] + 12.0)
    elif kind == "grid":  # the reference generator's rules on a random grid size
        o = oracle
        half = int(rng.integers(2, 12))
        sc = np.concatenate([o.random_spheres(-half, half), o.big_three_and_ground()])
        rows = None
        eye, look = (13.0, 2.0, 3.0), (0.0, 0.0, 0.0)
    elif kind == "line":
        rows = _line(rng, int(rng.integers(16, 120)))
        eye = (float(rng.uniform(-3, 3)), float(rng.uniform(0.5, 4)), 9.0)
    elif kind == "scaled":  # the same kind of cluster, far from unit scale
        s = float(10.0 ** rng.uniform(-2, 3))
        rows = [((c[0] * s, c[1] * s, c[2] * s), r * s, col, m, p)
                for c, r, col, m, p in _cluster(rng, int(rng.integers(16, 200)), 3.0)]
        eye, look = (4.0 * s, 3.0 * s, 12.0 * s), (0.0, 0.5 * s, 0.0)
    else:  # the camera inside a big glass sphere among others
        rows = _cluster(rng, int(rng.integers(16, 120)), 3.0)
        rows.append(((0.0, 1.0, 6.0), 3.0, (1.0, 1.0, 1.0), 3, float(rng.uniform(1.1, 1.9))))
        eye = (0.0, 1.0, 6.5)
    if bright and rows is not None:
        # Lambertian "reflect ratios" above 1 (textures.glsl:22 multiplies them in): radiance
        # grows with depth, so quantum sums leave the 2^32 scale and the per-pixel scale and
        # the re-render run (vcrt_math.h "Accumulation")
        rows = [(c, r, tuple(0.7 + 0.3 * v for v in col), m, float(rng.uniform(3.0, 4.5)))
                if m == 1 else (c, r, col, m, p) for c, r, col, m, p in rows]
    if rows is not None:
        sc = vc.make_spheres(rows)
    w, h = int(rng.integers(1, 161)), int(rng.integers(1, 97))
    spp, depth = int(rng.integers(1, 25)), int(rng.integers(1, 41))
    if big:  # (the oracle's linear scan: small frames)
        w, h, spp = int(rng.integers(1, 49)), int(rng.integers(1, 33)), int(rng.integers(1, 5))
    variant = VARIANTS[int(rng.integers(0, len(VARIANTS)))]
    chunk = quantum = 0
    if rng.uniform() < 0.5:
        quantum = int(2 ** rng.integers(0, 3))
        chunk = quantum * int(rng.integers(1, 4))
    world = [1, 1, 1, 2, 3, 8][int(rng.integers(0, 6))]
    rank = int(rng.integers(0, world))
    frames = 2 if rng.uniform() < 0.25 else 1
    vup = (0.0, 1.0, 0.0) if rng.uniform() < 0.7 else tuple(float(v) for v in rng.uniform(-1, 1, 3))
    if abs(float(np.dot(vup, np.subtract(eye, look)))) > 0.99 * float(
            np.linalg.norm(vup) * np.linalg.norm(np.subtract(eye, look))):
        vup = (0.0, 1.0, 0.0)  # (vup parallel to the view axis: no camera basis)
    cam = dict(lookfrom=eye, lookat=look, vup=vup, vfov=float(rng.uniform(8, 100)))
    return dict(kind=kind, scene=sc, w=w, h=h, spp=spp, depth=depth, variant=variant,
                chunk=chunk, quantum=quantum, world=world, rank=rank, frames=frames, cam=cam)


def check_case(oracle, c, seed):
    what = (f"seed {seed} {c['kind']} n{len(c['scene'])} {c['w']}x{c['h']} spp{c['spp']} "
            f"d{c['depth']} v{c['variant']} k{c['chunk']}/q{c['quantum']} "
            f"rank {c['rank']}/{c['world']} frames {c['frames']}")
    desc = vc.RenderDesc(width=c["w"], height=c["h"], samples_per_pixel=c["spp"],
                         max_depth=c["depth"], kernel_variant=c["variant"], device=0,
                         rank=c["rank"], world_size=c["world"], accumulate_chunk=c["chunk"],
                         accumulate_quantum=c["quantum"], progressive=c["frames"] > 1,
                         **c["cam"])
    with vc.Renderer(desc, c["scene"]) as r:
        for _ in range(c["frames"]):
            r.draw_next_frame()
        got, st = r.read_framebuffer(), r.stats()
    spp_total = c["spp"] * c["frames"]
    cfg = oracle.config(c["w"], c["h"], spp_total, c["depth"], **oracle.partition(st),
                        frame_spp=c["spp"] if c["frames"] > 1 else 0, **c["cam"])
    want, segs = oracle.render(cfg, c["scene"])
    if c["world"] == 1:
        assert_bitwise(got, want, what)
        if c["frames"] == 1:
            assert st["segments"] == segs, what
    else:
        m = vc.tile_pixel_map(c["w"], c["h"], c["world"])
        mine = m[..., 0] == c["rank"]
        ntiles = len(vc.tiles_for_rank(c["w"], c["h"], c["world"], c["rank"]))
        assert got.shape == (ntiles, 64, 4), what
        if mine.any():
            assert_bitwise(got.reshape(-1, 4)[m[..., 1][mine]], want[mine], what)
    return st


@pytest.mark.parametrize("seed", range(120))
def test_random_configuration_bitwise(oracle, seed):
    check_case(oracle, make_case(oracle, seed), seed)


@pytest.mark.parametrize("seed", range(24))
def test_random_large_scene_configuration_bitwise(oracle, seed):
    check_case(oracle, make_case(oracle, seed, big=True), seed)


def test_random_bright_configurations_bitwise(oracle):
    """40 of the cases with bright Lambertians (albedo 0.7-1, ratio 3-4.5, the ground too): the
    pixels whose quantum sums leave the first scale re-render at their own (vcrt_math.h
    "Accumulation"), on every variant, partition, rank and progressive frame; several cases
    must take that path."""
    rerenders = 0
    for seed in range(40):
        c = make_case(oracle, seed, bright=True)
        c["depth"] = max(c["depth"], 16)
        rerenders += check_case(oracle, c, seed)["scale_rerenders"] > 0
    assert rerenders >= 3, rerenders


@pytest.mark.parametrize("w,h,spp,depth", [(65535, 3, 2, 4),     # the widest frame (x in 16 bits)
                                           (5, 65535, 2, 4),     # the tallest
                                           (8192, 8192, 8, 3)])  # 2^26 pixels, summed quanta
def test_extreme_frame_shapes_bitwise(oracle, w, h, spp, depth):
    """Frames at the C ABI's size limits (vcrt.h: width, height <= 65535, <= 2^26 pixels in a
    rank's tiles): rows spread over the frame, bitwise against the oracle's render of the same
    rows; one tile more than 2^26 pixels is refused at vcrt_begin."""
    desc = vc.RenderDesc(width=w, height=h, samples_per_pixel=spp, max_depth=depth, device=0)
    with vc.Renderer(desc, "final") as r:
        r.draw_next_frame()
        got, st = r.read_framebuffer(), r.stats()
    assert got.shape == (h, w, 4)
    cfg = oracle.config(w, h, spp, depth, **oracle.partition(st))
    for y in sorted({0, h // 3, h // 2, h - 1}):
        xy = np.stack([np.arange(w), np.full(w, y)], axis=1)
        want, _ = oracle.render_pixels(cfg, oracle.scene("final"), xy)
        assert_bitwise(got[y], want, f"{w}x{h} row {y}")


def test_frame_beyond_the_slot_limit_is_refused():
    # 8200 x 8192: 1025 x 1024 tiles of 64 slots > 2^26 (vcrt.h vcrt_render_desc)
    desc = vc.RenderDesc(width=8200, height=8192, samples_per_pixel=8, max_depth=3, device=0)
    with pytest.raises(vc.VcrtError) as e:
        with vc.Renderer(desc, "final"):
            pass
    assert e.value.code == N.VK_ERROR_FORMAT_NOT_SUPPORTED
    # the same frame in four shards fits every rank
    with vc.Renderer(vc.RenderDesc(width=8200, height=8192, samples_per_pixel=1, max_depth=1,
                                   device=0, rank=3, world_size=4), "final") as r:
        r.draw_next_frame()


def _same_bits_or_both_nan(got, want, what):
    g, w = np.asarray(got, np.float32), np.asarray(want, np.float32)
    both_nan = np.isnan(g) & np.isnan(w)
    gb, wb = g.view(np.uint32).copy(), w.view(np.uint32).copy()
    gb[both_nan] = wb[both_nan] = 0
    assert_bitwise(gb.view(np.float32), wb.view(np.float32), what)


@pytest.mark.parametrize("case", ["huge_radius", "nan_centre", "zero_radius", "wide_fov",
                                  "narrow_fov", "eye_on_target", "many_samples", "deep"])
def test_edge_inputs_bitwise(oracle, case):
    """Inputs at the edge of the reference's arithmetic: a sphere too large for the culling
    guard (the linear scan then), a NaN centre (never hit), a zero radius, fields of view of 170
    and 0.5 degrees, the camera on its target (normalize(0) gives a NaN basis; hit_sphere's
    `disc < 0` rejection lets a NaN ray through, so every segment "hits" and the path ends at
    the depth limit with the canonical black), 2^16 samples (quantum 128: 512 quanta per pixel)
    and depth 500."""
    rows = [((0.0, -1000.0, 0.0), 1000.0, (0.5, 0.5, 0.5), 1, 1.0),
            ((0.0, 1.0, 0.0), 1.0, (1.0, 1.0, 1.0), 3, 1.5),
            ((-4.0, 1.0, 0.0), 1.0, (0.4, 0.2, 0.1), 1, 1.0),
            ((4.0, 1.0, 0.0), 1.0, (0.7, 0.6, 0.5), 2, 0.0)]
    rng = np.random.default_rng(7)
    for i in range(20):
        rows.append(((float(rng.uniform(-6, 6)), 0.2, float(rng.uniform(-6, 6))), 0.2,
                     tuple(float(v) for v in rng.uniform(0, 1, 3)), 1 + i % 3, 0.5))
    cam = dict(lookfrom=(13.0, 2.0, 3.0), lookat=(0.0, 0.0, 0.0), vfov=20.0)
    w, h, spp, depth = 48, 27, 4, 10
    if case == "huge_radius":
        rows.append(((0.0, 0.0, -3e9), 2.9e9, (0.9, 0.9, 0.9), 1, 0.8))
    elif case == "nan_centre":
        rows.append(((float("nan"), 1.0, 0.0), 0.5, (1.0, 0.0, 0.0), 1, 1.0))
    elif case == "zero_radius":
        rows.append(((1.0, 0.5, 1.0), 0.0, (1.0, 0.0, 0.0), 2, 0.0))
    elif case == "wide_fov":
        cam["vfov"] = 170.0
    elif case == "narrow_fov":
        cam["vfov"] = 0.5
    elif case == "eye_on_target":
        cam["lookat"] = cam["lookfrom"]
    elif case == "many_samples":
        w, h, spp, depth = 3, 2, 1 << 16, 6
    elif case == "deep":
        w, h, spp, depth = 16, 9, 4, 500
    sc = vc.make_spheres(rows)
    desc = vc.RenderDesc(width=w, height=h, samples_per_pixel=spp, max_depth=depth, device=0,
                         **cam)
    with vc.Renderer(desc, sc) as r:
        r.draw_next_frame()
        got, st = r.read_framebuffer(), r.stats()
    want, segs = oracle.render(oracle.config(w, h, spp, depth, **oracle.partition(st), **cam), sc)
    _same_bits_or_both_nan(got, want, case)
    assert st["segments"] == segs
    if case == "eye_on_target":  # every NaN ray "hits" and its path ends at the depth limit
        assert segs == w * h * spp * depth and (got[..., :3] == 0).all()


def test_progressive_limit_is_refused_cleanly(oracle):
    """Progressive frames add quanta to each pixel's exact sums, at most 512 (vcrt_math.h
    kAccumMaxChunks): with 64 spp in quanta of 4, frame 33 is refused, and the frame read back
    is still frame 32's, equal to the oracle's 2048-sample image."""
    w, h, spp, depth = 16, 9, 64, 6
    desc = vc.RenderDesc(width=w, height=h, samples_per_pixel=spp, max_depth=depth, device=0,
                         progressive=True)
    with vc.Renderer(desc, "final") as r:
        k = oracle.partition(r.stats())
        for _ in range(32):
            r.draw_next_frame()
        with pytest.raises(vc.VcrtError) as e:
            r.draw_next_frame()
        assert e.value.code == N.VK_ERROR_FORMAT_NOT_SUPPORTED
        got = r.read_framebuffer()
        assert r.stats()["accumulated_spp"] == 32 * spp
    want, _ = oracle.render(oracle.config(w, h, 32 * spp, depth, **k, frame_spp=spp),
                            oracle.scene("final"))
    assert_bitwise(got, want, "frame 32")


def test_scene_switch_and_reset_on_a_large_frame(oracle):
    """A 4096 x 2304 progressive renderer (600 MB of sums): two frames of the final scene, a
    switch to the three-sphere scene (another kernel; the sums restart), a frame, a reset and a
    frame of the final scene again: each read-back equals the oracle on spread rows (the
    stream-ordered resets of this round: a reset still running under a frame would zero some
    of its pixels)."""
    w, h, spp, depth = 4096, 2304, 8, 4
    desc = vc.RenderDesc(width=w, height=h, samples_per_pixel=spp, max_depth=depth, device=0,
                         progressive=True)
    rows = [0, 777, 1500, h - 1]

    def check(got, scene, frames, what, k):
        cfg = oracle.config(w, h, frames * spp, depth, **k, frame_spp=spp)
        for y in rows:
            xy = np.stack([np.arange(w), np.full(w, y)], axis=1)
            want, _ = oracle.render_pixels(cfg, oracle.scene(scene), xy)
            assert_bitwise(got[y], want, f"{what} row {y}")

    with vc.Renderer(desc, "final") as r:
        k = oracle.partition(r.stats())
        r.draw_next_frame()
        r.draw_next_frame()
        check(r.read_framebuffer(), "final", 2, "final x2", k)
        r.set_scene(oracle.scene("three"))
        r.draw_next_frame()
        assert r.stats()["kernel"].startswith("vcrt_trace_smem")
        check(r.read_framebuffer(), "three", 1, "three", k)
        r.set_scene(oracle.scene("final"))
        r.draw_next_frame()
        r.reset_accumulation()
        r.draw_next_frame()
        check(r.read_framebuffer(), "final", 1, "final after reset", k)


def test_a_replaced_renderer_is_stale(oracle):
    """libvcrt holds one renderer per process (vcrt.h): a second Renderer's vcrt_begin ends the
    first. The first object then raises instead of acting on the second's state, and closing it
    leaves the second running."""
    d = vc.RenderDesc(width=24, height=16, samples_per_pixel=2, max_depth=5, device=0)
    r1 = vc.Renderer(d, "final")
    r2 = vc.Renderer(d, "three")
    with pytest.raises(vc.VcrtError):
        r1.draw_next_frame()
    r1.close()
    r2.draw_next_frame()
    got, st = r2.read_framebuffer(), r2.stats()
    r2.close()
    with pytest.raises(vc.VcrtError):
        r2.stats()
    want, _ = oracle.render(oracle.config(24, 16, 2, 5, **oracle.partition(st)),
                            oracle.scene("three"))
    assert_bitwise(got, want, "second renderer")


def test_progressive_cost_order_across_a_code_object_reload(oracle, monkeypatch):
    """A progressive renderer on the cost order (forced), whose code object is reloaded between
    frames: the reload re-keys the block order, so the next frame measures again while it adds
    to the same sums -- three frames equal the oracle's 3 x spp image, bit for bit."""
    monkeypatch.setenv("VCRT_WORK_ORDER", "cost")
    w, h, spp, depth = 72, 40, 6, 12
    desc = vc.RenderDesc(width=w, height=h, samples_per_pixel=spp, max_depth=depth, device=0,
                         progressive=True)
    with vc.Renderer(desc, "final") as r:
        k = oracle.partition(r.stats())
        r.draw_next_frame()
        r.draw_next_frame()
        assert r.stats()["cost_order"] == 1
        r.shader_load(N.CODE_OBJECT_PATH)
        r.draw_next_frame()
        got, st = r.read_framebuffer(), r.stats()
    assert st["accumulated_spp"] == 3 * spp
    want, _ = oracle.render(oracle.config(w, h, 3 * spp, depth, **k, frame_spp=spp),
                            oracle.scene("final"))
    assert_bitwise(got, want, "3 progressive frames around a reload")


def test_srgb8_encode_edge_values_bitwise(oracle):
    """vcrt_encode_srgb8 on every kind of float the framebuffer can hold, through an external
    device framebuffer: each of the 255 thresholds and its neighbouring floats, values below 0 and
    above 1, -0, denormals, +-inf and NaN -- against the oracle's encoder byte for byte."""
    import torch
    th = np.zeros(255, dtype=np.float32)
    N.lib().vcrt_srgb8_thresholds(th.ctypes.data)
    vals = [th, np.nextafter(th, np.float32(-1)), np.nextafter(th, np.float32(2)),
            np.float32([0.0, -0.0, 1.0, 1e-45, -1e-45, 1e-38, -1.0, 2.0, 1e30, -1e30,
                        np.inf, -np.inf, np.nan]),
            np.random.default_rng(3).uniform(-0.5, 1.5, 4096).astype(np.float32)]
    v = np.concatenate(vals).astype(np.float32)
    w = 64
    h = (len(v) + 4 * w - 1) // (4 * w)
    flat = np.ones(w * h * 4, dtype=np.float32)
    flat[:len(v)] = v
    img = flat.reshape(h, w, 4)
    desc = vc.RenderDesc(width=w, height=h, samples_per_pixel=1, max_depth=1, device=0)
    buf = torch.from_numpy(img.copy()).to("cuda:0")
    with vc.Renderer(desc, "red") as r:
        r.set_framebuffer_device(buf.data_ptr(), buf.numel() * 4)
        torch.cuda.synchronize()
        got = r.read_framebuffer_srgb8()
    assert np.array_equal(got, oracle.encode_srgb8(img))


def _read_ppm(path):
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(b"\n", 3)
    assert parts[0] == b"P6" and parts[2] == b"255"
    w, h = (int(v) for v in parts[1].split())
    return np.frombuffer(parts[3], dtype=np.uint8, count=w * h * 3).reshape(h, w, 3)


@pytest.mark.parametrize("scene,w,h,spp,depth,frames,progressive,fmt", [
    ("three", 97, 41, 6, 9, 2, 1, "ppm"),
    ("final", 64, 36, 12, 10, 3, 1, "pfm"),
    ("red", 33, 70, 3, 4, 2, 0, "ppm"),
    ("stress4096", 48, 27, 2, 20, 1, 0, "pfm"),
])
def test_cpp_host_api_configurations(oracle, tmp_path, scene, w, h, spp, depth, frames,
                                     progressive, fmt):
    """bin/vcrt_render (the C++ Begin / Draw / End of Renderer.hpp:14-20 with
    SetRenderDescription / SetRenderScene) on several scenes, sizes and progressive frame counts,
    writing PFM (linear) or PPM (sRGB8 encoded on the GPU): the files equal the oracle's image
    (progressive: frames x spp samples) and its sRGB8 encoding."""
    import subprocess
    from tests.test_gpu_configs import read_pfm
    out = tmp_path / f"frame.{fmt}"
    cmd = [os.path.join(N.BIN_DIR, "vcrt_render"), "--scene", scene, "--width", str(w),
           "--height", str(h), "--spp", str(spp), "--depth", str(depth), "--frames",
           str(frames), "--progressive", str(progressive), "--out", str(out)]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stderr
    q = vc.renderer.work_quantum(vc.RenderDesc(width=w, height=h, samples_per_pixel=spp,
                                               max_depth=depth, progressive=bool(progressive)))
    total = spp * (frames if progressive else 1)
    want, _ = oracle.render(oracle.config(w, h, total, depth, quantum=q,
                                          frame_spp=spp if progressive else 0),
                            oracle.scene(scene))
    if fmt == "pfm":
        assert_bitwise(read_pfm(out), want[..., :3], f"{scene} pfm")
    else:
        assert np.array_equal(_read_ppm(out), oracle.encode_srgb8(want)[..., :3])


def test_cpp_host_api_unwritable_output_fails(tmp_path):
    import subprocess
    res = subprocess.run([os.path.join(N.BIN_DIR, "vcrt_render"), "--scene", "red", "--width",
                          "16", "--height", "16", "--out", str(tmp_path / "no" / "x.ppm")],
                         capture_output=True, text=True, timeout=120)
    assert res.returncode == 1 and "cannot write" in res.stderr


@pytest.mark.parametrize("fetch", [None, ("1", "0"), ("16", "4")])
def test_deferred_fetch_keeps_bits(oracle, monkeypatch, fetch):
    """The flat scan's deferred fetch (the LDS-table scan waits for 4 lanes by default) only
    changes when lanes start their items: the default, immediate fetches and long deferrals give
    the oracle's bits and segment counts."""
    if fetch is not None:
        monkeypatch.setenv("VCRT_FETCH_MIN", fetch[0])
        monkeypatch.setenv("VCRT_FETCH_WAIT", fetch[1])
    w, h, spp, depth = 160, 90, 16, 10
    desc = vc.RenderDesc(width=w, height=h, samples_per_pixel=spp, max_depth=depth, device=0)
    with vc.Renderer(desc, "final") as r:
        r.draw_next_frame()
        got, st = r.read_framebuffer(), r.stats()
    assert st["kernel"].startswith("vcrt_trace_cull_flat")
    want, segs = oracle.render(oracle.config(w, h, spp, depth, **oracle.partition(st)),
                               oracle.scene("final"))
    assert_bitwise(got, want, f"fetch {fetch}")
    assert st["segments"] == segs
