"""GPU parity at BASELINE.json's own workloads (configs C1-C5 at their exact width x height,
samples per pixel, depth and scene), through the C ABI, against the CPU oracle.

The HIP path renders every config's full frame. The oracle (a linear scan in C) cannot render
a 1024-spp 1080p frame in seconds, so each config is compared on a subset the CPU affords, at
the config's full spp and depth:
  C1  256x144, 1 spp, depth 1, red scene          whole frame
  C2  800x450, 64 spp, depth 8, three-material     whole frame
  C3  1920x1080, 256 spp, depth 10, final scene    8 rows spread over the frame
  C4  1920x1080, 1024 spp, depth 10, final scene   8 rows; also sharded 8 ways
  C5  3840x2160, 4096 spp, depth 50, 4100 spheres  64 pixels on an 8x8 grid
Bar: bit-identical to the oracle on the subset (same accumulation chunk, read back through the
ABI), per-channel RMS <= 1e-4 against the reference's sequential fp32 sum (north_star), and
whole-frame properties (alpha 1, finite, radiance in [0, 1] for these scenes, segment counts
between one and `depth` per sample). Reference loops: shader.comp:46-56, functions.glsl:73-91.
"""
import numpy as np
import pytest

import vulkancomputeraytracing_amd as vc

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-4  # north_star: per-channel RMS <= 1e-4 vs the reference

CONFIGS = {  # BASELINE.json configs, SURVEY.md 8(d)
    "c1": ("red", 256, 144, 1, 1),
    "c2": ("three", 800, 450, 64, 8),
    "c3": ("final", 1920, 1080, 256, 10),
    "c4": ("final", 1920, 1080, 1024, 10),
    "c5": ("stress4096", 3840, 2160, 4096, 50),
}


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def render_full(name, **kw):
    scene, w, h, spp, depth = CONFIGS[name]
    desc = vc.RenderDesc(width=w, height=h, samples_per_pixel=spp, max_depth=depth, device=0,
                         **kw)
    with vc.Renderer(desc, scene) as r:
        r.draw_next_frame()
        return r.read_framebuffer(), r.stats()


def frame_properties(img, st, name):
    scene, w, h, spp, depth = CONFIGS[name]
    assert img.shape == (h, w, 4)
    assert np.all(img[..., 3] == 1.0)
    rgb = img[..., :3]
    assert np.all(np.isfinite(rgb))
    # sky <= 1 and every attenuation <= 1 in these scenes: radiance in [0, 1]
    assert np.all(rgb >= 0.0) and np.all(rgb <= 1.0)
    assert st["samples"] == w * h * spp
    assert w * h * spp <= st["segments"] <= w * h * spp * depth


def check_subset(got, want, what):
    if not np.array_equal(bits(got), bits(want)):
        bad = np.argwhere(bits(got) != bits(want))
        raise AssertionError(f"{what}: {len(bad)} words differ, first {bad[:5].tolist()}")


def rms(a, b):
    d = a.astype(np.float64)[..., :3] - b.astype(np.float64)[..., :3]
    return np.sqrt((d.reshape(-1, 3) ** 2).mean(axis=0))


@pytest.mark.parametrize("name", ["c1", "c2"])
def test_small_configs_whole_frame(oracle, name):
    scene, w, h, spp, depth = CONFIGS[name]
    got, st = render_full(name)
    frame_properties(got, st, name)
    want, segs = oracle.render(oracle.config(w, h, spp, depth, **oracle.partition(st)),
                               oracle.scene(scene))
    check_subset(got, want, name)
    assert st["segments"] == segs
    seq, _ = oracle.render(oracle.config(w, h, spp, depth), oracle.scene(scene))
    assert np.all(rms(got, seq) <= RMS_TOL)


@pytest.mark.parametrize("name", ["c3", "c4"])
def test_final_scene_configs_row_subset(oracle, name):
    scene, w, h, spp, depth = CONFIGS[name]
    got, st = render_full(name)
    frame_properties(got, st, name)
    rows = range(67, h, 135)  # 8 rows: sky, the sphere field, the ground
    sel = list(rows)
    assert len(sel) == 8
    cfg = oracle.config(w, h, spp, depth, **oracle.partition(st))
    want, _ = oracle.render(cfg, oracle.scene(scene), rows=rows)
    check_subset(got[sel], want[sel], f"{name} rows {sel}")
    seq, _ = oracle.render(oracle.config(w, h, spp, depth), oracle.scene(scene), rows=rows)
    assert np.all(rms(got[sel], seq[sel]) <= RMS_TOL)
    # the subset saw every material and the sky
    assert got[sel][..., 2].max() > 0.9 and got[sel][..., 0].min() < 0.2


def test_c4_sharded_eight_ways_equals_one_gpu(oracle):
    """C4's 8-GPU decomposition rendered rank by rank on one GPU: every rank's tiles, gathered
    and re-interleaved by vcrt_assemble, give the 1-GPU frame with the same accumulation chunk
    bit for bit (chunk sums are combined exactly, in whatever order the ranks finish them)."""
    import torch
    from vulkancomputeraytracing_amd import distributed as D
    scene, w, h, spp, depth = CONFIGS["c4"]
    world = 8
    d8 = vc.RenderDesc(width=w, height=h, samples_per_pixel=spp, world_size=world)
    k8 = vc.renderer.work_chunk(d8)
    t8, kt8 = vc.renderer.work_tail(d8)
    assert (k8, t8, kt8) == (16, 128, 4)
    # the 8-way default partition (head chunk and tail) on one GPU
    full, st1 = render_full("c4", accumulate_chunk=k8, accumulate_tail=t8,
                            accumulate_tail_chunk=kt8)
    pad = D.tiles_per_rank(w, h, world)
    gathered = torch.zeros((world * pad * 64, 4), dtype=torch.float32, device="cuda:0")
    segs = 0
    for rank in range(world):
        desc = vc.RenderDesc(width=w, height=h, samples_per_pixel=spp, max_depth=depth,
                             device=0, rank=rank, world_size=world)  # default chunk: k8
        with vc.Renderer(desc, scene) as r:
            assert oracle.partition(r.stats()) == oracle.partition(st1)
            r.set_framebuffer_device(gathered[rank * pad * 64:].data_ptr(), pad * 64 * 16)
            r.draw_next_frame()
            segs += r.stats()["segments"]
            torch.cuda.synchronize()
            if rank == world - 1:
                frame = torch.empty((h, w, 4), dtype=torch.float32, device="cuda:0")
                r.assemble_tiles(gathered.data_ptr(), frame.data_ptr(), pad)
                torch.cuda.synchronize()
    check_subset(frame.cpu().numpy(), full, "c4 8-way shards vs 1 GPU")
    assert segs == st1["segments"]


def test_c5_stress_pixel_grid(oracle):
    scene, w, h, spp, depth = CONFIGS["c5"]
    got, st = render_full("c5")
    frame_properties(got, st, "c5")
    assert st["nspheres"] == 4100
    xs = np.linspace(17, w - 23, 8).astype(int)
    ys = np.linspace(31, h - 11, 8).astype(int)
    xy = [(int(x), int(y)) for y in ys for x in xs]
    cfg = oracle.config(w, h, spp, depth, **oracle.partition(st))
    want, _ = oracle.render_pixels(cfg, oracle.scene(scene), xy)
    sub = np.stack([got[y, x] for x, y in xy])
    check_subset(sub, want, "c5 8x8 pixel grid")
    seq, _ = oracle.render_pixels(oracle.config(w, h, spp, depth), oracle.scene(scene), xy)
    assert np.all(rms(sub, seq) <= RMS_TOL)
