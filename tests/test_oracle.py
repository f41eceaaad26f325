"""The CPU oracle pinned against the reference: SceneGenerator output (golden vectors from the
reference's own SceneGenerator.cpp compiled here), math KATs and the camera scalars, plus the
committed oracle images (regression pins). SURVEY.md section 8(c)."""
import hashlib
import json
import os

import numpy as np
import pytest

from tests import oracle_py

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def golden_meta():
    with open(os.path.join(GOLDEN, "scene_generator_stdout.json")) as f:
        return json.load(f)


def test_scene_generator_text_matches_reference_hash(oracle):
    text = oracle.scene_generator_text()
    meta = golden_meta()
    assert len(text) == meta["bytes"]
    assert hashlib.sha256(text).hexdigest() == meta["sha256"]


@pytest.mark.skipif(not os.path.exists(oracle_py.REF_SCENEGEN),
                    reason="reference SceneGenerator not built (needs /root/reference)")
def test_scene_generator_text_matches_reference_binary(oracle):
    import subprocess
    ref = subprocess.run([oracle_py.REF_SCENEGEN], capture_output=True, check=True).stdout
    assert oracle.scene_generator_text() == ref


def test_scene_spheres_match_reference_values(oracle):
    want = np.load(os.path.join(GOLDEN, "scene_generator_spheres.npy"))
    got = oracle.random_spheres(-11, 11)
    assert len(got) == len(want) == 481
    flat = np.concatenate([got["center"], got["radius"][:, None], got["colour"],
                           got["texture"]], axis=1)
    assert np.array_equal(flat.view(np.uint32), want.view(np.uint32))
    # counts from SURVEY.md 3.4: 371 Lambertian, 74 metal, 36 glass
    kinds = got["texture"][:, 0]
    assert (kinds == 1).sum() == 371 and (kinds == 2).sum() == 74 and (kinds == 3).sum() == 36


def test_scene_sizes(oracle):
    assert len(oracle.scene("final")) == 485
    assert len(oracle.scene("three")) == 4
    assert len(oracle.scene("red")) == 2
    s = oracle.scene("stress4096")
    assert len(s) == 4100
    # same generator rules on the wider grid: every generated sphere is small and on the floor
    assert np.all(s["radius"][:4096] == np.float32(0.2))
    assert np.all(s["center"][:4096, 1] == np.float32(0.2))


RAND_KAT = [0.0, 0.6875, 0.467773438, 0.068359375, 0.296875, 0.6875, 0.994140625, 0.947265625,
            0.8046875, 0.265625]


def test_rand_known_answers(oracle):
    # rand(i,i) for i=0..9, 1023, 1024 (fp32, no contraction)
    for i, want in enumerate(RAND_KAT):
        assert oracle.rand(float(i), float(i)) == pytest.approx(want, abs=5e-10)
    assert oracle.rand(1023.0, 1023.0) == pytest.approx(0.419921875, abs=5e-10)
    assert oracle.rand(1024.0, 1024.0) == pytest.approx(0.838012695, abs=5e-10)


def _correctly_rounded_sin(x32: np.ndarray) -> np.ndarray:
    return np.sin(x32.astype(np.float64)).astype(np.float32)


@pytest.mark.parametrize("lo,hi", [(-10.0, 10.0), (-1e5, 1e5), (1e5, 1e8), (-3e38, 3e38)])
def test_canonical_sin_is_correctly_rounded(oracle, lo, hi):
    rng = np.random.default_rng(int(abs(lo)) % 1000 + 7)
    if hi > 1e9:
        xs = (rng.standard_normal(20000) * 10.0 ** rng.uniform(-3, 38, 20000)).astype(np.float32)
        xs = xs[np.isfinite(xs)]
    else:
        xs = rng.uniform(lo, hi, 20000).astype(np.float32)
    want = _correctly_rounded_sin(xs)
    got = np.array([oracle.sin(float(x)) for x in xs], dtype=np.float32)
    assert np.array_equal(got, want)


def test_canonical_sin_special_values(oracle):
    assert oracle.sin(0.0) == 0.0
    assert np.isnan(oracle.sin(float("inf")))
    assert np.isnan(oracle.sin(float("nan")))
    # exponent boundary between the two reductions (2^20)
    for x in [2.0 ** 20, np.nextafter(np.float32(2.0 ** 20), np.float32(0)), 2.0 ** 20 + 1]:
        x = float(np.float32(x))
        assert oracle.sin(x) == _correctly_rounded_sin(np.array([x], np.float32))[0]


def test_camera_scalars(oracle):
    cam = oracle.camera(oracle.config(1280, 720, 1, 50))
    # focal=13.490738, vh=vw=4.757562 for every 16:9 config
    assert cam[12] == pytest.approx(13.490738, abs=1e-6)
    assert cam[13] == pytest.approx(4.757562, abs=1e-6)
    assert cam[14] == cam[13]  # integer IMAGE_WIDTH/IMAGE_HEIGHT == 1
    # delta_u divided by H, not W (shader.comp:35): |du| = vw / H
    du = cam[3:6]
    assert np.sqrt((du.astype(np.float64) ** 2).sum()) == pytest.approx(cam[14] / 720, rel=1e-6)


def test_depth_one_red_scene_semantics(oracle):
    # BASELINE config 1 at reduced size: with depth 1 every hit returns the undefined value
    # (canonical 0) and every miss returns the sky term.
    img, segs = oracle.render(oracle.config(64, 36, 1, 1), oracle.scene("red"))
    assert segs == 64 * 36
    assert np.all(img[..., 3] == 1.0)
    rgb = img[..., :3]
    hit = np.all(rgb == 0.0, axis=-1)
    assert 0 < hit.sum() < hit.size
    sky = rgb[~hit]
    assert np.all(sky[:, 2] == 1.0) or np.all(sky > 0)


def test_oracle_images_regression(oracle):
    from tests.golden.make_golden import IMAGES
    data = np.load(os.path.join(GOLDEN, "oracle_images.npz"))
    for name, scene, w, h, spp, depth in IMAGES:
        img, segs = oracle.render(oracle.config(w, h, spp, depth), oracle.scene(scene))
        assert np.array_equal(img.view(np.uint32), data[name].view(np.uint32)), name
        assert segs == int(data[name + "__segments"][0]), name


def test_oracle_row_subset_and_threads_are_deterministic(oracle):
    cfg = oracle.config(40, 24, 2, 6)
    scene = oracle.scene("three")
    full1, s1 = oracle.render(cfg, scene, threads=1)
    full8, s8 = oracle.render(cfg, scene, threads=8)
    assert np.array_equal(full1.view(np.uint32), full8.view(np.uint32)) and s1 == s8
    sub, _ = oracle.render(cfg, scene, rows=range(3, 24, 5))
    for y in range(24):
        if y >= 3 and (y - 3) % 5 == 0:
            assert np.array_equal(sub[y].view(np.uint32), full1[y].view(np.uint32))
        else:
            assert not sub[y].any()


def test_oracle_rejects_bad_config(oracle):
    with pytest.raises(ValueError):
        oracle.render(oracle.config(8, 8, 0, 1), oracle.scene("red"))


def test_chunked_order_is_close_to_sequential(oracle):
    cfg_seq = oracle.config(32, 18, 64, 10)
    cfg_chk = oracle.config(32, 18, 64, 10, chunk=16)
    a, sa = oracle.render(cfg_seq, oracle.scene("final"))
    b, sb = oracle.render(cfg_chk, oracle.scene("final"))
    assert sa == sb  # same paths, only the summation order differs
    rms = np.sqrt(((a.astype(np.float64) - b) ** 2).mean(axis=(0, 1)))
    assert np.all(rms < 1e-6), rms
    # chunk >= spp is exactly the sequential order
    c, _ = oracle.render(oracle.config(32, 18, 64, 10, chunk=64), oracle.scene("final"))
    assert np.array_equal(a.view(np.uint32), c.view(np.uint32))


def _chunked_pixel(oracle, cfg, scene, x, y, k):
    """DESIGN.md 3 / vcrt_math.h "Accumulation" restated in numpy from per-sample radiance:
    fp32 chunk sums in sample order, each quantized to RN_even(S * 2^32), summed as integers,
    one double division, rounded to fp32."""
    cam = oracle.camera(cfg)
    p00, du, dv, center = cam[0:3], cam[3:6], cam[6:9], cam[9:12]
    f = np.float32
    pc = (p00 + f(x) * du) + f(y) * dv
    total = [0, 0, 0]
    for c0 in range(0, cfg.spp, k):
        part = np.zeros(3, dtype=np.float32)
        for i in range(c0, min(c0 + k, cfg.spp)):
            jx = f(-0.5) + f(oracle.rand(float(i), float(i)))
            jy = f(-0.5) + f(oracle.rand(float(i + 1), float(i + 1)))
            ps = pc + (jx * du + jy * dv)
            c, _ = oracle.ray_color(scene, center, ps - center, cfg.max_depth)
            part = part + c
        assert np.abs(part).max() < 4096
        for ch in range(3):
            total[ch] += int(np.rint(part[ch] * f(2.0 ** 32)))
    return np.array([(t * 2.0 ** -32) / cfg.spp for t in total], dtype=np.float64).astype(
        np.float32)


def test_chunk_combination_definition(oracle):
    """The oracle's chunked accumulation equals its definition, recomputed from per-sample
    radiance with integer arithmetic."""
    scene = oracle.scene("final")
    cfg = oracle.config(20, 12, 24, 10, chunk=5)
    img, _ = oracle.render(cfg, scene)
    for x, y in [(0, 0), (7, 5), (19, 11), (13, 8), (3, 10)]:
        want = _chunked_pixel(oracle, cfg, scene, x, y, 5)
        assert np.array_equal(img[y, x, :3].view(np.uint32), want.view(np.uint32)), (x, y)
        assert img[y, x, 3] == 1.0


def test_render_pixels_equals_rows(oracle):
    scene = oracle.scene("three")
    for chunk in (0, 4):
        cfg = oracle.config(40, 24, 6, 8, chunk=chunk)
        full, segs = oracle.render(cfg, scene)
        xy = [(x, y) for y in range(24) for x in range(40)]
        px, psegs = oracle.render_pixels(cfg, scene, xy)
        assert psegs == segs
        assert np.array_equal(px.view(np.uint32), full.reshape(-1, 4).view(np.uint32))
        sub = [(39, 23), (0, 0), (17, 9)]
        px2, _ = oracle.render_pixels(cfg, scene, sub)
        for k, (x, y) in enumerate(sub):
            assert np.array_equal(px2[k].view(np.uint32), full[y, x].view(np.uint32))
    with pytest.raises(ValueError):
        oracle.render_pixels(cfg, scene, [(40, 0)])


def _srgb_reference(c):
    c = np.nan_to_num(np.asarray(c, dtype=np.float64), nan=0.0)
    c = np.clip(c, 0.0, 1.0)
    s = np.where(c <= 0.0031308, 12.92 * c, 1.055 * np.power(c, 1 / 2.4) - 0.055)
    return np.floor(s * 255.0 + 0.5).astype(np.uint8)


def test_srgb8_encode_matches_formula(oracle):
    rng = np.random.default_rng(5)
    vals = np.concatenate([rng.uniform(-0.1, 1.1, 200000), np.linspace(0, 1, 70001),
                           [0.0, -0.0, 1.0, 2.0, np.inf, -np.inf, np.nan, 0.0031308, 1e-30]])
    vals = vals.astype(np.float32)
    rgba = np.stack([vals, vals[::-1], vals, np.ones_like(vals)], axis=1)
    got = oracle.encode_srgb8(rgba)
    want = _srgb_reference(rgba[:, :3].astype(np.float64))
    assert np.array_equal(got[:, :3], want)
    assert np.all(got[:, 3] == 255)


def test_progressive_frame_blocks(oracle):
    scene = oracle.scene("three")
    # frame blocks of 4 with chunk 4 are the same chunks as a plain chunk-4 render
    a, sa = oracle.render(oracle.config(24, 16, 8, 6, chunk=4, frame_spp=4), scene)
    b, sb = oracle.render(oracle.config(24, 16, 8, 6, chunk=4), scene)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and sa == sb
    # frame blocks restart chunks: (3,1),(3,1) differs from (3,3,2) only in the chunk sums
    c, _ = oracle.render(oracle.config(24, 16, 8, 6, chunk=3, frame_spp=4), scene)
    d, _ = oracle.render(oracle.config(24, 16, 8, 6, chunk=3), scene)
    assert np.abs(c.astype(np.float64) - d).max() < 1e-6


def _full_frame_fixture():
    with open(os.path.join(GOLDEN, "full_frame_digests.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name,rows", [("c3", [0, 540, 1079]), ("c4", [700])])
def test_full_frame_digest_fixture(oracle, name, rows):
    """tests/golden/full_frame_digests.json (the oracle over the whole C3 / C4 frames and eight
    full C5 rows, made by make_full_frame_digests.py) is reproduced by the oracle on sample rows:
    the fixture's row digests are the oracle's own, at the renderer's default quantum. The GPU
    tests (test_gpu_configs.py) assert every row of the GPU frames against the same digests."""
    fx = _full_frame_fixture()
    if name not in fx:
        pytest.skip(f"{name} digests not generated yet")
    fx = fx[name]
    n = fx["height"] if fx["rows"] is None else len(fx["rows"])
    assert len(fx["row_sha256_16"]) == n and fx["finite"]
    assert max(fx["rms_vs_sequential"]) <= 1e-4  # north_star's per-channel bar, whole frame
    cfg = oracle.config(fx["width"], fx["height"], fx["spp"], fx["max_depth"],
                        quantum=fx["quantum"])
    sc = oracle.scene(fx["scene"])
    for i in rows:
        y = fx["rows"][i] if fx["rows"] else i
        img, _ = oracle.render(cfg, sc, rows=range(y, y + 1))
        d = hashlib.sha256(np.ascontiguousarray(img[y], dtype="<f4").tobytes()).hexdigest()[:16]
        assert d == fx["row_sha256_16"][i], (name, y)


@pytest.mark.parametrize("name", ["c3", "c4", "c5rows"])
def test_full_frame_digest_fixture_pixels(oracle, name):
    """The fixture's eight sample pixels (float bits) re-rendered by the oracle: cheap enough for
    C5's 4100-sphere, 4096-spp, depth-50 rows, whose full rows take minutes on the CPU."""
    fx = _full_frame_fixture()
    if name not in fx:
        pytest.skip(f"{name} digests not generated yet")
    fx = fx[name]
    cfg = oracle.config(fx["width"], fx["height"], fx["spp"], fx["max_depth"],
                        quantum=fx["quantum"])
    px = fx["sample_pixels"]
    got, _ = oracle.render_pixels(cfg, oracle.scene(fx["scene"]), [(p[0], p[1]) for p in px])
    assert got.view(np.uint32).tolist() == [p[2:] for p in px]
