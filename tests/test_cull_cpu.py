"""CPU checks of the CULL variant's grouped tables (vcrt_cull_tables, csrc/cluster.cpp).

The culled scan is exact only if (1) every sphere sits in exactly one group with the linear
table's values, and (2) a group whose box test rules it out for a ray holds no sphere whose
fp32 discriminant (hit_sphere, functions.glsl:14-22, as tracer.hip's pair_disc evaluates it) is
>= 0. (2) is checked here by emulating both fp32 evaluations in numpy on random rays (near and
far origins), on rays built to graze member spheres within 1e-7..1e-4 of their radius, and on
rays grazing a member where it touches its box. The kernels also rule out a box whose stretch of
the ray's line lies behind -tau (tracer.hip fact (4)): there the property is that a ruled-out box
holds no member the exact test may accept (disc >= 0 and hb or cc negative), checked on rays
leaving member spheres' surfaces and on rays just past a member, pointing away from it.
"""
import numpy as np
import pytest

from vulkancomputeraytracing_amd import _native as N
from vulkancomputeraytracing_amd import scene as S

f32 = np.float32


def fma(x, y, z):
    # fp32 fma through float64: the product is exact, the sum rounds twice (harmless here)
    return (x.astype(np.float64) * y.astype(np.float64) + z.astype(np.float64)).astype(f32)


def rn(x):
    return np.asarray(x, np.float64).astype(f32)


def ulp_noise(x, rng, ulps=1):
    """x perturbed by up to `ulps` ulp (v_rcp_f32 / v_sqrt_f32 are 1 ulp accurate)."""
    if rng is None:
        return x
    k = rng.integers(-ulps, ulps + 1, x.shape)
    out = x.copy()
    for step in range(1, ulps + 1):
        out = np.where(k >= step, np.nextafter(out, f32(np.inf)), out)
        out = np.where(k <= -step, np.nextafter(out, f32(-np.inf)), out)
    return out.astype(f32)


CLIP = True  # tracer.hip VCRT_BOX_CLIP: fact (4), the near end clamped at -tau


def box_ray(t, o, d, rng=None, tau_scale=1.0):
    """tracer.hip box_ray in fp32: per axis inv = v_rcp(d'), c = fma(-o, inv, tau) with
    tau = sqrt(3.2e-7 Q / a) (fact (4); tau_scale scales it for the checker's own test); c1, c2."""
    cmax, rmax2, lam = (f32(v) for v in t["margin"][:3])
    dd = np.where(np.abs(d) < f32(2.0 ** -40), np.copysign(f32(2.0 ** -40), d), d).astype(f32)
    inv = ulp_noise(rn(1.0 / dd.astype(np.float64)), rng)
    dot = rn(rn(rn(o[:, 0] * o[:, 0]) + rn(o[:, 1] * o[:, 1])) + rn(o[:, 2] * o[:, 2]))
    on = rn(ulp_noise(rn(np.sqrt(dot.astype(np.float64))), rng) + cmax)
    Q = rn(rn(on * on) + rmax2)
    tau = np.zeros(len(o), f32)
    if CLIP:
        a = rn(rn(rn(d[:, 0] * d[:, 0]) + rn(d[:, 1] * d[:, 1])) + rn(d[:, 2] * d[:, 2]))
        with np.errstate(divide="ignore", over="ignore"):
            ya = ulp_noise(rn(1.0 / a.astype(np.float64)), rng)
            arg = rn(rn(f32(3.2e-7) * Q) * ya)
        tau = ulp_noise(rn(np.sqrt(arg.astype(np.float64))), rng)
        tau = rn(tau.astype(np.float64) * tau_scale)
    c = fma(-o, inv, np.broadcast_to(tau[:, None], inv.shape))
    J = rn(f32(2.002) * np.abs(inv).max(1))
    oinf = np.abs(o).max(1)
    c1 = rn(J * rn(f32(3.04e-7) * rn(lam + oinf)))
    c2 = rn(J * Q)
    return inv, c, c1, c2


def group_culled(t, o, d, key="bound", rng=None, tau_scale=1.0):
    """[rays, boxes] bool: the kernel's box test (tracer.hip box_gap, facts (3) and (4)) on the
    group boxes (key "bound"), the node boxes ("node") or the chunk boxes ("top"), in fp32 with
    v_rcp_f32 / v_sqrt_f32's 1-ulp errors emulated by random perturbations (rng)."""
    b = t[key]
    G = 2 * b.shape[0]
    cols = lambda k: np.stack([b[:, k], b[:, k + 1]], 1).reshape(G)  # noqa: E731
    lo = [cols(0), cols(2), cols(4)]
    hi = [cols(6), cols(8), cols(10)]
    K = cols(12)
    inv, c, c1, c2 = box_ray(t, o, d, rng, tau_scale)
    tn = tf = None
    for k in range(3):
        tl = fma(lo[k][None, :], inv[:, k, None], c[:, k, None])
        th = fma(hi[k][None, :], inv[:, k, None], c[:, k, None])
        near, far = np.minimum(tl, th), np.maximum(tl, th)
        tn = near if tn is None else np.maximum(tn, near)
        tf = far if tf is None else np.minimum(tf, far)
    if CLIP:
        tn = np.maximum(tn, f32(0))
    with np.errstate(over="ignore", invalid="ignore"):
        gap = fma(np.broadcast_to(K[None, :], tn.shape), np.broadcast_to(c2[:, None], tn.shape),
                  rn(rn(tf - tn) + c1[:, None]))
    return gap < 0


def group_gap(t, o, d, key="bound", near_far=False):
    """[rays, boxes] fp32 box gaps: box_gap's per-axis min / max (near_far False) or the
    flat kernel's planes chosen by the sign of 1/d' (push_bound_pair_nf, near_far True)."""
    b = t[key]
    G = 2 * b.shape[0]
    cols = lambda k: np.stack([b[:, k], b[:, k + 1]], 1).reshape(G)  # noqa: E731
    lo = [cols(0), cols(2), cols(4)]
    hi = [cols(6), cols(8), cols(10)]
    K = cols(12)
    inv, c, c1, c2 = box_ray(t, o, d)
    tn = tf = None
    for k in range(3):
        tl = fma(lo[k][None, :], inv[:, k, None], c[:, k, None])
        th = fma(hi[k][None, :], inv[:, k, None], c[:, k, None])
        if near_far:
            neg = np.signbit(inv[:, k, None])
            near, far = np.where(neg, th, tl), np.where(neg, tl, th)
        else:
            near, far = np.minimum(tl, th), np.maximum(tl, th)
        tn = near if tn is None else np.maximum(tn, near)
        tf = far if tf is None else np.minimum(tf, far)
    if CLIP:
        tn = np.maximum(tn, f32(0))
    with np.errstate(over="ignore", invalid="ignore"):
        return fma(np.broadcast_to(K[None, :], tn.shape), np.broadcast_to(c2[:, None], tn.shape),
                   rn(rn(tf - tn) + c1[:, None]))


@pytest.mark.parametrize("name", ["final", "stress4096"])
def test_near_far_planes_equal_min_max(name):
    """The flat kernel's node passes read each axis' near and far plane by the sign of 1/d'
    (cbound_nf layout) instead of taking min / max: the gaps, sign bits included, are equal."""
    rng = np.random.default_rng(11)
    t = S.cull_tables(S.builtin_scene(name))
    o, d = random_rays(3000, rng, -20.0, 20.0)
    d[:100, 0] = 0.0   # zero and negative-zero directions: d' = +-2^-40
    d[100:200, 1] = -0.0
    o[200:300] = 0.0
    a = group_gap(t, o, d, near_far=False)
    b = group_gap(t, o, d, near_far=True)
    assert np.array_equal(np.signbit(a), np.signbit(b))
    assert np.array_equal(a, b)


def member_disc(t, o, d):
    """[rays, hierarchy groups, 4] fp32 discriminants exactly as pair_disc computes them."""
    g = t["geom"][t["nbig"]:]
    cx = np.stack([g[:, 0], g[:, 1], g[:, 8], g[:, 9]], 1)
    cy = np.stack([g[:, 2], g[:, 3], g[:, 10], g[:, 11]], 1)
    cz = np.stack([g[:, 4], g[:, 5], g[:, 12], g[:, 13]], 1)
    r2 = np.stack([g[:, 6], g[:, 7], g[:, 14], g[:, 15]], 1)
    a = ((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2])[:, None, None]
    ox, oy, oz = (o[:, k, None, None] for k in range(3))
    dx, dy, dz = (d[:, k, None, None] for k in range(3))
    ocx, ocy, ocz = ox - cx[None], oy - cy[None], oz - cz[None]
    hb = (ocx * dx + ocy * dy) + ocz * dz
    cc = ((ocx * ocx + ocy * ocy) + ocz * ocz) - r2[None]
    with np.errstate(over="ignore", invalid="ignore"):  # padding members: r^2 = -3e38
        return hb * hb - a * cc


def grazing_rays(spheres, n, rng):
    idx = rng.integers(0, len(spheres), n)
    c = spheres["center"][idx].astype(np.float64)
    r = np.abs(spheres["radius"][idx].astype(np.float64))
    dh = rng.normal(size=(n, 3))
    dh /= np.linalg.norm(dh, axis=1, keepdims=True)
    p = rng.normal(size=(n, 3))
    p -= (p * dh).sum(1, keepdims=True) * dh
    p /= np.linalg.norm(p, axis=1, keepdims=True)
    delta = rng.choice([-1e-6, 0.0, 1e-7, 3e-7, 1e-6, 1e-5, 1e-4], n)
    q = c + p * (r * (1 + delta))[:, None]
    s = rng.uniform(0.5, 40.0, n)[:, None]
    o = (q - s * dh).astype(f32)
    d = (dh * rng.choice([0.01, 0.3, 1.0, 7.0, 100.0], n)[:, None]).astype(f32)
    return o, d


def tangent_rays(spheres, t, n, rng):
    """Rays that graze a group's extreme member where it touches a face of the group's box
    (the tightest case for the box test): touching point c +- r e_a, direction in the face."""
    G = t["geom"].shape[0] - t["nbig"]
    os_, ds_ = [], []
    for gi in rng.integers(0, G, n):
        idx = t["index"][t["nbig"] + gi]
        m = idx[idx >= 0]
        if len(m) == 0:
            continue
        c = spheres["center"][m].astype(np.float64)
        r = np.abs(spheres["radius"][m].astype(np.float64))
        a, sgn = rng.integers(0, 3), rng.choice([-1.0, 1.0])
        i = np.argmax(sgn * c[:, a] + r)
        e = np.zeros(3)
        e[a] = sgn
        q = c[i] + e * r[i] * (1 + rng.choice([-1e-6, 0.0, 1e-7, 3e-7, 1e-6, 1e-5]))
        p = rng.normal(size=3)
        p -= (p @ e) * e
        p /= np.linalg.norm(p)
        os_.append(q - rng.uniform(0.5, 40.0) * p)
        ds_.append(p * rng.choice([0.01, 1.0, 100.0]))
    return np.array(os_, f32), np.array(ds_, f32)


def surface_rays(spheres, n, rng):
    """Secondary rays: origins on member spheres' surfaces (rounded to fp32, so just inside or
    outside), directions normal + a random unit vector (scattered) or random (refracted), and
    rays just past a member (0..1e-3 of its radius beyond the surface) pointing away from it."""
    idx = rng.integers(0, len(spheres), n)
    c = spheres["center"][idx].astype(np.float64)
    r = np.abs(spheres["radius"][idx].astype(np.float64))
    nrm = rng.normal(size=(n, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    gap = rng.choice([0.0, 0.0, 1e-7, 1e-5, 1e-3], n)[:, None]
    o = c + nrm * (r[:, None] * (1 + gap))
    kind = rng.integers(0, 3, n)[:, None]
    d = np.where(kind == 0, nrm + u, np.where(kind == 1, u, nrm + 0.05 * u))
    d *= rng.choice([0.05, 1.0, 3.0], n)[:, None]
    return o.astype(f32), d.astype(f32)


def random_rays(n, rng, lo, hi):
    o = rng.uniform(lo, hi, size=(n, 3)).astype(f32)
    d = (rng.normal(size=(n, 3)) * rng.choice([0.05, 1.0, 20.0], n)[:, None]).astype(f32)
    return o, d


@pytest.mark.parametrize("name", ["final", "stress4096"])
def test_groups_partition_the_scene(name):
    sp = S.builtin_scene(name)
    t = S.cull_tables(sp)
    assert t is not None
    nb = t["nbig"]
    G = t["geom"].shape[0] - nb
    assert G % 16 == 0 and t["node"].shape[0] == G // 16 and t["bound"].shape[0] == G // 2
    idx = t["index"].reshape(-1)
    members = np.sort(idx[idx >= 0])
    assert np.array_equal(members, np.arange(len(sp)))
    # the big-sphere list holds exactly the spheres above 8x the median radius and 5% of the
    # extent of the centres (at most 64)
    r = np.abs(sp["radius"]).astype(np.float64)
    c = sp["center"].astype(np.float64)
    extent = np.linalg.norm(c.max(0) - c.min(0))
    huge = max(8 * np.partition(r, len(r) // 2)[len(r) // 2], 0.05 * extent)
    big = set(np.nonzero(r > huge)[0].tolist())
    # ... plus the largest of the rest (ties by index) in the big list's free slots: the big
    # three join the ground in both scenes
    free = (4 - len(big) % 4) % 4
    if big and free:
        others = [i for i in np.argsort(-r, kind="stable").tolist() if i not in big]
        big |= set(others[:free])
    if name == "stress4096":
        assert big == {4096, 4097, 4098, 4099} and G == 1024
    else:
        assert big == {481, 482, 483, 484}
    bi = t["index"][:nb].reshape(-1)
    assert set(bi[bi >= 0].tolist()) == big
    g = t["geom"]
    for gi in range(nb + G):
        for k in range(4):
            j = t["index"][gi, k]
            if j < 0:
                continue
            base = 8 * (k // 2) + (k % 2)
            assert g[gi, base] == sp["center"][j, 0]
            assert g[gi, base + 2] == sp["center"][j, 1]
            assert g[gi, base + 4] == sp["center"][j, 2]
            assert g[gi, base + 6] == f32(sp["radius"][j]) * f32(sp["radius"][j])
            if gi < nb:
                continue
            h = gi - nb
            # the group's box holds the member (float64 geometry), and so do the node's and
            # the chunk's; their K covers its radius
            c = sp["center"][j].astype(np.float64)
            r = abs(float(sp["radius"][j]))
            for tab, i in (("bound", h), ("node", h // 8), ("top", h // 64)):
                e, b = i % 2, t[tab][i // 2].astype(np.float64)
                lo, hi = b[[0 + e, 2 + e, 4 + e]], b[[6 + e, 8 + e, 10 + e]]
                assert (lo <= c - r).all() and (hi >= c + r).all(), (tab, i)
                assert b[12 + e] >= 8.1 * 2.0 ** -24 / r, (tab, i)


def test_small_or_unbounded_scenes_do_not_cull():
    assert S.cull_tables(S.builtin_scene("three")) is None
    sp = S.builtin_scene("final").copy()
    sp["center"][7, 0] = 3e9
    assert S.cull_tables(sp) is None


@pytest.mark.parametrize("name", ["final", "stress4096"])
def test_bound_test_is_conservative(name):
    rng = np.random.default_rng(7)
    sp = S.builtin_scene(name)
    t = S.cull_tables(sp)
    valid = t["index"][t["nbig"]:] >= 0
    total_culled = 0
    total = 0
    chunks = [grazing_rays(sp, 1500, rng) for _ in range(3)]
    chunks += [tangent_rays(sp, t, 1500, rng) for _ in range(2)]
    chunks += [random_rays(1500, rng, -20.0, 20.0), random_rays(500, rng, -2.0, 2.0)]
    chunks += [random_rays(500, rng, -3000.0, 3000.0)]  # far origins: large margins
    chunks += [surface_rays(sp, 1500, rng) for _ in range(2)]
    for o, d in chunks:
        culled = group_culled(t, o, d, rng=rng)
        hb, cc, disc = member_hb_cc_disc(t, o, d)
        # members the exact test may accept (may_hit / hit_sign: -0 counts as negative)
        hit = (~(disc < 0)) & (np.signbit(hb) | np.signbit(cc)) & valid[None]
        bad = culled[:, :, None] & hit
        assert not bad.any(), f"{int(bad.sum())} culled group members that may be accepted"
        # a culled node (8 consecutive groups) holds no such member either
        node_culled = np.repeat(group_culled(t, o, d, "node", rng=rng), 8, axis=1)
        bad = node_culled[:, :, None] & hit
        assert not bad.any(), f"{int(bad.sum())} culled node members that may be accepted"
        G = hit.shape[1]
        top_culled = np.repeat(group_culled(t, o, d, "top", rng=rng), 64, axis=1)[:, :G]
        bad = top_culled[:, :, None] & hit
        assert not bad.any(), f"{int(bad.sum())} culled top-level members that may be accepted"
        total_culled += int(culled.sum())
        total += culled.size
    # and the test does cull (most groups are far from most rays)
    assert total_culled > 0.7 * total


def test_checker_detects_a_too_small_box():
    """The emulated check above has teeth: boxes shrunk by 1e-4 of their size with no margin
    are caught by the grazing rays."""
    rng = np.random.default_rng(11)
    sp = S.builtin_scene("final")
    t = S.cull_tables(sp)
    bad_t = {k: (v.copy() if hasattr(v, "copy") else v) for k, v in t.items()}
    b = bad_t["bound"]
    for k in range(3):
        lo, hi = b[:, 2 * k:2 * k + 2], b[:, 6 + 2 * k:8 + 2 * k]
        shrink = (hi - lo) * f32(1e-4)
        b[:, 2 * k:2 * k + 2], b[:, 6 + 2 * k:8 + 2 * k] = lo + shrink, hi - shrink
    b[:, 12:14] = 0                          # no per-box margin
    bad_t["margin"] = t["margin"].copy()
    bad_t["margin"][2] = 0                   # no rounding slack
    o, d = tangent_rays(sp, t, 1500, rng)
    culled = group_culled(bad_t, o, d)
    hit = ~(member_disc(t, o, d) < 0) & (t["index"][t["nbig"]:] >= 0)[None]
    assert (culled[:, :, None] & hit).any()


@pytest.mark.parametrize("name", ["final", "stress4096"])
def test_clip_behind_origin_culls_and_has_teeth(name):
    """Fact (4) rules out boxes the line test keeps (secondary rays leave a sphere: about half
    the boxes their line crosses lie behind the origin), and the check above would catch a clip
    that reached past -tau: planes shifted by -50 tau (the clamp then cuts the line ahead of the
    origin) cull members the exact test may accept."""
    global CLIP
    rng = np.random.default_rng(5)
    sp = S.builtin_scene(name)
    t = S.cull_tables(sp)
    valid = t["index"][t["nbig"]:] >= 0
    o, d = surface_rays(sp, 1500, rng)
    clipped = group_culled(t, o, d).sum()
    try:
        CLIP = False
        line = group_culled(t, o, d).sum()
    finally:
        CLIP = True
    assert clipped > line + 0.01 * (~group_culled(t, o, d)).sum()
    hb, cc, disc = member_hb_cc_disc(t, o, d)
    hit = (~(disc < 0)) & (np.signbit(hb) | np.signbit(cc)) & valid[None]
    assert (group_culled(t, o, d, tau_scale=-50.0)[:, :, None] & hit).any()


def test_margin_constants():
    """The host constants of the box test (cluster.cpp, tracer.hip (3)): per box K >= 8.1u /
    r_min (1 + 1e-5) of its members; margin = (>= max |centre|, >= r_max^2, >= max |box
    coordinate|) over the hierarchy."""
    sp = S.builtin_scene("final")
    t = S.cull_tables(sp)
    u = 2.0 ** -24
    nb = t["nbig"]
    hier = t["index"][nb:]
    m_all = hier[hier >= 0]
    c = sp["center"][m_all].astype(np.float64)
    r = np.abs(sp["radius"][m_all].astype(np.float64))
    cmax, rmax2, lam = (float(v) for v in t["margin"][:3])
    assert cmax >= np.linalg.norm(c, axis=1).max()
    assert rmax2 >= (r ** 2).max()
    assert lam >= (np.abs(c) + r[:, None]).max()
    for gi in range(hier.shape[0]):
        m = hier[gi][hier[gi] >= 0]
        if len(m) == 0:
            continue
        e, bb = gi % 2, t["bound"][gi // 2]
        rm = np.abs(sp["radius"][m].astype(np.float64)).min()
        assert float(bb[12 + e]) >= 8.1 * u / rm * (1 + 1e-5)


def test_hierarchy_is_aligned():
    """Nodes (8 groups) and chunks (64 groups) are whole k-d subtrees: a node's box is not much
    larger than its groups' (sanity: median node diagonal <= 4x the median group diagonal on
    the grid scenes)."""
    for name in ("final", "stress4096"):
        t = S.cull_tables(S.builtin_scene(name))

        def diag(tab):
            b = tab.astype(np.float64)
            out = []
            for e in (0, 1):
                lo, hi = b[:, [0 + e, 2 + e, 4 + e]], b[:, [6 + e, 8 + e, 10 + e]]
                out.append(np.linalg.norm(hi - lo, axis=1))
            dd = np.concatenate(out)
            return dd[dd > 0]
        assert np.median(diag(t["node"])) <= 4 * np.median(diag(t["bound"]))


def member_hb_cc_disc(t, o, d):
    """member_disc's fp32 hb, cc and disc (tracer.hip pair_disc_cc)."""
    g = t["geom"][t["nbig"]:]
    cx = np.stack([g[:, 0], g[:, 1], g[:, 8], g[:, 9]], 1)
    cy = np.stack([g[:, 2], g[:, 3], g[:, 10], g[:, 11]], 1)
    cz = np.stack([g[:, 4], g[:, 5], g[:, 12], g[:, 13]], 1)
    r2 = np.stack([g[:, 6], g[:, 7], g[:, 14], g[:, 15]], 1)
    a = ((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2])[:, None, None]
    ox, oy, oz = (o[:, k, None, None] for k in range(3))
    dx, dy, dz = (d[:, k, None, None] for k in range(3))
    ocx, ocy, ocz = ox - cx[None], oy - cy[None], oz - cz[None]
    hb = (ocx * dx + ocy * dy) + ocz * dz
    cc = ((ocx * ocx + ocy * ocy) + ocz * ocz) - r2[None]
    with np.errstate(over="ignore", invalid="ignore"):
        return hb, cc, hb * hb - a * cc


def camera_rays_f32(cam, px, py, jx, jy):
    """Camera rays exactly as tracer.hip trace_impl builds them in fp32 (shader.comp:43-52):
    pc = (p00 + px du) + py dv; ps = pc + (jx du + jy dv); d = ps - centre."""
    p00, du, dv, ctr = (cam[3 * k:3 * k + 3].astype(f32) for k in range(4))
    px, py = px.astype(f32)[:, None], py.astype(f32)[:, None]
    jx, jy = jx.astype(f32)[:, None], jy.astype(f32)[:, None]
    pc = (p00[None] + px * du[None]) + py * dv[None]
    ps = pc + (jx * du[None] + jy * dv[None])
    d = (ps - ctr[None]).astype(f32)
    o = np.broadcast_to(ctr, d.shape).astype(f32)
    return o, d


INSIDE = dict(lookfrom=(2, 0.3, 1.5), lookat=(-6, 0.2, -2), vfov=60)
DOWN = dict(lookfrom=(0.5, 30, 0.5), lookat=(0, 0, 0), vfov=30)


@pytest.mark.parametrize("name,w,h,world,rank,cam", [("final", 1920, 1080, 1, 0, {}),
                                                     ("final", 800, 450, 8, 3, {}),
                                                     ("final", 160, 90, 1, 0, {}),
                                                     ("final", 640, 360, 1, 0, INSIDE),
                                                     ("final", 640, 360, 1, 0, DOWN),
                                                     ("stress4096", 3840, 2160, 1, 0, {})])
def test_primary_lists_hold_every_camera_ray_candidate(name, w, h, world, rank, cam):
    """The flat scan's camera rays start from the group list of their 4x4-pixel quarter of a
    tile (csrc/primary.cpp) and skip the hierarchy, so a list must hold every group with a
    member that may be accepted (disc >= 0 and (hb < 0 or cc < 0), tracer.hip may_hit) for any
    camera ray of the quarter: checked on fp32 emulations of the kernel's rays for every pixel
    of sampled quarters, at the jitter table's extreme and random samples."""
    from tests import oracle_py
    from vulkancomputeraytracing_amd.renderer import RenderDesc, tiles_for_rank
    o = oracle_py.load()
    sp = S.builtin_scene(name)
    t = S.cull_tables(sp)
    desc = RenderDesc(width=w, height=h, world_size=world, rank=rank, **cam)
    pl = S.primary_lists(sp, desc)
    cam = o.camera(o.config(w, h, 1, 10, **cam))
    tiles = tiles_for_rank(w, h, world, rank)
    info = pl["info"]
    assert len(info) == 4 * len(tiles)
    cnt = info & 15
    listed = np.nonzero(cnt != 15)[0]
    assert len(listed) > 0.3 * len(info)  # most quarters get a list
    assert (cnt[listed] <= 8).all()
    # jitter of the first 1024 samples: -0.5 + rand(i, i), the extremes and a few others
    lib = N.lib()
    jit = np.array([[f32(-0.5) + f32(lib.vcrt_canonical_rand(float(i), float(i))),
                     f32(-0.5) + f32(lib.vcrt_canonical_rand(float(i + 1), float(i + 1)))]
                    for i in range(1024)], f32)
    rng = np.random.default_rng(11)
    pick = [int(np.argmin(jit[:, 0])), int(np.argmax(jit[:, 0])), int(np.argmin(jit[:, 1])),
            int(np.argmax(jit[:, 1]))] + list(rng.integers(0, 1024, 2))
    valid = t["index"][t["nbig"]:] >= 0
    tx_n = (w + 7) // 8
    sample = rng.choice(listed, size=min(160, len(listed)), replace=False)
    sample = np.concatenate([sample, listed[:4], listed[-4:]])
    total_may = control_hits = 0
    for e in sample:
        ty, tx = divmod(tiles[e >> 2], tx_n)
        qx, qy = e & 1, (e >> 1) & 1
        ids = pl["ids"][(info[e] >> 4):(info[e] >> 4) + cnt[e]]
        inlist = np.zeros(valid.shape[0], bool)
        inlist[ids] = True
        px = np.repeat(8 * tx + 4 * qx + np.arange(16) % 4, len(pick))
        py = np.repeat(8 * ty + 4 * qy + np.arange(16) // 4, len(pick))
        jj = np.tile(np.array(pick), 16)
        og, dg = camera_rays_f32(cam, px, py, jit[jj, 0], jit[jj, 1])
        hb, cc, disc = member_hb_cc_disc(t, og, dg)
        may = (~(disc < 0)) & ((hb < 0) | (cc < 0)) & valid[None]
        missing = may & ~inlist[None, :, None]
        assert not missing.any(), f"entry {e}: {int(missing.sum())} candidates not listed"
        total_may += int(may.sum())
        needed = [g for g in ids if may[:, g].any()]
        if needed:  # control: without a listed group that holds candidates, the check fails
            inlist[needed[-1]] = False
            control_hits += bool((may & ~inlist[None, :, None]).any())
    assert total_may > 0 and control_hits > 0


@pytest.mark.parametrize("name,w,h,world,rank,cam", [("final", 1920, 1080, 1, 0, {}),
                                                     ("final", 800, 450, 8, 3, {}),
                                                     ("final", 640, 360, 1, 0, INSIDE),
                                                     ("final", 640, 360, 1, 0, DOWN),
                                                     ("stress4096", 3840, 2160, 1, 0, {})])
def test_primary_sphere_lists_hold_every_camera_ray_candidate(name, w, h, world, rank, cam):
    """The camera fast trace tests a camera ray against its quarter's per-sphere list only
    (csrc/primary.cpp build_primary_sphere_lists; besides the big list), so the list must hold
    every hierarchy sphere that may be accepted (disc >= 0 and (hb < 0 or cc < 0)) for any camera
    ray of the quarter, and its records must be the fp32 oc / cc the exact test computes: checked
    on fp32 emulations of the kernel's rays for every pixel of sampled quarters at the jitter
    table's extreme and random samples. The lists are much shorter than the group lists."""
    from tests import oracle_py
    from vulkancomputeraytracing_amd.renderer import RenderDesc, tiles_for_rank
    o = oracle_py.load()
    sp = S.builtin_scene(name)
    t = S.cull_tables(sp)
    desc = RenderDesc(width=w, height=h, world_size=world, rank=rank, **cam)
    sl = S.primary_sphere_lists(sp, desc)
    pl = S.primary_lists(sp, desc)
    cam = o.camera(o.config(w, h, 1, 10, **cam))
    tiles = tiles_for_rank(w, h, world, rank)
    info, rec = sl["info"], sl["rec"]
    assert len(info) == 4 * len(tiles)
    cnt = info & 15
    listed = np.nonzero(cnt != 15)[0]
    assert len(listed) > 0.3 * len(info) and (cnt[listed] <= 14).all()
    # far fewer spheres than the group lists' members
    gl = pl["info"] & 15
    both = (gl != 15) & (cnt != 15)
    assert cnt[both].mean() < 0.5 * 4 * gl[both].mean()
    # records: oc = centre of projection - centre, cc = ((ocx^2 + ocy^2) + ocz^2) - r^2, fp32
    idx = rec[:, 8:10].view(np.int32)
    ctr = cam[9:12].astype(f32)
    for s_ in range(2):
        real = idx[:, s_] >= 0
        c = sp["center"][idx[real, s_]].astype(f32)
        oc = (ctr[None] - c).astype(f32)
        r2 = (sp["radius"][idx[real, s_]].astype(f32) ** 2).astype(f32)
        cc = (((oc[:, 0] * oc[:, 0] + oc[:, 1] * oc[:, 1]) + oc[:, 2] * oc[:, 2]) - r2).astype(f32)
        assert np.array_equal(rec[real, 0 + s_].view(np.uint32), oc[:, 0].view(np.uint32))
        assert np.array_equal(rec[real, 2 + s_].view(np.uint32), oc[:, 1].view(np.uint32))
        assert np.array_equal(rec[real, 4 + s_].view(np.uint32), oc[:, 2].view(np.uint32))
        assert np.array_equal(rec[real, 6 + s_].view(np.uint32), cc.view(np.uint32))
        assert (rec[~real, 6 + s_] == f32(3e38)).all()
    lib = N.lib()
    jit = np.array([[f32(-0.5) + f32(lib.vcrt_canonical_rand(float(i), float(i))),
                     f32(-0.5) + f32(lib.vcrt_canonical_rand(float(i + 1), float(i + 1)))]
                    for i in range(1024)], f32)
    rng = np.random.default_rng(12)
    pick = [int(np.argmin(jit[:, 0])), int(np.argmax(jit[:, 0])), int(np.argmin(jit[:, 1])),
            int(np.argmax(jit[:, 1]))] + list(rng.integers(0, 1024, 2))
    members = t["index"][t["nbig"]:]
    valid = members >= 0
    tx_n = (w + 7) // 8
    sample = rng.choice(listed, size=min(160, len(listed)), replace=False)
    sample = np.concatenate([sample, listed[:4], listed[-4:]])
    total_may = control_hits = 0
    for e in sample:
        ty, tx = divmod(tiles[e >> 2], tx_n)
        qx, qy = e & 1, (e >> 1) & 1
        first, n = int(info[e] >> 4), int(cnt[e])
        ids = idx[first:first + (n + 1) // 2].reshape(-1)[:n]
        inlist = np.isin(members, ids) & valid
        px = np.repeat(8 * tx + 4 * qx + np.arange(16) % 4, len(pick))
        py = np.repeat(8 * ty + 4 * qy + np.arange(16) // 4, len(pick))
        jj = np.tile(np.array(pick), 16)
        og, dg = camera_rays_f32(cam, px, py, jit[jj, 0], jit[jj, 1])
        hb, cc, disc = member_hb_cc_disc(t, og, dg)
        may = (~(disc < 0)) & ((hb < 0) | (cc < 0)) & valid[None]
        missing = may & ~inlist[None]
        assert not missing.any(), f"entry {e}: {int(missing.sum())} candidate spheres not listed"
        total_may += int(may.sum())
        if n:  # control: without its last sphere the list would miss candidates
            drop = inlist & (members == ids[-1])
            control_hits += bool((may & drop[None]).any())
    assert total_may > 0 and control_hits > 0


@pytest.mark.parametrize("name,w,h,world,rank", [("final", 1920, 1080, 1, 0),
                                                 ("final", 800, 450, 3, 1),
                                                 ("stress4096", 1280, 720, 1, 0)])
def test_camera_lists_threads_equal_serial(monkeypatch, name, w, h, world, rank):
    """vcrt_set_scene builds the camera-ray lists on up to 16 host threads (primary.cpp
    parallel_parts); the parts are concatenated in order, so the lists equal a one-thread build
    bit for bit."""
    from vulkancomputeraytracing_amd.renderer import RenderDesc
    sp = S.builtin_scene(name)
    d = RenderDesc(width=w, height=h, world_size=world, rank=rank)
    monkeypatch.setenv("VCRT_HOST_THREADS", "7")
    a, b = S.primary_lists(sp, d), S.primary_sphere_lists(sp, d)
    monkeypatch.setenv("VCRT_HOST_THREADS", "1")
    a1, b1 = S.primary_lists(sp, d), S.primary_sphere_lists(sp, d)
    for k in a:
        assert np.array_equal(a[k], a1[k]), k
    for k in b:
        assert np.array_equal(b[k].view(np.uint32), b1[k].view(np.uint32)), k
