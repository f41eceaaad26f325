"""CPU checks of the CULL variant's grouped tables (vcrt_cull_tables, csrc/cluster.cpp).

The culled scan is exact only if (1) every sphere sits in exactly one group with the linear
table's values, and (2) a group whose bound test culls it for a ray holds no sphere whose fp32
discriminant (hit_sphere, functions.glsl:14-22, as tracer.hip's pair_disc evaluates it) is
>= 0. (2) is checked here by emulating both fp32 evaluations in numpy on random rays and on
rays built to graze member spheres within 1e-7..1e-4 of their radius.
"""
import numpy as np
import pytest

from vulkancomputeraytracing_amd import scene as S

f32 = np.float32


def fma(x, y, z):
    # fp32 fma through float64: the product is exact, the sum rounds twice (harmless here)
    return (x.astype(np.float64) * y.astype(np.float64) + z.astype(np.float64)).astype(f32)


def group_culled(t, o, d, key="bound", rng=None):
    """[rays, bounds] bool: the kernel's bound test (tracer.hip bound_pair_need) on the group
    bounds (key "bound") or the node bounds ("node"). v_rsq_f32's error (~1 ulp) is emulated
    by a random +-2 ulp perturbation of the exact reciprocal square root."""
    b = t[key]
    G = 2 * b.shape[0]
    cols = lambda k: np.stack([b[:, k], b[:, k + 1]], 1).reshape(G)  # noqa: E731
    C = [cols(0), cols(2), cols(4)]
    K, Rk = cols(6), cols(8)
    a = ((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2])
    inv = (1.0 / np.sqrt(a.astype(np.float64))).astype(f32)
    if rng is not None:
        inv = (inv * (1 + rng.uniform(-2.4e-7, 2.4e-7, inv.shape))).astype(f32)
    w = (d * inv[:, None]).astype(f32)
    oc = [(o[:, k, None] - C[k][None, :]).astype(f32) for k in range(3)]
    ww = [np.broadcast_to(w[:, k, None], oc[0].shape) for k in range(3)]
    oc2 = fma(oc[2], oc[2], fma(oc[1], oc[1], oc[0] * oc[0]))
    h = fma(oc[2], ww[2], fma(oc[1], ww[1], oc[0] * ww[0]))
    X = fma(-h, h, oc2)
    with np.errstate(invalid="ignore", over="ignore"):
        RM = fma(np.broadcast_to(K, oc2.shape), oc2, np.broadcast_to(Rk, oc2.shape))
        T = RM * RM
        return X > T


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


def bound_of(t, gi):
    e, bb = gi % 2, t["bound"][gi // 2]
    return np.array([bb[0 + e], bb[2 + e], bb[4 + e]], np.float64)


def tangent_rays(spheres, t, n, rng):
    """Rays tangent to a group's outermost member on the side facing away from the group
    centre: they graze the member where it touches the bounding sphere (the tightest case for
    the bound test)."""
    G = t["geom"].shape[0] - t["nbig"]
    os_, ds_ = [], []
    for gi in rng.integers(0, G, n):
        C = bound_of(t, gi)
        idx = t["index"][t["nbig"] + gi]
        m = idx[idx >= 0]
        if len(m) == 0:
            continue
        c = spheres["center"][m].astype(np.float64)
        r = np.abs(spheres["radius"][m].astype(np.float64))
        i = np.argmax(np.linalg.norm(c - C, axis=1) + r)
        u = c[i] - C
        u = u / np.linalg.norm(u) if np.linalg.norm(u) > 0 else np.array([0.0, 1.0, 0.0])
        q = c[i] + u * r[i] * (1 + rng.choice([-1e-6, 0.0, 1e-7, 3e-7, 1e-6, 1e-5]))
        p = rng.normal(size=3)
        p -= (p @ u) * u
        p /= np.linalg.norm(p)
        os_.append(q - rng.uniform(0.5, 40.0) * p)
        ds_.append(p * rng.choice([0.01, 1.0, 100.0]))
    return np.array(os_, f32), np.array(ds_, f32)


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
            # the bound covers the member: Rk >= R (float64 geometry), and so do the node's
            # and the chunk's
            for tab, i in (("bound", h), ("node", h // 8), ("top", h // 64)):
                e, b = i % 2, t[tab][i // 2]
                C = np.array([b[0 + e], b[2 + e], b[4 + e]], np.float64)
                dist = np.linalg.norm(sp["center"][j].astype(np.float64) - C)
                assert dist + abs(float(sp["radius"][j])) <= float(b[8 + e]), (tab, i)


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
    for o, d in chunks:
        culled = group_culled(t, o, d, rng=rng)
        disc = member_disc(t, o, d)
        hit = (~(disc < 0)) & valid[None]
        bad = culled[:, :, None] & hit
        assert not bad.any(), f"{int(bad.sum())} culled group members with disc >= 0"
        # a culled node (8 consecutive groups) holds no hit either
        node_culled = np.repeat(group_culled(t, o, d, "node", rng=rng), 8, axis=1)
        bad = node_culled[:, :, None] & hit
        assert not bad.any(), f"{int(bad.sum())} culled node members with disc >= 0"
        G = hit.shape[1]
        top_culled = np.repeat(group_culled(t, o, d, "top", rng=rng), 64, axis=1)[:, :G]
        bad = top_culled[:, :, None] & hit
        assert not bad.any(), f"{int(bad.sum())} culled top-level members with disc >= 0"
        total_culled += int(culled.sum())
        total += culled.size
    # and the test does cull (most groups are far from most rays)
    assert total_culled > 0.5 * total


def test_checker_detects_a_too_small_bound():
    """The emulated check above has teeth: bounds shrunk by 1% are caught."""
    rng = np.random.default_rng(11)
    sp = S.builtin_scene("final")
    t = S.cull_tables(sp)
    bad_t = {k: (v.copy() if hasattr(v, "copy") else v) for k, v in t.items()}
    bad_t["bound"][:, 6:8] = 0                   # no margin
    bad_t["bound"][:, 8:10] *= f32(0.99)         # radius 1% short
    o, d = tangent_rays(sp, t, 1500, rng)
    culled = group_culled(bad_t, o, d)
    hit = ~(member_disc(t, o, d) < 0) & (t["index"][t["nbig"]:] >= 0)[None]
    assert (culled[:, :, None] & hit).any()


def test_margin_constants():
    """K and Rk as tracer.hip derives them: K >= 32.4u / r_min (1 + 1e-5) + 6e-6 / (2R) and
    Rk >= (R + 1.5 Kc R^2)(1 + 1e-5) with R the covering radius."""
    sp = S.builtin_scene("final")
    t = S.cull_tables(sp)
    u = 2.0 ** -24
    nb = t["nbig"]
    for gi in range(t["geom"].shape[0] - nb):
        m = t["index"][nb + gi][t["index"][nb + gi] >= 0]
        if len(m) == 0:
            continue
        e, bb = gi % 2, t["bound"][gi // 2]
        C = bound_of(t, gi)
        r = np.abs(sp["radius"][m].astype(np.float64))
        R = (np.linalg.norm(sp["center"][m].astype(np.float64) - C, axis=1) + r).max()
        Kc = 32.4 * u / r.min()
        assert float(bb[6 + e]) >= Kc * (1 + 1e-5) + 6e-6 / (2 * R * (1 + 1e-6))
        assert float(bb[8 + e]) >= (R + 1.5 * Kc * R * R) * (1 + 1e-5)


def test_hierarchy_is_aligned():
    """Nodes (8 groups) and chunks (64 groups) are whole k-d subtrees: a node's bound is no
    larger than the union of its groups' bounds needs (sanity: node radius <= 4x median group
    radius on the grid scenes)."""
    for name in ("final", "stress4096"):
        t = S.cull_tables(S.builtin_scene(name))
        gR = np.concatenate([t["bound"][:, 8], t["bound"][:, 9]])
        nR = np.concatenate([t["node"][:, 8], t["node"][:, 9]])
        real = nR > 0
        assert np.median(nR[real]) <= 4 * np.median(gR[gR > 0])
