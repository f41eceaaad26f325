"""SceneGenerator surface (reference: SceneGenerator.cpp:10-56, globals.glsl:29-518).

Scenes are numpy structured arrays with the GLSL ``struct sphere`` layout
(structures.glsl:10-16): center[3], radius, colour[3], texture[3] -- 40 bytes per sphere.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N

SPHERE_DTYPE = np.dtype([
    ("center", np.float32, (3,)),
    ("radius", np.float32),
    ("colour", np.float32, (3,)),
    ("texture", np.float32, (3,)),
])
assert SPHERE_DTYPE.itemsize == ctypes.sizeof(N.vcrt_sphere) == 40

SCENES = {
    "final": N.SCENE_FINAL,        # 481 generated + big three + ground = 485
    "three": N.SCENE_THREE,        # big three + ground (globals.glsl:513-517)
    "red": N.SCENE_RED,            # red Lambertian sphere + ground (BASELINE config 1)
    "stress4096": N.SCENE_STRESS4096,  # 4096 generated + big three + ground = 4100
}


def builtin_scene(name_or_id) -> np.ndarray:
    """Spheres of a built-in scene, in world[] order."""
    sid = SCENES[name_or_id] if isinstance(name_or_id, str) else int(name_or_id)
    lib = N.lib()
    n = lib.vcrt_scene_builtin(sid, None, 0)
    if n < 0:
        raise N.VcrtError("vcrt_scene_builtin", n)
    arr = np.zeros(n, dtype=SPHERE_DTYPE)
    got = lib.vcrt_scene_builtin(sid, arr.ctypes.data_as(ctypes.POINTER(N.vcrt_sphere)), n)
    assert got == n
    return arr


def scene_generator_text() -> str:
    """The SceneGenerator executable's stdout, byte for byte."""
    lib = N.lib()
    n = lib.vcrt_scene_generator_text(None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    lib.vcrt_scene_generator_text(buf, n + 1)
    return buf.raw[:n].decode()


def make_spheres(rows) -> np.ndarray:
    """Build a scene from (center(3), radius, colour(3), material id, param) tuples."""
    arr = np.zeros(len(rows), dtype=SPHERE_DTYPE)
    for i, (c, r, col, mat, param) in enumerate(rows):
        arr[i]["center"] = c
        arr[i]["radius"] = r
        arr[i]["colour"] = col
        arr[i]["texture"] = (mat, param, 0.0)
    return arr


def cull_tables(spheres: np.ndarray) -> dict | None:
    """The culled scans' tables for `spheres` (host computation, no GPU): ``nbig`` big-sphere
    groups tested for every ray, then ``G`` hierarchy groups. ``geom`` [nbig + G, 16] pair-SoA
    groups and ``index`` [nbig + G, 4] world[] indices (-1 = padding), big groups first;
    ``bound`` [G/2, 12] hierarchy group-pair boxes, ``node`` [G/16, 12] node-pair boxes
    (node i = hierarchy groups 8i..8i+7), ``top`` chunk-pair boxes (entry i = hierarchy
    groups 64i..64i+63), ``margin`` the box-test constants (max |centre|, r_max^2, max |box
    coordinate|, 0). None when culling does not apply (< 16 spheres, unbounded)."""
    spheres = np.ascontiguousarray(spheres, dtype=SPHERE_DTYPE)
    lib = N.lib()
    ptr = spheres.ctypes.data
    nbig = ctypes.c_int32(0)
    g = lib.vcrt_cull_tables(ptr, len(spheres), None, None, None, None, None,
                             ctypes.byref(nbig), None, 0)
    if g == 0:
        return None
    nb = nbig.value
    geom = np.zeros((nb + g, 16), np.float32)
    bound = np.zeros((g // 2, 16), np.float32)
    node = np.zeros((g // 16, 16), np.float32)
    nt = (g + 63) // 64
    top = np.zeros(((nt + (nt & 1)) // 2, 16), np.float32)
    index = np.zeros((nb + g, 4), np.int32)
    margin = np.zeros(4, np.float32)
    got = lib.vcrt_cull_tables(ptr, len(spheres), geom.ctypes.data, bound.ctypes.data,
                               node.ctypes.data, top.ctypes.data, index.ctypes.data,
                               ctypes.byref(nbig), margin.ctypes.data, nb + g)
    assert got == g
    return {"nbig": nb, "geom": geom, "bound": bound, "node": node, "top": top, "index": index,
            "margin": margin}


def primary_lists(spheres: np.ndarray, desc) -> dict | None:
    """The flat scan's camera-ray lists (host computation, no GPU; csrc/primary.cpp) for
    `spheres` and a RenderDesc: ``info`` [4 x local tiles] uint32, entry 4 lt + 2 qy + qx for the
    4x4-pixel quarter (qx, qy) of local tile lt (offset << 4 | count, count 15 = no list), and
    ``ids`` uint16 hierarchy group indices. None without culling tables."""
    spheres = np.ascontiguousarray(spheres, dtype=SPHERE_DTYPE)
    lib = N.lib()
    d = desc.to_c()
    n = lib.vcrt_primary_lists(spheres.ctypes.data, len(spheres), ctypes.byref(d), None, 0,
                               None, 0)
    if n < 0:
        return None
    from .renderer import tiles_for_rank
    nt = 4 * len(tiles_for_rank(desc.width, desc.height, desc.world_size, desc.rank))
    info = np.zeros(nt, np.uint32)
    ids = np.zeros(max(n, 1), np.uint16)
    got = lib.vcrt_primary_lists(spheres.ctypes.data, len(spheres), ctypes.byref(d),
                                 info.ctypes.data, nt, ids.ctypes.data, len(ids))
    assert got == n
    return {"info": info, "ids": ids[:n]}


def primary_sphere_lists(spheres: np.ndarray, desc) -> dict | None:
    """The camera fast trace's per-sphere lists (host computation, no GPU; csrc/primary.cpp):
    ``info`` [4 x local tiles] uint32 (first pair << 4 | spheres, 15 = no list) and ``rec``
    [pairs, 12] float32 camera-relative pair records (ocx0 ocx1 ocy0 ocy1 ocz0 ocz1 cc0 cc1
    index0 index1 0 0, the indices as int32 bits). None without culling tables."""
    spheres = np.ascontiguousarray(spheres, dtype=SPHERE_DTYPE)
    lib = N.lib()
    d = desc.to_c()
    n = lib.vcrt_primary_sphere_lists(spheres.ctypes.data, len(spheres), ctypes.byref(d), None,
                                      0, None, 0)
    if n < 0:
        return None
    from .renderer import tiles_for_rank
    nt = 4 * len(tiles_for_rank(desc.width, desc.height, desc.world_size, desc.rank))
    info = np.zeros(nt, np.uint32)
    rec = np.zeros((max(n, 1), 12), np.float32)
    got = lib.vcrt_primary_sphere_lists(spheres.ctypes.data, len(spheres), ctypes.byref(d),
                                        info.ctypes.data, nt, rec.ctypes.data, rec.size)
    assert got == n
    return {"info": info, "rec": rec[:n]}
