"""Python mirror of the reference's Renderer lifecycle (include/Renderer.hpp:14-20).

``BeginRenderingOperation`` / ``DrawNextFrame`` / ``EndRenderingOperation`` keep the reference's
names and VkResult return convention (0 = VK_SUCCESS, negative = error). ``RenderDesc`` carries
what the reference fixed at compile time (globals.glsl:9-24). ``Renderer`` is the same lifecycle
as a context manager that raises on error. Everything goes through libvcrt.so (the C ABI of
include/vcrt.h); the compute runs in the gfx950 kernels of vcrt_tracer.hsaco.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _native as N
from .scene import SPHERE_DTYPE, builtin_scene


@dataclass
class RenderDesc:
    width: int = 1280               # IMAGE_WIDTH  (globals.glsl:16)
    height: int = 720               # IMAGE_HEIGHT (globals.glsl:17)
    samples_per_pixel: int = 1      # SAMPLES_PER_PIXEL (globals.glsl:9-13)
    max_depth: int = 50             # MAX_RECURSION_LEVEL (globals.glsl:14)
    lookfrom: tuple = (13.0, 2.0, 3.0)   # globals.glsl:21-24
    lookat: tuple = (0.0, 0.0, 0.0)
    vup: tuple = (0.0, 1.0, 0.0)
    vfov: float = 20.0
    device: int = -1
    rank: int = 0
    world_size: int = 1             # shards: rank owns the 8x8 tiles with (tx + ty) % world == rank
    kernel_variant: int = N.KERNEL_AUTO
    blocks_per_cu: int = 0
    accumulate_chunk: int = 0       # samples per work item: 0 = from the frame (work_chunk)
    progressive: bool = False       # frame f continues the sample sequence; average of all frames
    code_object_path: str | None = None
    accumulate_tail: int = 0        # tail samples per pixel: 0 = the rule (work_tail), -1 = none
    accumulate_tail_chunk: int = 0  # samples per tail item; 0 = the rule
    accumulate_quantum: int = 0     # accumulation quantum G (the image depends on it alone):
                                    # 0 = the rule (work_quantum); >= spp: sequential order
    _path_keepalive: bytes | None = field(default=None, repr=False)

    def to_c(self) -> N.vcrt_render_desc:
        d = N.vcrt_render_desc()
        N.lib().vcrt_default_desc(ctypes.byref(d))
        d.width, d.height = self.width, self.height
        d.samples_per_pixel, d.max_depth = self.samples_per_pixel, self.max_depth
        d.camera.lookfrom[:] = [float(v) for v in self.lookfrom]
        d.camera.lookat[:] = [float(v) for v in self.lookat]
        d.camera.vup[:] = [float(v) for v in self.vup]
        d.camera.vfov = float(self.vfov)
        d.device = self.device
        d.rank, d.world_size = self.rank, self.world_size
        d.kernel_variant = self.kernel_variant
        d.blocks_per_cu = self.blocks_per_cu
        d.accumulate_chunk = self.accumulate_chunk
        d.progressive = 1 if self.progressive else 0
        d.accumulate_tail = self.accumulate_tail
        d.accumulate_tail_chunk = self.accumulate_tail_chunk
        d.accumulate_quantum = self.accumulate_quantum
        if self.code_object_path:
            self._path_keepalive = self.code_object_path.encode()
            d.code_object_path = self._path_keepalive
        return d


def work_quantum(desc: RenderDesc) -> int:
    """The accumulation quantum G the renderer uses for `desc`, from the C ABI
    (vcrt_work_quantum: host only, no GPU): the oracle's `quantum` for the same image."""
    return N.check_count("vcrt_work_quantum",
                         N.lib().vcrt_work_quantum(ctypes.byref(desc.to_c())))


def work_chunk(desc: RenderDesc) -> int:
    """Samples per work item of the head the renderer uses for `desc`, from the C ABI
    (vcrt_work_chunk: host only, no GPU). A scheduling choice: the image depends on the
    quantum (work_quantum) only."""
    return N.check_count("vcrt_work_chunk", N.lib().vcrt_work_chunk(ctypes.byref(desc.to_c())))


def work_tail(desc: RenderDesc) -> tuple[int, int]:
    """(tail samples per pixel, samples per tail item) the renderer uses for `desc`, from the
    C ABI (vcrt_work_tail: host only, no GPU); (0, 0) when there is no tail."""
    kt = ctypes.c_int32(0)
    t = N.check_count("vcrt_work_tail", N.lib().vcrt_work_tail(ctypes.byref(desc.to_c()),
                                                                ctypes.byref(kt)))
    return (t, kt.value) if t > 0 else (0, 0)


def pixel_scale_log2(max_abs_quantum_sum: float) -> int:
    """s of a pixel's quantization scale 2^s from its largest |quantum sum| (vcrt_pixel_scale_log2:
    host only, no GPU): 32 below 2^12, else the largest s with max * 2^s < 2^44. The oracle
    restates the same rule (oracle_pixel_scale_log2)."""
    return N.lib().vcrt_pixel_scale_log2(float(max_abs_quantum_sum))


def tiles_for_rank(width: int, height: int, world: int, rank: int) -> list[int]:
    """Row-major 8x8 tile indices (ty * tiles_x + tx) rank `rank` renders, in its local order:
    the tiles with (tx + ty) % world == rank (csrc/vcrt_math.h tile_of)."""
    tx_n, ty_n = (width + 7) // 8, (height + 7) // 8
    return [ty * tx_n + tx for ty in range(ty_n) for tx in range(tx_n)
            if (tx + ty) % world == rank]


def tile_slots(width: int, height: int, world: int = 1, rank: int = 0) -> int:
    """64 work slots per owned tile (edge tiles included whole)."""
    return 64 * len(tiles_for_rank(width, height, world, rank))


def tile_pixel_map(width: int, height: int, world: int) -> np.ndarray:
    """For every frame pixel [y, x]: (rank, element index in that rank's packed tile buffer).
    The host statement of the index map the vcrt_assemble kernel applies (owner_of)."""
    tx_n, ty_n = (width + 7) // 8, (height + 7) // 8
    rank_of = np.zeros((ty_n, tx_n), np.int64)
    local_of = np.zeros((ty_n, tx_n), np.int64)
    for r in range(world):
        for lt, t in enumerate(tiles_for_rank(width, height, world, r)):
            rank_of[t // tx_n, t % tx_n] = r
            local_of[t // tx_n, t % tx_n] = lt
    y, x = np.mgrid[0:height, 0:width]
    return np.stack([rank_of[y // 8, x // 8],
                     local_of[y // 8, x // 8] * 64 + (y % 8) * 8 + x % 8], axis=-1)


# ---- reference-named lifecycle (VkResult codes, no exceptions) ----------------------------

_desc = RenderDesc()
_scene: np.ndarray | None = None


def SetRenderDescription(desc: RenderDesc) -> int:
    global _desc
    _desc = desc
    return N.VK_SUCCESS


def SetRenderScene(spheres) -> int:
    global _scene
    _scene = None if spheres is None else np.ascontiguousarray(spheres, dtype=SPHERE_DTYPE)
    return N.VK_SUCCESS


# The C ABI holds one renderer per process (vcrt.h): a vcrt_begin ends the one before it. The
# Renderer object that owns the current state; an older one is stale and its calls raise
# instead of acting on its successor's state (or ending it on close).
_live = None


def _retire_live() -> None:
    global _live
    if _live is not None:
        _live._open = False
        _live = None


def BeginRenderingOperation() -> int:
    _retire_live()
    lib = N.lib()
    d = _desc.to_c()
    r = lib.vcrt_begin(ctypes.byref(d))
    if r == N.VK_SUCCESS and _scene is not None:
        r = lib.vcrt_set_scene(_scene.ctypes.data_as(ctypes.POINTER(N.vcrt_sphere)), len(_scene))
        if r != N.VK_SUCCESS:
            lib.vcrt_end()
    return r


def DrawNextFrame() -> int:
    return N.lib().vcrt_draw_next_frame()


def EndRenderingOperation() -> int:
    _retire_live()
    return N.lib().vcrt_end()


# ---- the same lifecycle as an object --------------------------------------------------------

class Renderer:
    """Begin on construction / __enter__, End on close / __exit__; raises VcrtError."""

    def __init__(self, desc: RenderDesc | None = None, scene=None):
        self.desc = desc or RenderDesc()
        self._lib = N.lib()
        self._frame_stats = N.vcrt_stats()  # frame_times()' reused struct
        self._c_desc = self.desc.to_c()
        _retire_live()  # vcrt_begin ends the previous renderer's state
        N.check("vcrt_begin", self._lib.vcrt_begin(ctypes.byref(self._c_desc)))
        global _live
        _live = self
        self._open = True
        if scene is not None:
            self.set_scene(scene)

    def _L(self):
        """The library, for the renderer that owns the C ABI's state; a stale one raises."""
        if not getattr(self, "_open", False) or _live is not self:
            raise N.VcrtError("Renderer (closed, or replaced by a later one)",
                              N.VK_ERROR_INITIALIZATION_FAILED)
        return self._lib

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def close(self):
        global _live
        if getattr(self, "_open", False) and _live is self:
            self._lib.vcrt_end()
            _live = None
        self._open = False

    def set_scene(self, scene) -> None:
        arr = builtin_scene(scene) if isinstance(scene, (str, int)) else scene
        arr = np.ascontiguousarray(arr, dtype=SPHERE_DTYPE)
        self._scene = arr
        N.check("vcrt_set_scene", self._L().vcrt_set_scene(
            arr.ctypes.data_as(ctypes.POINTER(N.vcrt_sphere)), len(arr)))

    def draw_next_frame(self) -> None:
        N.check("vcrt_draw_next_frame", self._L().vcrt_draw_next_frame())

    def comm_init(self, comm_id: bytes) -> None:
        """Join the multi-GPU frame gather (vcrt_comm_init, RCCL inside libvcrt): every rank
        passes the same id (comm_unique_id() of rank 0). Afterwards draw_next_frame on rank 0
        returns the whole frame, which read_framebuffer gives as [height, width, 4]."""
        raw = bytes(comm_id)
        if len(raw) != ctypes.sizeof(N.vcrt_comm_id):
            raise ValueError("a comm id is 128 bytes (vcrt_comm_unique_id)")
        cid = N.vcrt_comm_id()
        ctypes.memmove(ctypes.addressof(cid), raw, len(raw))  # c_char arrays stop at NUL
        N.check("vcrt_comm_init", self._L().vcrt_comm_init(ctypes.byref(cid)))
        self._gathering = True

    def local_layout(self) -> tuple[int, int]:
        """(float4 elements, tiles) of the rank-local framebuffer."""
        e, t = ctypes.c_uint32(), ctypes.c_uint32()
        N.check("vcrt_local_layout", self._L().vcrt_local_layout(ctypes.byref(e), ctypes.byref(t)))
        return e.value, t.value

    def _frame_shape(self) -> tuple[int, ...]:
        elems, tiles = self.local_layout()
        if elems == self.desc.width * self.desc.height and (
                self.desc.world_size == 1 or getattr(self, "_gathering", False)):
            return (self.desc.height, self.desc.width, 4)
        return (tiles, 64, 4)

    def read_framebuffer(self) -> np.ndarray:
        """Framebuffer, float32 rgba: the frame [height, width, 4] (top row first) at world 1 and
        on rank 0 after comm_init; otherwise the rank's packed tiles [tiles, 64, 4] (element
        8*(y%8) + x%8)."""
        shape = self._frame_shape()
        out = np.empty(shape, dtype=np.float32)
        N.check("vcrt_read_framebuffer", self._L().vcrt_read_framebuffer(
            out.ctypes.data_as(ctypes.c_void_p), out.size))
        return out

    def read_framebuffer_srgb8(self) -> np.ndarray:
        """The rank-local framebuffer as sRGB8 RGBA (what the reference's B8G8R8A8_SRGB
        swapchain shows), uint8 with the read_framebuffer shape."""
        shape = self._frame_shape()
        out = np.empty(shape, dtype=np.uint8)
        N.check("vcrt_read_framebuffer_srgb8", self._L().vcrt_read_framebuffer_srgb8(
            out.ctypes.data_as(ctypes.c_void_p), out.size))
        return out

    def reset_accumulation(self) -> None:
        N.check("vcrt_reset_accumulation", self._L().vcrt_reset_accumulation())

    def framebuffer_device(self) -> tuple[int, int]:
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        N.check("vcrt_framebuffer_device",
                self._L().vcrt_framebuffer_device(ctypes.byref(p), ctypes.byref(n)))
        return p.value or 0, n.value

    def set_framebuffer_device(self, ptr: int | None, nbytes: int = 0) -> None:
        N.check("vcrt_set_framebuffer_device",
                self._L().vcrt_set_framebuffer_device(ctypes.c_void_p(ptr or None), nbytes))

    def assemble_tiles(self, gathered_ptr: int, frame_ptr: int, tiles_per_rank: int) -> None:
        d = self.desc
        N.check("vcrt_assemble_tiles", self._L().vcrt_assemble_tiles(
            ctypes.c_void_p(gathered_ptr), ctypes.c_void_p(frame_ptr), d.width, d.height,
            d.world_size, tiles_per_rank))

    def shader_load(self, path: str) -> None:
        N.check("vcrt_shader_load", self._L().vcrt_shader_load(path.encode()))

    def frame_times(self) -> tuple:
        """(kernel_ms, segments, gather_ms, frame_ms) of the last frame: vcrt_get_stats into a
        reused struct, without building stats()'s dict (a timed loop's per-frame bookkeeping)."""
        s = self._frame_stats
        N.check("vcrt_get_stats", self._L().vcrt_get_stats(ctypes.byref(s)))
        return s.kernel_ms, s.segments, s.gather_ms, s.frame_ms

    def stats(self) -> dict:
        s = N.vcrt_stats()
        N.check("vcrt_get_stats", self._L().vcrt_get_stats(ctypes.byref(s)))
        out = {name: getattr(s, name) for name, _ in N.vcrt_stats._fields_}
        out["debug"] = list(s.debug)
        out["kernel"] = s.kernel.decode()
        return out


def comm_unique_id() -> bytes:
    """A fresh RCCL communicator id (vcrt_comm_unique_id) for rank 0 to hand to every rank."""
    cid = N.vcrt_comm_id()
    N.check("vcrt_comm_unique_id", N.lib().vcrt_comm_unique_id(ctypes.byref(cid)))
    return ctypes.string_at(ctypes.addressof(cid), ctypes.sizeof(cid))


def render(desc: RenderDesc, scene="final", frames: int = 1) -> tuple[np.ndarray, dict]:
    """Convenience: Begin, draw `frames` frames, read the rank-local framebuffer, End."""
    with Renderer(desc, scene) as r:
        for _ in range(frames):
            r.draw_next_frame()
        return r.read_framebuffer(), r.stats()
