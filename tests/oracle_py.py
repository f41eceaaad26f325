"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "_build", "liboracle.so")
REF_SCENEGEN = os.path.join(ORACLE_DIR, "_ref", "SceneGenerator")

SPHERE_DTYPE = np.dtype([
    ("center", np.float32, (3,)),
    ("radius", np.float32),
    ("colour", np.float32, (3,)),
    ("texture", np.float32, (3,)),
])


class OracleConfig(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32),
        ("spp", ctypes.c_int32), ("max_depth", ctypes.c_int32),
        ("lookfrom", ctypes.c_float * 3), ("lookat", ctypes.c_float * 3),
        ("vup", ctypes.c_float * 3), ("vfov", ctypes.c_float),
        ("accumulate_chunk", ctypes.c_int32),
        ("frame_spp", ctypes.c_int32),
        ("accumulate_tail", ctypes.c_int32),
        ("accumulate_tail_chunk", ctypes.c_int32),
        ("accumulate_quantum", ctypes.c_int32),
    ]


def build() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR, "all"], check=True)


class Oracle:
    def __init__(self, path: str = LIB):
        if not os.path.exists(path):
            build()
        self.lib = ctypes.CDLL(path)
        L = self.lib
        L.oracle_sin.restype = ctypes.c_float
        L.oracle_sin.argtypes = [ctypes.c_float]
        L.oracle_rand.restype = ctypes.c_float
        L.oracle_rand.argtypes = [ctypes.c_float, ctypes.c_float]
        L.oracle_camera.restype = None
        L.oracle_camera.argtypes = [ctypes.POINTER(OracleConfig), ctypes.c_void_p]
        L.oracle_render.restype = ctypes.c_int
        L.oracle_render.argtypes = [ctypes.POINTER(OracleConfig), ctypes.c_void_p, ctypes.c_int32,
                                    ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_int32, ctypes.c_int32,
                                    ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_render_pixels.restype = ctypes.c_int
        L.oracle_render_pixels.argtypes = [ctypes.POINTER(OracleConfig), ctypes.c_void_p,
                                           ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                           ctypes.c_void_p, ctypes.c_int32,
                                           ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_ray_color.restype = None
        L.oracle_ray_color.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                       ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_encode_srgb8.restype = None
        L.oracle_encode_srgb8.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.oracle_scene_generator_text.restype = ctypes.c_size_t
        L.oracle_scene_generator_text.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_reference_constants.restype = None
        L.oracle_reference_constants.argtypes = [ctypes.c_void_p]
        L.oracle_pixel_scale_log2.restype = ctypes.c_int32
        L.oracle_pixel_scale_log2.argtypes = [ctypes.c_float]
        L.oracle_render_seq.restype = ctypes.c_int
        L.oracle_render_seq.argtypes = [ctypes.POINTER(OracleConfig), ctypes.c_void_p,
                                        ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_int32, ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_render_pixels_seq.restype = ctypes.c_int
        L.oracle_render_pixels_seq.argtypes = [ctypes.POINTER(OracleConfig), ctypes.c_void_p,
                                               ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                                               ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_scene_random_spheres.restype = ctypes.c_int32
        L.oracle_scene_random_spheres.argtypes = [ctypes.c_int32] * 3 + [ctypes.c_void_p,
                                                                         ctypes.c_int32]

    # ---- math ----
    def sin(self, x: float) -> float:
        return self.lib.oracle_sin(x)

    def rand(self, x: float, y: float) -> float:
        return self.lib.oracle_rand(x, y)

    CONSTANT_NAMES = ("rand_dot_x", "rand_dot_y", "rand_scale", "min_t", "infinity", "sky_half",
                      "sky_one", "sky_bottom", "sky_top_r", "sky_top_g", "sky_top_b",
                      "jitter_offset")

    def reference_constants(self) -> dict:
        """The reference literals the oracle's restatement uses (vcrt_oracle.h order)."""
        out = np.zeros(len(self.CONSTANT_NAMES), dtype=np.float32)
        self.lib.oracle_reference_constants(out.ctypes.data)
        return dict(zip(self.CONSTANT_NAMES, out))

    @staticmethod
    def config(width, height, spp, max_depth, lookfrom=(13, 2, 3), lookat=(0, 0, 0),
               vup=(0, 1, 0), vfov=20.0, chunk=0, frame_spp=0, tail=0,
               tail_chunk=0, quantum=0) -> OracleConfig:
        c = OracleConfig()
        c.accumulate_quantum = quantum
        c.accumulate_chunk = chunk
        c.frame_spp = frame_spp
        c.accumulate_tail = tail
        c.accumulate_tail_chunk = tail_chunk
        c.width, c.height, c.spp, c.max_depth = width, height, spp, max_depth
        c.lookfrom[:] = [float(v) for v in lookfrom]
        c.lookat[:] = [float(v) for v in lookat]
        c.vup[:] = [float(v) for v in vup]
        c.vfov = float(vfov)
        return c

    def camera(self, cfg: OracleConfig) -> np.ndarray:
        out = np.zeros(15, dtype=np.float32)
        self.lib.oracle_camera(ctypes.byref(cfg), out.ctypes.data)
        return out

    @staticmethod
    def partition(stats: dict) -> dict:
        """config() keywords for the accumulation a render used (its stats): the quantum G (round
        4), with the work partition beside it (which no longer changes the image)."""
        return dict(chunk=stats["accumulate_chunk"], tail=stats["accumulate_tail"],
                    tail_chunk=stats["accumulate_tail_chunk"],
                    quantum=stats["accumulate_quantum"])

    def pixel_scale_log2(self, max_abs: float) -> int:
        """s of a pixel's quantization scale 2^s from its largest |quantum sum|
        (oracle_pixel_scale_log2)."""
        return self.lib.oracle_pixel_scale_log2(max_abs)

    # ---- render ----
    def render(self, cfg: OracleConfig, spheres: np.ndarray, rows=None, threads: int = 0):
        """Full-frame float32 [H, W, 4]; only `rows` (range(begin, end, step)) are rendered.
        Returns (image, segments)."""
        spheres = np.ascontiguousarray(spheres, dtype=SPHERE_DTYPE)
        img = np.zeros((cfg.height, cfg.width, 4), dtype=np.float32)
        if rows is None:
            rows = range(0, cfg.height, 1)
        if threads <= 0:
            threads = min(os.cpu_count() or 1, 16)
        segs = ctypes.c_uint64()
        r = self.lib.oracle_render(ctypes.byref(cfg), spheres.ctypes.data, len(spheres),
                                   img.ctypes.data, rows.start, rows.stop, rows.step or 1,
                                   threads, ctypes.byref(segs))
        if r != 0:
            raise ValueError("oracle_render rejected its arguments")
        return img, segs.value

    def render_seq(self, cfg: OracleConfig, spheres: np.ndarray, rows=None, threads: int = 0):
        """render() plus the reference's sequential fp32 sum / spp of the same rows, in one pass:
        (image, sequential image, segments)."""
        spheres = np.ascontiguousarray(spheres, dtype=SPHERE_DTYPE)
        img = np.zeros((cfg.height, cfg.width, 4), dtype=np.float32)
        seq = np.zeros_like(img)
        if rows is None:
            rows = range(0, cfg.height, 1)
        if threads <= 0:
            threads = min(os.cpu_count() or 1, 16)
        segs = ctypes.c_uint64()
        r = self.lib.oracle_render_seq(ctypes.byref(cfg), spheres.ctypes.data, len(spheres),
                                       img.ctypes.data, seq.ctypes.data, rows.start, rows.stop,
                                       rows.step or 1, threads, ctypes.byref(segs))
        if r != 0:
            raise ValueError("oracle_render_seq rejected its arguments")
        return img, seq, segs.value

    def render_pixels_seq(self, cfg: OracleConfig, spheres: np.ndarray, xy, threads: int = 0):
        """render_pixels() plus the sequential fp32 sum / spp: (rgba, sequential, segments)."""
        spheres = np.ascontiguousarray(spheres, dtype=SPHERE_DTYPE)
        xy = np.ascontiguousarray(np.asarray(xy, dtype=np.int32).reshape(-1, 2))
        out = np.zeros((len(xy), 4), dtype=np.float32)
        seq = np.zeros_like(out)
        if threads <= 0:
            threads = min(os.cpu_count() or 1, 16)
        segs = ctypes.c_uint64()
        r = self.lib.oracle_render_pixels_seq(ctypes.byref(cfg), spheres.ctypes.data,
                                              len(spheres), xy.ctypes.data, len(xy),
                                              out.ctypes.data, seq.ctypes.data, threads,
                                              ctypes.byref(segs))
        if r != 0:
            raise ValueError("oracle_render_pixels_seq rejected its arguments")
        return out, seq, segs.value

    def render_pixels(self, cfg: OracleConfig, spheres: np.ndarray, xy, threads: int = 0):
        """Pixels xy [(x, y), ...] of a W x H frame -> (float32 [len(xy), 4], segments)."""
        spheres = np.ascontiguousarray(spheres, dtype=SPHERE_DTYPE)
        xy = np.ascontiguousarray(np.asarray(xy, dtype=np.int32).reshape(-1, 2))
        out = np.zeros((len(xy), 4), dtype=np.float32)
        if threads <= 0:
            threads = min(os.cpu_count() or 1, 16)
        segs = ctypes.c_uint64()
        r = self.lib.oracle_render_pixels(ctypes.byref(cfg), spheres.ctypes.data, len(spheres),
                                          xy.ctypes.data, len(xy), out.ctypes.data, threads,
                                          ctypes.byref(segs))
        if r != 0:
            raise ValueError("oracle_render_pixels rejected its arguments")
        return out, segs.value

    def encode_srgb8(self, rgba: np.ndarray) -> np.ndarray:
        rgba = np.ascontiguousarray(rgba, dtype=np.float32)
        out = np.zeros(rgba.shape, dtype=np.uint8)
        self.lib.oracle_encode_srgb8(rgba.ctypes.data, rgba.size // 4, out.ctypes.data)
        return out

    def ray_color(self, spheres, origin, direction, max_depth):
        spheres = np.ascontiguousarray(spheres, dtype=SPHERE_DTYPE)
        o = np.asarray(origin, dtype=np.float32)
        d = np.asarray(direction, dtype=np.float32)
        out = np.zeros(3, dtype=np.float32)
        segs = ctypes.c_uint64()
        self.lib.oracle_ray_color(spheres.ctypes.data, len(spheres), o.ctypes.data,
                                  d.ctypes.data, max_depth, out.ctypes.data, ctypes.byref(segs))
        return out, segs.value

    # ---- scenes ----
    def scene_generator_text(self) -> bytes:
        n = self.lib.oracle_scene_generator_text(None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        self.lib.oracle_scene_generator_text(buf, n + 1)
        return buf.raw[:n]

    def random_spheres(self, lo, hi, max_accept=0) -> np.ndarray:
        cap = (hi - lo) ** 2
        arr = np.zeros(cap, dtype=SPHERE_DTYPE)
        n = self.lib.oracle_scene_random_spheres(lo, hi, max_accept, arr.ctypes.data, cap)
        return arr[:n].copy()

    # world[] tails (globals.glsl:513-517) and BASELINE config 1's red sphere
    @staticmethod
    def _s(c, r, col, mat, p):
        a = np.zeros(1, dtype=SPHERE_DTYPE)
        a[0]["center"], a[0]["radius"], a[0]["colour"] = c, r, col
        a[0]["texture"] = (mat, p, 0.0)
        return a

    def big_three_and_ground(self) -> np.ndarray:
        return np.concatenate([
            self._s((0, 1, 0), 1.0, (1.0, 1.0, 1.0), 3, 1.5),
            self._s((-4, 1, 0), 1.0, (0.4, 0.2, 0.1), 1, 1.0),
            self._s((4, 1, 0), 1.0, (0.7, 0.6, 0.5), 2, 1.0),
            self._s((0, -1000, 0), 1000.0, (0.5, 0.5, 0.5), 1, 1.0),
        ])

    def bright_scene(self, param: float = 3.0) -> np.ndarray:
        """A test scene (not the reference's) whose radiance passes 1 per sample: white
        Lambertian ground and balls with param (the reference's unbounded "reflect ratio",
        textures.glsl:22) > 1, so that a path's attenuation grows with every bounce. Three big
        balls and 16 small ones (the culled scans need >= 16 spheres)."""
        parts = [self._s((0, 1.2, 0), 1.0, (1.0, 1.0, 1.0), 1, param),
                 self._s((-2.2, 1.0, 0), 1.0, (0.9, 0.8, 0.7), 1, param),
                 self._s((2.2, 1.0, 0), 1.0, (0.8, 0.9, 1.0), 1, param)]
        for k in range(16):
            x, z = -3.0 + 0.4 * k, 1.6 + 0.3 * (k % 3)
            parts.append(self._s((x, 0.15, z), 0.15, (1.0, 0.9 - 0.02 * k, 0.6 + 0.02 * k), 1,
                                 param))
        parts.append(self._s((0, -1000, 0), 1000.0, (1.0, 1.0, 1.0), 1, param))
        return np.concatenate(parts)

    def scene(self, name: str) -> np.ndarray:
        if name == "bright":
            return self.bright_scene()
        if name == "final":
            return np.concatenate([self.random_spheres(-11, 11), self.big_three_and_ground()])
        if name == "three":
            return self.big_three_and_ground()
        if name == "red":
            return np.concatenate([self._s((0, 1, 0), 1.0, (1.0, 0.0, 0.0), 1, 1.0),
                                   self.big_three_and_ground()[3:]])
        if name == "stress4096":
            return np.concatenate([self.random_spheres(-33, 33, 4096),
                                   self.big_three_and_ground()])
        raise KeyError(name)


_singleton = None


def load() -> Oracle:
    global _singleton
    if _singleton is None:
        _singleton = Oracle()
    return _singleton
