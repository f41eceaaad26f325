"""ctypes view of the C ABI in include/vcrt.h (libvcrt.so, built in-tree by ``make``).

There is no fallback: if the library is missing the import of the renderer fails loudly.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libvcrt.so")
CODE_OBJECT_PATH = os.path.join(LIB_DIR, "vcrt_tracer.hsaco")
BIN_DIR = os.path.join(HERE, "bin")

# VkResult values (vcrt.h)
VK_SUCCESS = 0
VK_NOT_READY = 1
VK_ERROR_OUT_OF_HOST_MEMORY = -1
VK_ERROR_OUT_OF_DEVICE_MEMORY = -2
VK_ERROR_INITIALIZATION_FAILED = -3
VK_ERROR_DEVICE_LOST = -4
VK_ERROR_FEATURE_NOT_PRESENT = -8
VK_ERROR_FORMAT_NOT_SUPPORTED = -11
VK_ERROR_UNKNOWN = -13
VK_ERROR_INCOMPATIBLE_SHADER_BINARY_EXT = 1000482000

TEXTURE_LAMBERTIAN = 1
TEXTURE_METAL = 2
TEXTURE_GLASS = 3

KERNEL_AUTO = 0
KERNEL_LDS = 1
KERNEL_SMEM = 2
KERNEL_CULL = 3
KERNEL_CULL_LANE = 4
KERNEL_CULL_FLAT = 5

SCENE_FINAL = 0
SCENE_THREE = 1
SCENE_RED = 2
SCENE_STRESS4096 = 3


class vcrt_sphere(ctypes.Structure):
    _fields_ = [
        ("center", ctypes.c_float * 3),
        ("radius", ctypes.c_float),
        ("colour", ctypes.c_float * 3),
        ("texture", ctypes.c_float * 3),
    ]


class vcrt_camera(ctypes.Structure):
    _fields_ = [
        ("lookfrom", ctypes.c_float * 3),
        ("lookat", ctypes.c_float * 3),
        ("vup", ctypes.c_float * 3),
        ("vfov", ctypes.c_float),
    ]


class vcrt_render_desc(ctypes.Structure):
    _fields_ = [
        ("struct_size", ctypes.c_uint32),
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("samples_per_pixel", ctypes.c_int32),
        ("max_depth", ctypes.c_int32),
        ("camera", vcrt_camera),
        ("device", ctypes.c_int32),
        ("rank", ctypes.c_int32),
        ("world_size", ctypes.c_int32),
        ("kernel_variant", ctypes.c_int32),
        ("blocks_per_cu", ctypes.c_int32),
        ("accumulate_chunk", ctypes.c_int32),
        ("progressive", ctypes.c_int32),
        ("code_object_path", ctypes.c_char_p),
        ("accumulate_tail", ctypes.c_int32),
        ("accumulate_tail_chunk", ctypes.c_int32),
        ("accumulate_quantum", ctypes.c_int32),
    ]


class vcrt_stats(ctypes.Structure):
    _fields_ = [
        ("segments", ctypes.c_uint64),
        ("sphere_tests", ctypes.c_uint64),
        ("samples", ctypes.c_uint64),
        ("kernel_ms", ctypes.c_double),
        ("frame_ms", ctypes.c_double),
        ("resolve_ms", ctypes.c_double),
        ("gather_ms", ctypes.c_double),
        ("frames", ctypes.c_int32),
        ("grid_blocks", ctypes.c_int32),
        ("block_threads", ctypes.c_int32),
        ("kernel_variant", ctypes.c_int32),
        ("local_tiles", ctypes.c_int32),
        ("nspheres", ctypes.c_int32),
        ("lds_bytes", ctypes.c_uint32),
        ("accumulate_chunk", ctypes.c_int32),
        ("tables_in_lds", ctypes.c_int32),
        ("accumulated_spp", ctypes.c_uint64),
        ("group_tests", ctypes.c_uint64),
        ("bound_tests", ctypes.c_uint64),
        ("kernel", ctypes.c_char * 48),
        ("debug", ctypes.c_uint64 * 128),
        ("accumulate_tail", ctypes.c_int32),
        ("accumulate_tail_chunk", ctypes.c_int32),
        ("ring_entries", ctypes.c_int32),
        ("accumulate_quantum", ctypes.c_int32),
        ("accumulate_scale_log2", ctypes.c_int32),
        ("cost_order", ctypes.c_int32),
        ("scale_rerenders", ctypes.c_int32),
    ]


class vcrt_comm_id(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]  # an ncclUniqueId


# name -> (restype, argtypes); every symbol include/vcrt.h declares.
SIGNATURES = {
    "vcrt_default_desc": (ctypes.c_int32, [ctypes.POINTER(vcrt_render_desc)]),
    "vcrt_begin": (ctypes.c_int32, [ctypes.POINTER(vcrt_render_desc)]),
    "vcrt_work_quantum": (ctypes.c_int32, [ctypes.POINTER(vcrt_render_desc)]),
    "vcrt_work_chunk": (ctypes.c_int32, [ctypes.POINTER(vcrt_render_desc)]),
    "vcrt_work_tail": (ctypes.c_int32, [ctypes.POINTER(vcrt_render_desc),
                                        ctypes.POINTER(ctypes.c_int32)]),
    "vcrt_pixel_scale_log2": (ctypes.c_int32, [ctypes.c_float]),
    "vcrt_set_scene": (ctypes.c_int32, [ctypes.POINTER(vcrt_sphere), ctypes.c_int32]),
    "vcrt_draw_next_frame": (ctypes.c_int32, []),
    "vcrt_end": (ctypes.c_int32, []),
    "vcrt_comm_unique_id": (ctypes.c_int32, [ctypes.POINTER(vcrt_comm_id)]),
    "vcrt_comm_init": (ctypes.c_int32, [ctypes.POINTER(vcrt_comm_id)]),
    "vcrt_local_layout": (ctypes.c_int32, [ctypes.POINTER(ctypes.c_uint32),
                                           ctypes.POINTER(ctypes.c_uint32)]),
    "vcrt_read_framebuffer": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_size_t]),
    "vcrt_framebuffer_device": (
        ctypes.c_int32, [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]),
    "vcrt_set_framebuffer_device": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_size_t]),
    "vcrt_assemble_tiles": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_void_p] +
                            [ctypes.c_int32] * 3 + [ctypes.c_uint32]),
    "vcrt_get_stats": (ctypes.c_int32, [ctypes.POINTER(vcrt_stats)]),
    "vcrt_reset_accumulation": (ctypes.c_int32, []),
    "vcrt_read_framebuffer_srgb8": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_size_t]),
    "vcrt_selftest_sin": (ctypes.c_int32, [ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.POINTER(ctypes.c_uint32)]),
    "vcrt_srgb8_thresholds": (None, [ctypes.c_void_p]),
    "vcrt_shader_load": (ctypes.c_int32, [ctypes.c_char_p]),
    "vcrt_scene_builtin": (ctypes.c_int32,
                           [ctypes.c_int32, ctypes.POINTER(vcrt_sphere), ctypes.c_int32]),
    "vcrt_scene_generator_text": (ctypes.c_size_t, [ctypes.c_char_p, ctypes.c_size_t]),
    "vcrt_cull_tables": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                                          ctypes.c_void_p, ctypes.c_int32]),
    "vcrt_primary_lists": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_int32,
                                            ctypes.POINTER(vcrt_render_desc), ctypes.c_void_p,
                                            ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]),
    "vcrt_primary_sphere_lists": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_int32,
                                                   ctypes.POINTER(vcrt_render_desc),
                                                   ctypes.c_void_p, ctypes.c_int32,
                                                   ctypes.c_void_p, ctypes.c_int32]),
    "vcrt_canonical_sin": (ctypes.c_float, [ctypes.c_float]),
    "vcrt_canonical_rand": (ctypes.c_float, [ctypes.c_float, ctypes.c_float]),
    "vcrt_result_string": (ctypes.c_char_p, [ctypes.c_int32]),
}

_lib = None


def _share_torch_hip_runtime() -> None:
    """One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 (SONAME
    libamdhip64.so.7, the same as /opt/rocm's). If it is loaded first, libvcrt.so's
    DT_NEEDED libamdhip64.so.7 binds to it and torch tensors, streams and RCCL share one runtime
    with the tracer; loaded the other way round the process would hold two HIP/HSA runtimes."""
    try:
        import torch  # noqa: F401
    except ImportError:
        return
    # the same for RCCL (SONAME librccl.so.1 in both): libvcrt's gather and torch's
    # process group then use one RCCL
    for name in ("libamdhip64.so", "librccl.so"):
        torch_lib = os.path.join(os.path.dirname(torch.__file__), "lib", name)
        if os.path.exists(torch_lib):
            ctypes.CDLL(torch_lib, mode=ctypes.RTLD_GLOBAL)


def lib() -> ctypes.CDLL:
    """Load libvcrt.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `make -C {HERE}` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        if os.environ.get("VCRT_SYSTEM_HIP", "0") != "1":
            _share_torch_hip_runtime()
        handle = ctypes.CDLL(LIB_PATH)
        for name, (restype, argtypes) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = restype
            fn.argtypes = argtypes
        _lib = handle
    return _lib


def result_string(code: int) -> str:
    return lib().vcrt_result_string(code).decode()


class VcrtError(RuntimeError):
    def __init__(self, where: str, code: int):
        super().__init__(f"{where} failed: {result_string(code)} ({code})")
        self.code = code


def check_count(where: str, value: int) -> int:
    """A count-or-VkResult return: negative values are errors."""
    if value < 0:
        raise VcrtError(where, value)
    return value


def check(where: str, code: int) -> int:
    if code != VK_SUCCESS:
        raise VcrtError(where, code)
    return code
