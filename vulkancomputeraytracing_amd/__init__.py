"""MI355X-native drop-in for the fhh200000/VulkanComputeRayTracing hot path.

The per-pixel ray-gen -> sphere-list intersect -> scatter -> multi-bounce accumulate path of
shaders/shader.comp runs as hand-written HIP kernels for gfx950 (csrc/tracer.hip) behind the
C ABI of include/vcrt.h (lib/libvcrt.so). This package is the Python mirror of the reference's
host API (Renderer Begin/Draw/End, Shader loading, SceneGenerator) over that ABI.
"""
from . import _native
from ._native import (VK_SUCCESS, VK_ERROR_INITIALIZATION_FAILED, VcrtError, KERNEL_AUTO,
                      KERNEL_LDS, KERNEL_SMEM, KERNEL_CULL, KERNEL_CULL_LANE, KERNEL_CULL_FLAT,
                      TEXTURE_GLASS, TEXTURE_LAMBERTIAN, TEXTURE_METAL)
from .renderer import (BeginRenderingOperation, DrawNextFrame, EndRenderingOperation, Renderer,
                       RenderDesc, SetRenderDescription, SetRenderScene, render, tile_pixel_map,
                       tile_slots, tiles_for_rank)
from .scene import SPHERE_DTYPE, builtin_scene, make_spheres, scene_generator_text

__all__ = [
    "BeginRenderingOperation", "DrawNextFrame", "EndRenderingOperation", "Renderer",
    "RenderDesc", "SetRenderDescription", "SetRenderScene", "render", "tiles_for_rank",
    "tile_slots", "tile_pixel_map",
    "SPHERE_DTYPE", "builtin_scene", "make_spheres", "scene_generator_text", "VcrtError",
    "VK_SUCCESS", "VK_ERROR_INITIALIZATION_FAILED", "KERNEL_AUTO", "KERNEL_LDS", "KERNEL_SMEM",
    "KERNEL_CULL", "KERNEL_CULL_LANE", "KERNEL_CULL_FLAT", "TEXTURE_GLASS", "TEXTURE_LAMBERTIAN", "TEXTURE_METAL", "_native",
]
