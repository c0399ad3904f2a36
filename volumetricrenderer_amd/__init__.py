"""volumetricrenderer_amd -- MI355X-native volumetric ray-march integrator.

The hot path of Raspy-Py/VolumetricRenderer (shaders/frag.glsl), re-built as
hand-written HIP kernels for gfx950 behind a C ABI (include/vr.h, libvr.so).
This package is the Python host side: ctypes bindings (_lib), the renderer
interface (renderer) and the multi-GPU band sharding (distributed).
"""
from ._lib import (FMT_R8_SRGB, FMT_R8_UNORM, FMT_R32F, FMT_RGBA8_SRGB, FMT_RGBA8_UNORM, FMT_RGBA32F,  # noqa: F401
                   GREY_OF, GlobalShaderData, MarchParams, ObjectShaderData, Target, VolumeRecipe, VRError)
from ._lib import Procedural  # noqa: F401
from .renderer import (Renderer, band_rows_packed, march_defaults, procedural_defaults,  # noqa: F401
                       reference_shader_data, scaled_recipe, shader_data_arrays, volume_recipe_defaults)

__all__ = [
    "Renderer", "VRError", "march_defaults", "procedural_defaults", "Procedural", "reference_shader_data", "volume_recipe_defaults",
    "scaled_recipe", "band_rows_packed", "shader_data_arrays", "FMT_RGBA32F", "FMT_RGBA8_UNORM",
    "FMT_RGBA8_SRGB", "FMT_R8_UNORM", "FMT_R8_SRGB", "FMT_R32F", "GREY_OF", "ObjectShaderData", "GlobalShaderData", "MarchParams", "VolumeRecipe", "Target",
]
