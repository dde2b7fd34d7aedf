"""ptgpu -- MI355X render loop for the smallpt-style path tracer
(AlexandruIca/cpu-path-tracing), host side.

The hot path (camera rays, sphere scan, radiance bounce loop, BRDFs, counter
RNG) is one HIP megakernel in libptgpu.so behind the C ABI include/ptgpu.h;
this package mirrors the reference's host-side types/scenes and binds the
ABI.  Importing it does not touch the GPU.
"""
from ._abi import ABI_VERSION, EXPORTS, LIB_PATH, Params, PtgError, lib
from .render import (DEFAULT_BAND_ROWS, DEFAULT_SEED, FLAG_COUNT_NONFINITE, FLAG_COUNT_TESTS, FLAG_EXACT_MATH, FLAG_REFERENCE_F64, Context, MultiContext, kernel_source_hash, make_params, pci_bus_id, render,
                     render_multi, render_sharded,
                     scene_layout, shard_rows, slab_to_image_rows, tonemap_device, unshard_device, unshard_host)
from .scene import (CAMERA_DT, SPHERE_DT, SceneFileError, box_mirror_scene, box_scene, camera, camera_config, length,
                    load_scene_file, make_scene, parse_scene_text, reflection_type, save_scene_file, scene, scene_text,
                    simple_scene, sphere, synthetic_scene)

__all__ = [
    "ABI_VERSION", "EXPORTS", "LIB_PATH", "Params", "PtgError", "lib",
    "DEFAULT_BAND_ROWS", "DEFAULT_SEED", "FLAG_COUNT_NONFINITE", "FLAG_COUNT_TESTS", "FLAG_EXACT_MATH", "FLAG_REFERENCE_F64", "Context", "MultiContext", "kernel_source_hash", "make_params", "pci_bus_id", "render", "render_multi",
    "render_sharded",
    "scene_layout", "shard_rows", "slab_to_image_rows", "tonemap_device", "unshard_device", "unshard_host",
    "CAMERA_DT", "SPHERE_DT", "SceneFileError", "box_mirror_scene", "box_scene", "camera", "camera_config", "length",
    "load_scene_file", "make_scene", "parse_scene_text", "reflection_type", "save_scene_file", "scene", "scene_text",
    "simple_scene", "sphere", "synthetic_scene",
]
