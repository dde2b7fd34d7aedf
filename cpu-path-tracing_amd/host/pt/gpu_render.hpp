// pt/gpu_render.hpp -- the drop-in for the reference's row loop
// (src/main.cpp:214-236).  Where main() did
//
//     tf::Executor executor{}; tf::Taskflow taskflow{};
//     for (int y = 0; y < height; y++) taskflow.emplace([...] { ... render_subpixel ... });
//     executor.run(taskflow).wait();
//
// it now calls
//
//     pt::gpu::render_image(some_scene, cam, image, width, height, samps, num_subpixels);
//
// with the same scene, camera, zero-initialised std::vector<pt::vec3> image and
// ints; the image afterwards holds what the loop would leave in it (the same
// estimator, fp32 arithmetic, counter-RNG draws).  Errors surface as a
// negative ptg_status, like the C ABI (the reference has no error channel).
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

#include "ptgpu.h"
#include "types.hpp"

namespace pt {

static_assert(sizeof(vec3) == 24, "pt::vec3 must be 3 packed doubles");
static_assert(sizeof(sphere) == sizeof(ptg_sphere), "pt::sphere layout != ptg_sphere");
static_assert(offsetof(sphere, position) == offsetof(ptg_sphere, position), "pt::sphere layout");
static_assert(offsetof(sphere, emission) == offsetof(ptg_sphere, emission), "pt::sphere layout");
static_assert(offsetof(sphere, color) == offsetof(ptg_sphere, color), "pt::sphere layout");
static_assert(offsetof(sphere, reflection) == offsetof(ptg_sphere, material), "pt::sphere layout");
static_assert(sizeof(reflection_type) == sizeof(int32_t), "reflection_type must be an int");
static_assert(sizeof(camera) == sizeof(ptg_camera), "pt::camera layout != ptg_camera");
static_assert(offsetof(camera, lens_radius) == offsetof(ptg_camera, lens_radius), "pt::camera layout");

namespace gpu {

inline constexpr std::uint64_t default_seed = 0x5EED0001ull;

// main.cpp:214-236 replacement.  `samps` is per sub-pixel (main.cpp:206).
inline int render_image(scene const &scn, camera const &cam, std::vector<vec3> &image, int width, int height,
                        int samps, int num_subpixels = 2, std::uint64_t seed = default_seed, int device = -1,
                        int flags = 0)
{
    if (image.size() != static_cast<std::size_t>(width) * static_cast<std::size_t>(height))
        return PTG_ERR_INVALID_ARGUMENT;
    ptg_params p{};
    p.width = width;
    p.height = height;
    p.samples = samps;
    p.num_subpixels = num_subpixels;
    p.seed = seed;
    p.band_rows = 1;  // single-row bands: equal shards whenever shard_count divides H
    p.shard_rank = 0;
    p.shard_count = 1;
    p.flags = flags;  // e.g. PTG_FLAG_EXACT_MATH: bit for bit the CPU oracle's image
    return ptg_render(reinterpret_cast<ptg_sphere const *>(scn.spheres.data()), scn.spheres.size(),
                      reinterpret_cast<ptg_camera const *>(&cam), &p, device,
                      reinterpret_cast<double *>(image.data()));
}

}  // namespace gpu
}  // namespace pt
