// ref_boundary.cpp -- TEST INFRASTRUCTURE (tests/test_boundary_reference.py).
//
// The drop-in boundary checked against the reference's REAL headers
// (/root/reference/src: sphere.hpp:10-22, camera.hpp:23-43, scene.hpp:12-16,
// vec.hpp, reflection.hpp, box_scene.hpp), not the repo's re-typed mirrors:
// every field offset of pt::sphere / pt::camera equals ptg_sphere /
// ptg_camera's (include/ptgpu.h), and INTEGRATION.md section 2's casts are
// compiled and called as written -- against libptgpu.so and the reference's
// own pt library (camera::with_config, compiled from its sources by
// oracle/Makefile `ref`).  Without a visible GPU the call must fail cleanly
// with PTG_ERR_NO_DEVICE; with one it must render.
#include <cstddef>
#include <cstdio>
#include <type_traits>
#include <vector>

#include "box_scene.hpp"  // reference: pt::box_scene (box_scene.hpp:14), pulls scene/sphere/camera/vec
#include "ptgpu.h"

#define SAME_FIELD(ref, abi, rf, af)                                                             \
    static_assert(offsetof(ref, rf) == offsetof(abi, af), #ref "::" #rf " offset != " #abi "::" #af)

static_assert(std::is_standard_layout_v<pt::sphere> && std::is_standard_layout_v<pt::camera>);
static_assert(std::is_trivially_copyable_v<pt::sphere> && std::is_trivially_copyable_v<pt::camera>);
static_assert(sizeof(pt::vec3) == 3 * sizeof(double) && std::is_standard_layout_v<pt::vec3>);
static_assert(sizeof(pt::reflection_type) == sizeof(int32_t));
static_assert(static_cast<int>(pt::reflection_type::diffuse) == PTG_DIFFUSE &&
              static_cast<int>(pt::reflection_type::specular) == PTG_SPECULAR &&
              static_cast<int>(pt::reflection_type::dielectric) == PTG_DIELECTRIC);
static_assert(sizeof(pt::sphere) == sizeof(ptg_sphere) && alignof(pt::sphere) == alignof(ptg_sphere));
SAME_FIELD(pt::sphere, ptg_sphere, radius, radius);
SAME_FIELD(pt::sphere, ptg_sphere, position, position);
SAME_FIELD(pt::sphere, ptg_sphere, emission, emission);
SAME_FIELD(pt::sphere, ptg_sphere, color, color);
SAME_FIELD(pt::sphere, ptg_sphere, reflection, material);
static_assert(sizeof(pt::camera) == sizeof(ptg_camera) && alignof(pt::camera) == alignof(ptg_camera));
SAME_FIELD(pt::camera, ptg_camera, position, position);
SAME_FIELD(pt::camera, ptg_camera, lower_left_corner, lower_left_corner);
SAME_FIELD(pt::camera, ptg_camera, cam_x_axis, cam_x_axis);
SAME_FIELD(pt::camera, ptg_camera, cam_y_axis, cam_y_axis);
SAME_FIELD(pt::camera, ptg_camera, u, u);
SAME_FIELD(pt::camera, ptg_camera, v, v);
SAME_FIELD(pt::camera, ptg_camera, w, w);
SAME_FIELD(pt::camera, ptg_camera, lens_radius, lens_radius);
static_assert(offsetof(pt::vec3, x) == 0 && offsetof(pt::vec3, y) == 8 && offsetof(pt::vec3, z) == 16);

int main()
{
    // main.cpp:202-212, then INTEGRATION.md section 2 verbatim
    constexpr int width = 64, height = 48, num_subpixels = 2, samps = 2;
    auto const some_scene = pt::box_scene(width, height);
    auto const cam = pt::camera::with_config(some_scene.camera_parameters);
    std::vector<pt::vec3> image{};
    image.resize(width * height, pt::vec3{0, 0, 0});
    ptg_params p{};
    p.width = width;
    p.height = height;
    p.samples = samps;
    p.num_subpixels = num_subpixels;
    p.seed = 0x5EED0001;
    p.band_rows = 1;
    p.shard_rank = 0;
    p.shard_count = 1;
    int const rc = ptg_render(reinterpret_cast<ptg_sphere const *>(some_scene.spheres.data()),
                              some_scene.spheres.size(), reinterpret_cast<ptg_camera const *>(&cam), &p,
                              /*device=*/-1, reinterpret_cast<double *>(image.data()));
    int count = 0;
    ptg_device_count(&count);
    // the host-side preparation runs without a GPU: the box walls are paired
    int32_t axis[8], order[8];
    int const lrc = ptg_scene_layout(reinterpret_cast<ptg_sphere const *>(some_scene.spheres.data()),
                                     some_scene.spheres.size(), reinterpret_cast<ptg_camera const *>(&cam), axis, order);
    double sum = 0.0;
    for (auto const &px : image)
        sum += px.x + px.y + px.z;
    std::printf("rc %d devices %d layout %d axis %d %d %d %d %d sum %.6f err '%s'\n", rc, count, lrc, axis[0], axis[1],
                axis[2], axis[3], axis[4], sum, ptg_last_error());
    if (lrc != PTG_OK)
        return 3;
    if (count == 0)
        return rc == PTG_ERR_NO_DEVICE && sum == 0.0 ? 0 : 1;
    return rc == PTG_OK && sum > 0.0 ? 0 : 2;
}
