// pt/scenes.hpp -- the reference's three scenes, values as in
// simple_scene.hpp:14-52, box_scene.hpp:14-72 and box_mirror_scene.hpp:14-72
// (same double expressions), plus the synthetic N-sphere scene of
// BASELINE.json configs[4] (defined in DESIGN.md; the reference has none).
// Unlike the reference (whose box headers both define pt::box_scene under one
// include guard), the two box variants get distinct names here.
#pragma once

#include <cstdint>
#include <random>

#include "types.hpp"

namespace pt {

namespace detail {
inline scene finish(scene scn, int w, int h, double fov, double aperture)
{
    auto &c = scn.camera_parameters;
    c.aspect_ratio = (w * 1.0) / (h * 1.0);
    c.vertical_fov_radians = fov;
    c.aperture = aperture;
    c.focus_distance = (c.position - c.direction).length();
    return scn;
}

inline scene box(int w, int h, bool mirror)
{
    constexpr double big = 1E6, off = 0.4, y = 0.0, z = -1.0;
    auto const wall = mirror ? reflection_type::specular : reflection_type::diffuse;
    vec3 const black{0.0, 0.0, 0.0};
    vec3 const white{1.0, 1.0, 1.0};
    scene scn{};
    scn.spheres = {
        {big, {-big - off, y, z}, black, {0.9, 0.1, 0.2}, wall},
        {big, {big + off, y, z}, black, {0.3, 0.1, 0.9}, wall},
        {big, {0.0, 0.0, z - big}, black, {0.1, 0.7, 0.2}, wall},
        {big, {0.0, big + off, z}, black, {0.3, 0.7, 0.2}, wall},
        {big, {0.0, -big - off, z}, black, {0.9, 0.9, 0.9}, wall},
    };
    if (mirror) {
        vec3 const light{1.92, 1.91, 1.9};
        scn.spheres.push_back({off / 2.0, {0.0, 0.0 + off / 4.0, z + off * 1.5}, light, light, reflection_type::diffuse});
        scn.spheres.push_back({off / 2.0, {off / 2.0, -off / 2.0, z + off}, black, white, reflection_type::specular});
        scn.spheres.push_back({off / 2.0, {-off / 2.0, -off / 2.0, z + off}, black, white, reflection_type::dielectric});
    } else {
        scn.spheres.push_back(
            {off / 2.0, {0.0, 0.0 + off / 4.0, z - off / 2.5}, {9.0, 9.0, 9.0}, {1.8, 1.8, 1.8}, reflection_type::diffuse});
        scn.spheres.push_back({off / 2.0, {off / 2.0, -off / 2.0, z + off * 1.5}, black, white, reflection_type::specular});
        scn.spheres.push_back(
            {off / 2.0, {-off / 2.0, -off / 2.0, z + off * 1.5}, black, white, reflection_type::dielectric});
    }
    scn.camera_parameters.position = vec3{0.0, 0.0, 2.0};
    scn.camera_parameters.direction = vec3{0.0, 0.0, z + off * 1.5};
    return finish(scn, w, h, mirror ? 0.75 : 0.5, 0.2);
}
}  // namespace detail

[[nodiscard]] inline scene simple_scene(int w, int h)
{
    vec3 const black{0.0, 0.0, 0.0};
    scene scn{};
    scn.spheres = {
        {100.0, {0.0, -100.5, -1.0}, black, {0.8, 0.8, 0.0}, reflection_type::diffuse},
        {0.5, {1.0, 0.0, -1.0}, black, {0.999, 0.999, 0.999}, reflection_type::specular},
        {0.5, {-1.0, 0.0, -1.0}, black, {0.999, 0.999, 0.999}, reflection_type::dielectric},
        {0.5, {0.0, 0.0, -1.0}, {0.1, 0.1, 0.9}, {0.0, 0.7, 0.1}, reflection_type::diffuse},
        {1.0, {1.0, 3.1, -1.0}, {30.0, 30.0, 30.0}, black, reflection_type::diffuse},
    };
    scn.camera_parameters.position = vec3{-2.0, 2.0, 1.0};
    scn.camera_parameters.direction = vec3{0.0, 0.0, -1.0};
    return detail::finish(scn, w, h, 1.2, 0.2);
}

[[nodiscard]] inline scene box_scene(int w, int h) { return detail::box(w, h, false); }
[[nodiscard]] inline scene box_mirror_scene(int w, int h) { return detail::box(w, h, true); }

// std::mt19937(gen_seed) + generate_canonical<double,53>, 7 draws per sphere.
[[nodiscard]] inline scene synthetic_scene(int n, int w, int h, std::uint32_t gen_seed = 42)
{
    std::mt19937 g{gen_seed};
    std::uniform_real_distribution<double> u{0.0, 1.0};
    vec3 const black{0.0, 0.0, 0.0};
    scene scn{};
    scn.spheres.push_back({1000.0, {0.0, -1000.0, 0.0}, black, {0.5, 0.5, 0.5}, reflection_type::diffuse});
    scn.spheres.push_back({2.0, {0.0, 8.0, 0.0}, {8.0, 8.0, 8.0}, {0.8, 0.8, 0.8}, reflection_type::diffuse});
    for (int i = 2; i < n; ++i) {
        double const r = 0.05 + 0.1 * u(g);
        double const x = -10.0 + 20.0 * u(g);
        double const zz = -10.0 + 20.0 * u(g);
        double const m = u(g);
        double const cr = 0.2 + 0.75 * u(g);
        double const cg = 0.2 + 0.75 * u(g);
        double const cb = 0.2 + 0.75 * u(g);
        auto const mat = m < 0.80 ? reflection_type::diffuse : (m < 0.95 ? reflection_type::specular : reflection_type::dielectric);
        scn.spheres.push_back({r, {x, r, zz}, black, {cr, cg, cb}, mat});
    }
    scn.camera_parameters.position = vec3{0.0, 2.0, 12.0};
    scn.camera_parameters.direction = vec3{0.0, 0.0, 0.0};
    return detail::finish(scn, w, h, 0.8, 0.0);
}

}  // namespace pt
