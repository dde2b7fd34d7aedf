// pt/types.hpp -- host-side mirror of the reference's value types, so code
// written against AlexandruIca/cpu-path-tracing's headers compiles against
// this render loop unchanged: pt::vec3 (vec.hpp:7-32), pt::ray (ray.hpp:9-15),
// pt::reflection_type (reflection.hpp:7-12), pt::sphere (sphere.hpp:10-22),
// pt::camera_config / pt::camera (camera.hpp:11-43), pt::scene (scene.hpp:12-16).
// Layouts are pinned to the C ABI structs (include/ptgpu.h) by static_asserts
// in pt/gpu_render.hpp; arithmetic follows the reference's evaluation order.
#pragma once

#include <cmath>
#include <vector>

namespace pt {

struct vec3 {
    double x{0.0};
    double y{0.0};
    double z{0.0};

    vec3() noexcept = delete;  // vec.hpp:13: not default-constructible
    vec3(double x_, double y_, double z_) noexcept : x{x_}, y{y_}, z{z_} {}

    [[nodiscard]] vec3 operator+(vec3 const &b) const noexcept { return {x + b.x, y + b.y, z + b.z}; }
    [[nodiscard]] vec3 operator-(vec3 const &b) const noexcept { return {x - b.x, y - b.y, z - b.z}; }
    [[nodiscard]] vec3 operator*(double s) const noexcept { return {x * s, y * s, z * s}; }
    [[nodiscard]] vec3 blend(vec3 const &b) const noexcept { return {x * b.x, y * b.y, z * b.z}; }
    [[nodiscard]] double dot(vec3 const &b) const noexcept { return x * b.x + y * b.y + z * b.z; }
    [[nodiscard]] vec3 cross(vec3 const &b) const noexcept
    {
        return {y * b.z - z * b.y, z * b.x - x * b.z, x * b.y - y * b.x};
    }
    // vec.cpp:35-38: normalises in place and returns *this
    vec3 &norm() noexcept { return *this = *this * (1 / std::sqrt(x * x + y * y + z * z)); }
    [[nodiscard]] double length() const noexcept { return std::hypot(x, y, z); }
};

struct ray {
    vec3 origin{0, 0, 0};
    vec3 direction{0, 0, 0};
    [[nodiscard]] vec3 at(double t) const noexcept { return origin + direction * t; }
};

enum class reflection_type { diffuse, specular, dielectric };

struct sphere {
    double radius{0.0};
    vec3 position{0, 0, 0};
    vec3 emission{0, 0, 0};
    vec3 color{0, 0, 0};
    reflection_type reflection{reflection_type::diffuse};
};

struct camera_config {
    vec3 position{0, 0, 0};
    vec3 direction{0, 0, 0};  // the look-at point (camera.cpp:8)
    vec3 up{0, 1, 0};
    double aspect_ratio{16.0 / 9.0};
    double vertical_fov_radians{0.785398163};
    double focal_length{1.0};  // unused by the reference too
    double aperture{0.0};
    double focus_distance{0.0};
};

struct camera {
    vec3 position{0, 0, 0};
    vec3 lower_left_corner{0, 0, 0};
    vec3 cam_x_axis{0, 0, 0};
    vec3 cam_y_axis{0, 0, 0};
    vec3 u{0, 0, 0};
    vec3 v{0, 0, 0};
    vec3 w{0, 0, 0};
    double lens_radius{0.0};

    // camera.cpp:3-17
    [[nodiscard]] static camera with_config(camera_config const &cfg) noexcept
    {
        double const vh = 2.0 * std::tan(0.5 * cfg.vertical_fov_radians);
        double const vw = cfg.aspect_ratio * vh;
        vec3 w_ = (cfg.position - cfg.direction).norm();
        vec3 u_ = cfg.up.cross(w_).norm();
        vec3 v_ = w_.cross(u_);
        vec3 const X = u_ * vw * cfg.focus_distance;
        vec3 const Y = v_ * vh * cfg.focus_distance;
        vec3 const llc = cfg.position - X * 0.5 - Y * 0.5 - w_ * cfg.focus_distance;
        return camera{cfg.position, llc, X, Y, u_, v_, w_, cfg.aperture / 2.0};
    }
};

struct scene {
    std::vector<sphere> spheres{};
    camera_config camera_parameters{};
};

}  // namespace pt
