// ref_golden.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Golden-vector generator.  Compiled (by oracle/Makefile, target `golden`)
// against the REFERENCE's own sources in /root/reference/src: the `pt`
// library (vec/ray/sphere/hit_record/camera/random_state/utils .cpp,
// src/CMakeLists.txt:1-9) and one scene header pre-included with -include
// (all three share the guard PT_SMALLPT_SCENE_HPP, so one binary per scene).
// src/main.cpp is NOT built: it needs cpp-taskflow 2.4.0 (conanfile.txt:3),
// which the image lacks, and no stand-in header is written for it.
//
// The determinism fix: pt::rand_state::default_with_seed multiplies the seed
// by std::random_device{}() (random_state.cpp:5), so this harness aggregate-
// initialises pt::rand_state{std::mt19937{seed}, uniform_real_distribution}
// directly (C++17 aggregate, random_state.hpp:12-22) and calls the
// reference's own generate()/generate_between().
//
// Output: one JSON document on stdout; doubles printed with %.17g (exact
// round trip).  tests/golden/*.json are produced by oracle/gen_golden.sh.
#include "camera.hpp"
#include "constants.hpp"
#include "hit_record.hpp"
#include "random_state.hpp"
#include "ray.hpp"
#include "reflection.hpp"
#include "scene.hpp"
#include "sphere.hpp"
#include "utils.hpp"
#include "vec.hpp"

#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#ifndef SCENE_FN
#error "compile with -include <scene header> -DSCENE_FN=box_scene|simple_scene -DSCENE_NAME=..."
#endif

namespace {

struct out_t {
    bool first_field = true;
    void key(const char* k)
    {
        std::printf("%s\"%s\": ", first_field ? "" : ",\n", k);
        first_field = false;
    }
};

void pd(double v) { std::printf("%.17g", v); }

void pvec(pt::vec3 const& v)
{
    std::printf("[");
    pd(v.x);
    std::printf(", ");
    pd(v.y);
    std::printf(", ");
    pd(v.z);
    std::printf("]");
}

auto seeded(unsigned seed) -> pt::rand_state
{
    return pt::rand_state{ std::mt19937{ seed }, std::uniform_real_distribution<double>{ 0.0, 1.0 } };
}

void dump_scene(out_t& o, int w, int h, char const* tag)
{
    auto const scn = pt::SCENE_FN(w, h);
    auto const cam = pt::camera::with_config(scn.camera_parameters);
    auto const& c = scn.camera_parameters;
    std::string k = std::string("scene_") + tag;
    o.key(k.c_str());
    std::printf("{\"w\": %d, \"h\": %d, \"spheres\": [", w, h);
    for(std::size_t i = 0; i < scn.spheres.size(); ++i) {
        auto const& s = scn.spheres[i];
        std::printf("%s{\"radius\": ", i ? ", " : "");
        pd(s.radius);
        std::printf(", \"position\": ");
        pvec(s.position);
        std::printf(", \"emission\": ");
        pvec(s.emission);
        std::printf(", \"color\": ");
        pvec(s.color);
        std::printf(", \"material\": %d}", static_cast<int>(s.reflection));
    }
    std::printf("], \"camera_config\": {\"position\": ");
    pvec(c.position);
    std::printf(", \"direction\": ");
    pvec(c.direction);
    std::printf(", \"up\": ");
    pvec(c.up);
    std::printf(", \"aspect_ratio\": ");
    pd(c.aspect_ratio);
    std::printf(", \"vertical_fov_radians\": ");
    pd(c.vertical_fov_radians);
    std::printf(", \"focal_length\": ");
    pd(c.focal_length);
    std::printf(", \"aperture\": ");
    pd(c.aperture);
    std::printf(", \"focus_distance\": ");
    pd(c.focus_distance);
    std::printf("}, \"camera\": {\"position\": ");
    pvec(cam.position);
    std::printf(", \"lower_left_corner\": ");
    pvec(cam.lower_left_corner);
    std::printf(", \"cam_x_axis\": ");
    pvec(cam.cam_x_axis);
    std::printf(", \"cam_y_axis\": ");
    pvec(cam.cam_y_axis);
    std::printf(", \"u\": ");
    pvec(cam.u);
    std::printf(", \"v\": ");
    pvec(cam.v);
    std::printf(", \"w\": ");
    pvec(cam.w);
    std::printf(", \"lens_radius\": ");
    pd(cam.lens_radius);
    std::printf("}}");
}

// Rays aimed at the scene: origins in the region the camera sees, plus rays
// leaving sphere surfaces (the epsilon / self-intersection cases), rays from
// inside the small spheres and grazing rays.
void dump_intersections(out_t& o, int w, int h)
{
    auto const scn = pt::SCENE_FN(w, h);
    auto rng = seeded(20240607u);
    o.key("intersect");
    std::printf("[");
    bool first = true;
    auto emit = [&](pt::ray const& r) {
        for(std::size_t i = 0; i < scn.spheres.size(); ++i) {
            auto const& s = scn.spheres[i];
            double const t = s.intersect(r);
            std::printf("%s{\"o\": ", first ? "" : ",\n ");
            first = false;
            pvec(r.origin);
            std::printf(", \"d\": ");
            pvec(r.direction);
            std::printf(", \"i\": %zu, \"t\": ", i);
            pd(t);
            if(t > 0) {
                auto const rec = pt::get_hit_record_at(s, r, t);
                std::printf(", \"p\": ");
                pvec(rec.hit_point);
                std::printf(", \"on\": ");
                pvec(rec.outward_normal);
                std::printf(", \"n\": ");
                pvec(rec.normal);
                std::printf(", \"front\": %d", rec.front_facing ? 1 : 0);
            }
            std::printf("}");
        }
    };
    for(int k = 0; k < 120; ++k) {
        pt::vec3 const org{ rng.generate_between(-0.9, 0.9),
                            rng.generate_between(-0.9, 0.9),
                            rng.generate_between(-1.5, 2.5) };
        pt::vec3 const dir{ rng.generate_between(-1.0, 1.0) * 2.5,
                            rng.generate_between(-1.0, 1.0) * 2.5,
                            rng.generate_between(-1.0, 1.0) * 2.5 };
        emit(pt::ray{ org, dir });
    }
    // rays leaving a surface point of each sphere (self-hit must be rejected by epsilon)
    for(std::size_t i = 0; i < scn.spheres.size(); ++i) {
        auto const& s = scn.spheres[i];
        for(int k = 0; k < 4; ++k) {
            pt::vec3 probe{ rng.generate_between(-0.3, 0.3), rng.generate_between(-0.3, 0.3), -1.0 };
            pt::vec3 const dir0 = probe - s.position;
            pt::vec3 const dirn = pt::vec3{ dir0 }.norm();
            pt::vec3 const surf = s.position + dirn * s.radius;
            pt::vec3 const dir{ rng.generate_between(-1.0, 1.0),
                                rng.generate_between(-1.0, 1.0),
                                rng.generate_between(-1.0, 1.0) };
            emit(pt::ray{ surf, dir });
        }
        // from the centre (inside) and a grazing ray along the tangent
        emit(pt::ray{ s.position, pt::vec3{ 0.3, -0.2, 0.9 } });
    }
    std::printf("]");
}

void dump_camera_rays(out_t& o, int w, int h)
{
    auto const scn = pt::SCENE_FN(w, h);
    auto const cam = pt::camera::with_config(scn.camera_parameters);
    o.key("get_ray");
    std::printf("[");
    for(int k = 0; k < 64; ++k) {
        unsigned const seed = 1000u + static_cast<unsigned>(k) * 7919u;
        auto rng = seeded(seed);
        double const s = (k % 8) / 8.0 + 0.03;
        double const t = (k / 8) / 8.0 + 0.07;
        auto const r = cam.get_ray(s, t, rng);
        double const next = rng.generate();
        std::printf("%s{\"seed\": %u, \"s\": ", k ? ",\n " : "", seed);
        pd(s);
        std::printf(", \"t\": ");
        pd(t);
        std::printf(", \"origin\": ");
        pvec(r.origin);
        std::printf(", \"direction\": ");
        pvec(r.direction);
        std::printf(", \"next\": ");
        pd(next);
        std::printf("}");
    }
    std::printf("]");
}

void dump_rng(out_t& o)
{
    o.key("rng");
    std::printf("[");
    unsigned const seeds[] = { 0u, 1u, 5489u, 123456789u, 0xDEADBEEFu, 7u * 343u };
    bool first = true;
    for(unsigned const seed : seeds) {
        auto rng = seeded(seed);
        std::printf("%s{\"seed\": %u, \"generate\": [", first ? "" : ",\n ", seed);
        first = false;
        for(int i = 0; i < 700; ++i) {  // > 624 words: crosses an mt19937 twist
            std::printf("%s", i ? ", " : "");
            pd(rng.generate());
        }
        std::printf("], \"between\": [");
        for(int i = 0; i < 16; ++i) {
            std::printf("%s", i ? ", " : "");
            pd(rng.generate_between(-1.0, 1.0));
        }
        std::printf("]}");
    }
    std::printf("]");
}

void dump_utils(out_t& o)
{
    o.key("utils");
    double const xs[] = { -1.0, -0.0, 0.0, 1e-9, 0.001, 0.0031308, 0.1, 0.25, 0.5, 0.73, 0.999, 1.0, 1.5, 42.0 };
    std::printf("[");
    for(std::size_t i = 0; i < sizeof(xs) / sizeof(xs[0]); ++i) {
        std::printf("%s{\"x\": ", i ? ", " : "");
        pd(xs[i]);
        std::printf(", \"clamp\": ");
        pd(pt::clamp(xs[i]));
        std::printf(", \"color_to_int\": %d}", pt::color_to_int(xs[i]));
    }
    std::printf("]");
}

}  // namespace

auto main(int argc, char** argv) -> int
{
    bool const with_common = argc > 1 && std::strcmp(argv[1], "--common") == 0;
    out_t o;
    std::printf("{");
    o.key("scene_name");
    std::printf("\"%s\"", SCENE_NAME);
#ifdef SIMPLE
    dump_scene(o, 400, 300, "400x300");
    dump_intersections(o, 400, 300);
    dump_camera_rays(o, 400, 300);
#else
    dump_scene(o, 1024, 768, "1024x768");
    dump_scene(o, 1920, 1080, "1920x1080");
    dump_scene(o, 3840, 2160, "3840x2160");
    dump_intersections(o, 1024, 768);
    dump_camera_rays(o, 1024, 768);
#endif
    if(with_common) {
        dump_rng(o);
        dump_utils(o);
        o.key("sizeof");
        std::printf("{\"sphere\": %zu, \"camera\": %zu, \"camera_config\": %zu, \"vec3\": %zu}",
                    sizeof(pt::sphere), sizeof(pt::camera), sizeof(pt::camera_config), sizeof(pt::vec3));
    }
    std::printf("}\n");
    return 0;
}
