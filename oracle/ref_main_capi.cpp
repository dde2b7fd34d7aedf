// ref_main_capi.cpp -- TEST INFRASTRUCTURE ONLY (the reference's own path
// functions, callable from the tests' generators and bench.py's cpu_baseline).
//
// oracle/Makefile compiles ONE translation unit made of
//   (1) ref_main_prelude.hpp (force-included: main.cpp:1-21's includes minus
//       fmt/taskflow, which only main() uses),
//   (2) /root/reference/src/main.cpp lines 27-197 VERBATIM, streamed from the
//       reference's file by `sed` into the compiler (no copy is written
//       anywhere): intersect :30-42, diffuse_ray :44-58, specular_ray :60-67,
//       dielectric_ray :69-97, radiance :104-158, render_state :160-170,
//       render_subpixel :179-197,
//   (3) this file,
// and links the reference's `pt` library (_ref/libpt_ref.a, its own sources).
// The result, _ref/libref_main.so, is the reference's per-pixel hot path as the
// reference compiles it: double arithmetic, std::mt19937 +
// uniform_real_distribution draws (random_state.cpp:9-17), glibc libm.
//
// What this file adds is only plumbing around those functions:
//   * C entry points over plain arrays (pt::sphere / pt::camera layouts),
//   * deterministic seeding: pt::rand_state::default_with_seed multiplies by
//     std::random_device{}() (random_state.cpp:5), so every entry point takes
//     the mt19937 seed itself and aggregate-initialises pt::rand_state
//     (random_state.hpp:12-16, a C++17 aggregate),
//   * the row loop: main.cpp:217-234's task body (per-row rand_state, then
//     render_subpixel over x, sy, sx) run over rows by OpenMP
//     schedule(dynamic,1) instead of cpp-taskflow (absent here) -- the
//     north star's "OpenMP loop" -- with each row's seed supplied by the
//     caller (main.cpp:222-223 uses random_device() * (unsigned short)(y^3)),
//   * draw counting: a draw is two mt19937 outputs (generate_canonical<double,
//     53> from 32-bit words), counted by stepping a copy of the engine until it
//     equals the engine after the call.
#include <omp.h>

#include <cstdint>
#include <random>

#define REF_API extern "C" __attribute__((visibility("default")))

namespace {

struct ref_sphere {  // pt::sphere (sphere.hpp:10-17), 88 bytes
    double radius;
    double position[3];
    double emission[3];
    double color[3];
    int32_t material;
    int32_t pad_;
};
static_assert(sizeof(ref_sphere) == sizeof(pt::sphere), "pt::sphere layout");

auto v3(const double *p) -> pt::vec3 { return pt::vec3{ p[0], p[1], p[2] }; }
void put(const pt::vec3 &v, double *p)
{
    p[0] = v.x;
    p[1] = v.y;
    p[2] = v.z;
}

auto make_scene(const ref_sphere *s, int n) -> pt::scene
{
    pt::scene scn{};
    scn.spheres.reserve(static_cast<std::size_t>(n));
    for(int i = 0; i < n; ++i)
        scn.spheres.push_back(pt::sphere{ s[i].radius, v3(s[i].position), v3(s[i].emission), v3(s[i].color),
                                          static_cast<pt::reflection_type>(s[i].material) });
    return scn;
}

// pt::camera (camera.hpp:23-33): 7 vec3 + lens_radius, as with_config returns it
auto make_camera(const double *c) -> pt::camera
{
    return pt::camera{ v3(c), v3(c + 3), v3(c + 6), v3(c + 9), v3(c + 12), v3(c + 15), v3(c + 18), c[21] };
}

auto seeded(uint32_t seed) -> pt::rand_state
{
    return pt::rand_state{ std::mt19937{ seed }, std::uniform_real_distribution<double>{ 0.0, 1.0 } };
}

auto draws_between(std::mt19937 from, std::mt19937 const &to) -> int
{
    int k = 0;
    while(!(from == to)) {
        from();
        from();
        if(++k > 1 << 20)
            return -1;
    }
    return k;
}

}  // namespace

REF_API int ref_abi_version(void) { return 1; }

// intersect(scene, ray, t, id) main.cpp:30-42; returns the hit flag
REF_API int ref_intersect_scene(const ref_sphere *s, int n, const double o[3], const double d[3], double *t,
                                int64_t *id)
{
    auto const scn = make_scene(s, n);
    std::size_t i = 0;
    bool const hit = intersect(scn, pt::ray{ v3(o), v3(d) }, *t, i);
    *id = hit ? static_cast<int64_t>(i) : -1;
    return hit ? 1 : 0;
}

// One BRDF sampler (kind 0 diffuse_ray main.cpp:44-58, 1 specular_ray :60-67,
// 2 dielectric_ray :69-97) on the hit record get_hit_record_at(sphere, ray, t)
// (hit_record.cpp:3-12), with rand_state{mt19937{seed}}.  Returns the draws
// consumed; *next = the draw after them.
REF_API int ref_brdf(int kind, const ref_sphere *sp, const double o[3], const double d[3], double t, uint32_t seed,
                     double ro[3], double rd[3], double *next)
{
    auto const one = make_scene(sp, 1);
    auto const rec = pt::get_hit_record_at(one.spheres[0], pt::ray{ v3(o), v3(d) }, t);
    auto rng = seeded(seed);
    auto const start = rng.rng;
    pt::ray out{ pt::vec3{ 0, 0, 0 }, pt::vec3{ 0, 0, 0 } };
    switch(kind) {
    case 0: out = diffuse_ray(rec, rng); break;
    case 1: out = specular_ray(rec, rng); break;
    case 2: out = dielectric_ray(rec, rng); break;
    default: return -1;
    }
    put(out.origin, ro);
    put(out.direction, rd);
    int const draws = draws_between(start, rng.rng);
    *next = rng.generate();
    return draws;
}

// `count` seeded camera paths: path k uses rand_state{mt19937{seed0 + k}}:
// s = generate(), t = generate(), ray = cam.get_ray(s, t, rng)
// (camera.cpp:32-38), c = radiance(scene, ray, rng) (main.cpp:104-158).
// Per path: ray[6] = origin, direction; value[3] = c; draws = draws radiance
// consumed (after get_ray's); next = the draw after radiance.
REF_API int ref_paths(const ref_sphere *s, int n, const double *cam, uint32_t seed0, int count, int nthreads,
                      double *ray, double *value, int32_t *draws, double *next)
{
    auto const scn = make_scene(s, n);
    auto const cm = make_camera(cam);
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads > 0 ? nthreads : 1)
    for(int k = 0; k < count; ++k) {
        auto rng = seeded(seed0 + static_cast<uint32_t>(k));
        double const u = rng.generate();
        double const v = rng.generate();
        pt::ray const r = cm.get_ray(u, v, rng);
        auto const mark = rng.rng;
        pt::vec3 const c = radiance(scn, r, rng);
        put(r.origin, ray + 6 * k);
        put(r.direction, ray + 6 * k + 3);
        put(c, value + 3 * k);
        draws[k] = draws_between(mark, rng.rng);
        next[k] = rng.generate();
    }
    return 0;
}

// The reference row loop (main.cpp:217-234's task body) over rows y0, y0 +
// ystep, ... < y1, OpenMP schedule(dynamic,1) on nthreads threads: row y gets
// rand_state{mt19937{row_seed[y]}} and render_state{scene, cam, rng, image, W,
// H, samps, nsub}, then render_subpixel(x, y, sx, sy) for x < W, sy, sx < nsub
// (main.cpp:226-232).  image: W*H*3 doubles in the reference's row order
// (main.cpp:181), ADDED into as render_subpixel does (main.cpp:196).
REF_API int ref_render_rows(const ref_sphere *s, int n, const double *cam, int W, int H, int samps, int nsub,
                            const uint32_t *row_seed, int y0, int y1, int ystep, int nthreads, double *image)
{
    if(W <= 0 || H <= 0 || samps < 0 || nsub < 1 || ystep < 1 || y0 < 0 || y1 > H)
        return -1;
    auto const scn = make_scene(s, n);
    auto const cm = make_camera(cam);
    std::vector<pt::vec3> img;
    img.reserve(static_cast<std::size_t>(W) * H);
    for(std::size_t i = 0; i < static_cast<std::size_t>(W) * H; ++i)
        img.push_back(v3(image + 3 * i));
    int const rows = y0 < y1 ? (y1 - y0 + ystep - 1) / ystep : 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
    for(int j = 0; j < rows; ++j) {
        int const y = y0 + j * ystep;
        auto rng = seeded(row_seed[y]);
        render_state state{ scn, cm, rng, img, W, H, samps, nsub };
        for(int x = 0; x < W; x++)
            for(int sy = 0; sy < nsub; sy++)
                for(int sx = 0; sx < nsub; sx++)
                    render_subpixel(x, y, sx, sy, state);
    }
    for(std::size_t i = 0; i < img.size(); ++i)
        put(img[i], image + 3 * i);
    return 0;
}
