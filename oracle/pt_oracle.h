/*
 * pt_oracle.h -- TEST INFRASTRUCTURE ONLY (the parity oracle).
 *
 * A plain-C CPU restatement of AlexandruIca/cpu-path-tracing's per-pixel hot
 * path (src/main.cpp:30-197 and the `pt` library sources in src/).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline -- never as the
 * product path.  The product is the HIP megakernel in
 * cpu-path-tracing_amd/csrc behind include/ptgpu.h.
 *
 * Three arithmetic modes share one algorithm:
 *   Mode A / mt : double, std::mt19937 + generate_canonical<double,53> draws,
 *                 libm sin/cos/pow -- the reference's arithmetic exactly.
 *                 Pinned bit-exactly at the `pt` library level against
 *                 golden vectors produced by oracle/ref_golden.cpp compiled
 *                 against /root/reference/src (tests/golden/).
 *   Mode A / xs : double, reference arithmetic, counter-based xorshift32 draws
 *                 keyed by (seed, pixel, sub-pixel, sample) instead of a
 *                 per-row mt19937 (the RNG swap the north star asks for).
 *   Mode B / xs : float, the op sequence the GPU kernel executes in its
 *                 exact arithmetic mode (PTG_FLAG_EXACT_MATH: explicit fmaf,
 *                 deterministic div/sqrt/rsqrt sequences, table sin/cos,
 *                 anchored quadratic for huge spheres).  The exact-mode GPU
 *                 image must equal it bit for bit; the default mode (the
 *                 GPU's v_sqrt/v_rsq/v_rcp/v_sin/v_cos) is held to the
 *                 RMSE bar against Mode A/xs instead.
 *
 * Parity status: L0 (vec/ray/sphere/hit_record/camera/random_state/utils) is
 * pinned against the compiled reference; main.cpp (radiance, BRDFs,
 * render_subpixel) cannot be compiled here (it needs cpp-taskflow 2.4.0,
 * absent from the image), so those functions are restated from the source
 * text and pinned only through the L0 vectors they are built from.
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same memory layout as pt::sphere (sphere.hpp:10-17): 88 bytes. */
typedef struct {
    double radius;
    double position[3];
    double emission[3];
    double color[3];
    int32_t material; /* reflection.hpp:7-12: 0 diffuse, 1 specular, 2 dielectric */
    int32_t pad_;
} po_sphere;

/* Same layout as pt::camera_config (camera.hpp:11-21): 112 bytes. */
typedef struct {
    double position[3];
    double direction[3];
    double up[3];
    double aspect_ratio;
    double vertical_fov_radians;
    double focal_length;
    double aperture;
    double focus_distance;
} po_camera_config;

/* Same layout as pt::camera (camera.hpp:23-33): 176 bytes. */
typedef struct {
    double position[3];
    double lower_left_corner[3];
    double cam_x_axis[3];
    double cam_y_axis[3];
    double u[3];
    double v[3];
    double w[3];
    double lens_radius;
} po_camera;

/* std::mt19937 state (libstdc++ layout-independent restatement). */
typedef struct {
    uint32_t mt[624];
    int32_t idx;
} po_mt19937;

/* ---- L0: the `pt` library ------------------------------------------------ */
void po_mt_seed(po_mt19937 *g, uint32_t seed);
uint32_t po_mt_next(po_mt19937 *g);
double po_mt_generate(po_mt19937 *g);                             /* random_state.cpp:9-12 */
double po_mt_generate_between(po_mt19937 *g, double lo, double hi); /* random_state.cpp:14-17 */

void po_camera_with_config(const po_camera_config *cfg, po_camera *out); /* camera.cpp:3-17 */
/* camera.cpp:32-38; returns the number of draws consumed */
int po_camera_get_ray_mt(const po_camera *cam, double s, double t, po_mt19937 *g,
                         double origin[3], double direction[3]);
double po_sphere_intersect(const po_sphere *sp, const double origin[3], const double direction[3]); /* sphere.cpp:6-30 */
/* hit_record.cpp:3-12: out = hit_point[3], outward_normal[3], normal[3], front_facing */
void po_hit_record(const po_sphere *sp, const double origin[3], const double direction[3], double t,
                   double out[10]);
double po_clamp(double x);     /* utils.cpp:6-9 */
int po_color_to_int(double x); /* utils.cpp:11-16 */
double po_vec_length(const double v[3]); /* vec.cpp:66-69 */

/* ---- scenes (simple_scene.hpp:14-52, box_scene.hpp:14-72, box_mirror_scene.hpp:14-72) */
/* id: 0 simple, 1 box, 2 box_mirror.  Returns sphere count (<= cap). */
int po_scene(int id, int w, int h, po_sphere *out, int cap, po_camera_config *cfg);
/* Synthetic N-sphere scene (BASELINE configs[4]); generator defined in DESIGN.md. */
int po_scene_synthetic(int n, int w, int h, uint32_t gen_seed, po_sphere *out, po_camera_config *cfg);

/* ---- L1: path tracer (main.cpp:30-158), Mode A / mt ------------------------ */
int po_intersect_scene(const po_sphere *s, int n, const double o[3], const double d[3], double *t, int *id);
/* BRDF samplers main.cpp:44-97.  rec = 10 doubles from po_hit_record plus the
 * original ray (o,d).  Return draws consumed. */
int po_diffuse_ray_mt(const double rec[10], const double o[3], const double d[3], po_mt19937 *g,
                      double ro[3], double rd[3]);
int po_specular_ray_mt(const double rec[10], const double o[3], const double d[3], po_mt19937 *g,
                       double ro[3], double rd[3]);
int po_dielectric_ray_mt(const double rec[10], const double o[3], const double d[3], po_mt19937 *g,
                         double ro[3], double rd[3]);
/* radiance main.cpp:104-158; returns the number of segments (scene scans) */
int po_radiance_mt(const po_sphere *s, int n, const double o[3], const double d[3], po_mt19937 *g,
                   double out[3]);

/* ---- L2/L3: whole-image renders ------------------------------------------ */
/* Reference row loop (main.cpp:214-236) with the reference's per-row seeding
 * mt19937(rd_value * (unsigned short)(y*y*y)) where rd_value stands in for
 * std::random_device{}() (random_state.cpp:5).  Renders rows y in
 * [y0, y1) with step ystep using nthreads OpenMP threads (schedule dynamic,1).
 * image: W*H*3 doubles, reference row order (main.cpp:181), accumulated into. */
int po_render_mt(const po_sphere *s, int n, const po_camera *cam, int W, int H, int samps, int nsub,
                 uint32_t rd_value, int y0, int y1, int ystep, int nthreads, double *image);

/* Counter RNG (DESIGN.md "RNG"): key (seed, pixel=y*W+x, sub=sy*nsub+sx, sample). */
uint64_t po_key_hash(uint64_t seed, uint64_t pixel_sub);
uint32_t po_sample_state(uint64_t key, uint32_t sample);
uint32_t po_xorshift32(uint32_t *state);

/* Mode A / xs: double arithmetic, counter xorshift draws. */
int po_render_xs_f64(const po_sphere *s, int n, const po_camera *cam, int W, int H, int samps, int nsub,
                     uint64_t seed, int y0, int y1, int ystep, int nthreads, double *image,
                     uint64_t *segments);
/* Mode B / xs: float arithmetic (GPU op sequence).  image: W*H*3 floats,
 * reference row order, overwritten for the rows rendered. */
int po_render_xs_f32(const po_sphere *s, int n, const po_camera *cam, int W, int H, int samps, int nsub,
                     uint64_t seed, int y0, int y1, int ystep, int nthreads, float *image,
                     uint64_t *segments);
/* ... and *out_of_range = paths with a radiance component outside [0, 2^30]
 * (NaN, negative, huge: clipped by the exact accumulation; the kernel's
 * PTG_FLAG_COUNT_NONFINITE counter) */
int po_render_xs_f32_ex(const po_sphere *s, int n, const po_camera *cam, int W, int H, int samps, int nsub,
                        uint64_t seed, int y0, int y1, int ystep, int nthreads, float *image, uint64_t *segments,
                        uint64_t *out_of_range);
/* The same for the pixels x in [x0, x1) of rows y0, y0 + ystep, ... < y1,
 * parallel over pixels (for single rows at large sample counts). */
int po_render_xs_f64_rect(const po_sphere *s, int n, const po_camera *cam, int W, int H, int samps, int nsub,
                          uint64_t seed, int x0, int x1, int y0, int y1, int ystep, int nthreads, double *image,
                          uint64_t *segments);
int po_render_xs_f32_rect(const po_sphere *s, int n, const po_camera *cam, int W, int H, int samps, int nsub,
                          uint64_t seed, int x0, int x1, int y0, int y1, int ystep, int nthreads, float *image,
                          uint64_t *segments);
/* One Mode-B path for a given (pixel, sub, sample): returns radiance and
 * segment count -- used by the per-sample GPU parity test. */
/* Mode B arithmetic primitives: quot[i] = div_B(a[i], b[i]) (b > 0),
 * root[i] = sqrt_B(a[i]) */
void po_mode_b_math(const float *a, const float *b, size_t n, float *quot, float *root);
/* the scan's square root (sqrt_scan_B) and the normalising rsqrt (rsqrt_B) of a[i] > 0 */
void po_mode_b_roots(const float *a, size_t n, float *sq_scan, float *rsq);
/* Mode B' (error decomposition): flags swap Mode B's approximations for
 * accurate fp32 operations (pt_oracle.c PO_BV_*); 0 = Mode B */
void po_set_mode_b_variant(int flags);
int po_get_mode_b_variant(void);
/* Mode B cos/sin(2 pi m 2^-24) of 24-bit integers m (out: n {cos, sin} pairs) */
void po_sincos2pi(const uint32_t *m, size_t n, float *out);
/* Mode B scene layout: anchor axis per sphere (-1: camera-facing anchor or not
 * huge) and the linear scan order (order[j] = sphere visited j-th) */
int po_scan_layout(const po_sphere *s, int n, const po_camera *cam, int32_t *axis, int32_t *order);
int po_sample_f32(const po_sphere *s, int n, const po_camera *cam, int W, int H, int nsub, uint64_t seed,
                  int x, int y, int sx, int sy, uint32_t sample, float out[3]);

/* Output stage (main.cpp:240-247 + utils.cpp:11-16): gamma-2.2 8-bit values. */
void po_tonemap(const double *image, size_t count, int32_t *out);

#ifdef __cplusplus
}
#endif
#endif
