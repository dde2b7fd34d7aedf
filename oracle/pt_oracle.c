/*
 * pt_oracle.c -- TEST INFRASTRUCTURE ONLY: the CPU parity oracle and the
 * timed CPU baseline ("port", the repo's own OpenMP loop).  See pt_oracle.h
 * for the modes and the pinning status.  Never linked into the product.
 *
 * Every function cites the reference file:line it restates
 * (AlexandruIca/cpu-path-tracing, /root/reference/src).  Build flags:
 * -ffp-contract=off so that double arithmetic is evaluated exactly as the
 * reference's out-of-line vec3 operators evaluate it (vec.cpp:15-69), and so
 * that Mode B's float sequence only fuses where fmaf() is written.
 */
#include "pt_oracle.h"

#include <math.h>
#include <string.h>
#include <stdlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define PO_EPS 1e-4      /* constants.hpp:7 */
#define PO_PI 3.14159265358979323846 /* constants.hpp:8 */
#define PO_INF 1e20      /* constants.hpp:9 */
#define PO_DEPTH_LIMIT 100 /* constants.hpp:10 */
#define PO_RR_THRESHOLD 4  /* main.cpp:106 */

/* ========================================================================= */
/* std::mt19937 (libstdc++ bits/random.tcc) + generate_canonical<double,53>   */
/* ========================================================================= */
void po_mt_seed(po_mt19937 *g, uint32_t seed)
{
    g->mt[0] = seed;
    for (int i = 1; i < 624; ++i) {
        uint32_t x = g->mt[i - 1];
        g->mt[i] = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i;
    }
    g->idx = 624;
}

static void po_mt_twist(po_mt19937 *g)
{
    const uint32_t upper = 0x80000000u, lower = 0x7fffffffu;
    for (int k = 0; k < 624; ++k) {
        uint32_t y = (g->mt[k] & upper) | (g->mt[(k + 1) % 624] & lower);
        g->mt[k] = g->mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    g->idx = 0;
}

uint32_t po_mt_next(po_mt19937 *g)
{
    if (g->idx >= 624)
        po_mt_twist(g);
    uint32_t z = g->mt[g->idx++];
    z ^= (z >> 11) & 0xffffffffu;
    z ^= (z << 7) & 0x9d2c5680u;
    z ^= (z << 15) & 0xefc60000u;
    z ^= (z >> 18);
    return z;
}

/* random_state.cpp:9-12 -> uniform_real_distribution<double>{0,1}(mt19937):
 * generate_canonical<double,53> (random.tcc:3348-3380) draws two 32-bit words:
 * (g0 + g1*2^32) / 2^64, clamped below 1; then *(1-0)+0. */
double po_mt_generate(po_mt19937 *g)
{
    double sum = 0.0, tmp = 1.0;
    for (int k = 0; k < 2; ++k) {
        sum += (double)po_mt_next(g) * tmp;
        tmp *= 4294967296.0;
    }
    double ret = sum / tmp;
    if (ret >= 1.0)
        ret = nextafter(1.0, 0.0);
    return ret * (1.0 - 0.0) + 0.0;
}

/* random_state.cpp:14-17 */
double po_mt_generate_between(po_mt19937 *g, double lo, double hi)
{
    return lo + (hi - lo) * po_mt_generate(g);
}

/* ========================================================================= */
/* Counter-based xorshift (replaces pt::rand_state on the hot path)           */
/* ========================================================================= */
static uint64_t po_mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* key = mix64(seed ^ mix64(pixel_sub + 1)), pixel_sub = (y*W + x)*nsub^2 + sub */
uint64_t po_key_hash(uint64_t seed, uint64_t pixel_sub)
{
    return po_mix64(seed ^ po_mix64(pixel_sub + 1ull));
}

/* per-sample xorshift32 state: high word of mix64(key + (s+1)*golden), never 0 */
uint32_t po_sample_state(uint64_t key, uint32_t sample)
{
    uint32_t st = (uint32_t)(po_mix64(key + ((uint64_t)sample + 1ull) * 0x9E3779B97F4A7C15ull) >> 32);
    return st ? st : 0x6D2B79F5u;
}

uint32_t po_xorshift32(uint32_t *state)
{
    uint32_t x = *state;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    *state = x;
    return x;
}

/* one U[0,1) draw: top 24 bits, exact in float and in double */
static float po_xs_f32(uint32_t *st) { return (float)(po_xorshift32(st) >> 8) * 0x1p-24f; }
static double po_xs_f64(uint32_t *st) { return (double)(po_xorshift32(st) >> 8) * 0x1p-24; }

/* ========================================================================= */
/* Mode A: double vec3 with the reference's evaluation order (vec.cpp)        */
/* ========================================================================= */
typedef struct { double x, y, z; } v3;
static v3 mk(double x, double y, double z) { v3 r = {x, y, z}; return r; }
static v3 vadd(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }  /* vec.cpp:15-18 */
static v3 vsub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }  /* vec.cpp:20-23 */
static v3 vmul(v3 a, double b) { return mk(a.x * b, a.y * b, a.z * b); }    /* vec.cpp:25-28 */
static v3 vblend(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); } /* vec.cpp:30-33 */
static double vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* vec.cpp:40-43 */
static v3 vnorm(v3 a) { return vmul(a, 1 / sqrt(a.x * a.x + a.y * a.y + a.z * a.z)); } /* vec.cpp:35-38 */
static v3 vcross(v3 a, v3 b)                                                   /* vec.cpp:45-48 */
{
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static v3 ld3(const double *p) { return mk(p[0], p[1], p[2]); }
static void st3(double *p, v3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }

/* vec.cpp:66-69 -> std::hypot(x,y,z) as libstdc++-11 __hypot3 implements it */
double po_vec_length(const double v[3])
{
    double x = fabs(v[0]), y = fabs(v[1]), z = fabs(v[2]);
    double a = x < y ? (y < z ? z : y) : (x < z ? z : x);
    if (a != 0.0)
        return a * sqrt((x / a) * (x / a) + (y / a) * (y / a) + (z / a) * (z / a));
    return 0.0;
}

/* utils.cpp:6-9 (std::clamp(x, 0, 1)) */
double po_clamp(double x) { return x < 0.0 ? 0.0 : (1.0 < x ? 1.0 : x); }

/* utils.cpp:11-16 */
int po_color_to_int(double x) { return (int)round(pow(po_clamp(x), 1.0 / 2.2) * 255.0); }

void po_tonemap(const double *image, size_t count, int32_t *out)
{
    for (size_t i = 0; i < count; ++i)
        out[i] = po_color_to_int(image[i]);
}

/* camera.cpp:3-17 */
void po_camera_with_config(const po_camera_config *cfg, po_camera *out)
{
    double vh = 2.0 * tan(0.5 * cfg->vertical_fov_radians);
    double vw = cfg->aspect_ratio * vh;
    v3 pos = ld3(cfg->position);
    v3 w = vnorm(vsub(pos, ld3(cfg->direction)));
    v3 u = vnorm(vcross(ld3(cfg->up), w));
    v3 v = vcross(w, u);
    v3 X = vmul(vmul(u, vw), cfg->focus_distance);
    v3 Y = vmul(vmul(v, vh), cfg->focus_distance);
    v3 llc = vsub(vsub(vsub(pos, vmul(X, 0.5)), vmul(Y, 0.5)), vmul(w, cfg->focus_distance));
    st3(out->position, pos);
    st3(out->lower_left_corner, llc);
    st3(out->cam_x_axis, X);
    st3(out->cam_y_axis, Y);
    st3(out->u, u);
    st3(out->v, v);
    st3(out->w, w);
    out->lens_radius = cfg->aperture / 2.0;
}

/* A generic draw source for Mode A: the reference's mt19937 or the counter RNG */
typedef struct {
    po_mt19937 *mt;
    uint32_t xs;
    int draws;
} rngA;

static double drawA(rngA *r)
{
    r->draws++;
    return r->mt ? po_mt_generate(r->mt) : po_xs_f64(&r->xs);
}
static double drawA_between(rngA *r, double lo, double hi) { return lo + (hi - lo) * drawA(r); }

/* camera.cpp:19-30 + camera.cpp:32-38 */
static void cam_get_ray_A(const po_camera *cam, double s, double t, rngA *r, v3 *ro, v3 *rd)
{
    v3 p;
    for (;;) {
        double px = drawA_between(r, -1.0, 1.0);
        double py = drawA_between(r, -1.0, 1.0);
        p = mk(px, py, 0.0);
        if (vdot(p, p) >= 1.0)
            continue;
        break;
    }
    v3 rdisk = vmul(p, cam->lens_radius);
    v3 off = vadd(vmul(rdisk, s), vmul(rdisk, t)); /* camera.cpp:35 quirk: rd*s + rd*t */
    v3 dir = vsub(vsub(vadd(vadd(ld3(cam->lower_left_corner), vmul(ld3(cam->cam_x_axis), s)),
                            vmul(ld3(cam->cam_y_axis), t)),
                       ld3(cam->position)),
                  off);
    *ro = vadd(ld3(cam->position), off);
    *rd = dir;
}

int po_camera_get_ray_mt(const po_camera *cam, double s, double t, po_mt19937 *g, double origin[3],
                         double direction[3])
{
    rngA r = {g, 0, 0};
    v3 o, d;
    cam_get_ray_A(cam, s, t, &r, &o, &d);
    st3(origin, o);
    st3(direction, d);
    return r.draws;
}

/* sphere.cpp:6-30 */
static double sphere_intersect_A(const po_sphere *sp, v3 o, v3 d)
{
    v3 oc = vsub(o, ld3(sp->position));
    double a = vdot(d, d);
    double hb = vdot(oc, d);
    double c = vdot(oc, oc) - sp->radius * sp->radius;
    double disc = hb * hb - a * c;
    if (disc < 0)
        return 0.0;
    double sq = sqrt(disc);
    double root = (-hb - sq) / a;
    if (root < PO_EPS) {
        root = (-hb + sq) / a;
        if (root < PO_EPS)
            return 0.0;
    }
    return root;
}

double po_sphere_intersect(const po_sphere *sp, const double origin[3], const double direction[3])
{
    return sphere_intersect_A(sp, ld3(origin), ld3(direction));
}

/* main.cpp:30-42 (strict < keeps the lowest index on ties) */
static int intersect_A(const po_sphere *s, int n, v3 o, v3 d, double *t, int *id)
{
    *t = PO_INF;
    for (int i = 0; i < n; ++i) {
        double dd = sphere_intersect_A(&s[i], o, d);
        if (dd > 0 && dd < *t) {
            *t = dd;
            *id = i;
        }
    }
    return *t < PO_INF;
}

int po_intersect_scene(const po_sphere *s, int n, const double o[3], const double d[3], double *t, int *id)
{
    *id = -1;
    return intersect_A(s, n, ld3(o), ld3(d), t, id);
}

/* hit_record.cpp:3-12 */
typedef struct {
    v3 o, d;   /* original ray */
    v3 p, on, n;
    int front;
} recA;

static recA hit_record_A(const po_sphere *sp, v3 o, v3 d, double t)
{
    recA r;
    r.o = o;
    r.d = d;
    r.p = vadd(o, vmul(d, t)); /* ray.cpp:3-6 */
    r.on = vnorm(vsub(r.p, ld3(sp->position)));
    r.front = vdot(r.on, d) < 0;
    r.n = r.front ? r.on : vmul(r.on, -1);
    return r;
}

void po_hit_record(const po_sphere *sp, const double origin[3], const double direction[3], double t,
                   double out[10])
{
    recA r = hit_record_A(sp, ld3(origin), ld3(direction), t);
    st3(out, r.p);
    st3(out + 3, r.on);
    st3(out + 6, r.n);
    out[9] = r.front;
}

static recA rec_from(const double rec[10], const double o[3], const double d[3])
{
    recA r;
    r.o = ld3(o);
    r.d = ld3(d);
    r.p = ld3(rec);
    r.on = ld3(rec + 3);
    r.n = ld3(rec + 6);
    r.front = rec[9] != 0.0;
    return r;
}

/* main.cpp:44-58 */
static void diffuse_A(const recA *rec, rngA *r, v3 *ro, v3 *rd)
{
    double phi = 2 * PO_PI * drawA(r);
    double ra = drawA(r);
    double st = sqrt(ra);
    double ct = sqrt(1.0 - ra);
    v3 w = rec->n;
    v3 u = vnorm(vcross(fabs(w.x) > 0.1 ? mk(0, 1, 0) : mk(1, 0, 0), w));
    v3 v = vcross(w, u);
    v3 nd = vnorm(vadd(vadd(vmul(vmul(u, cos(phi)), st), vmul(vmul(v, sin(phi)), st)), vmul(w, ct)));
    *ro = rec->p;
    *rd = nd;
}

/* main.cpp:60-67 */
static void specular_A(const recA *rec, rngA *r, v3 *ro, v3 *rd)
{
    const double fuzziness = 0.0;
    v3 refl = vsub(rec->d, vmul(vmul(rec->on, 2.0), vdot(rec->on, rec->d)));
    double f = drawA(r) * fuzziness;
    *ro = rec->p;
    *rd = vadd(refl, mk(f, f, f));
}

/* main.cpp:82-87 */
static double reflectance_A(double cosine, double ref_idx)
{
    double r0 = (1.0 - ref_idx) / (1.0 + ref_idx);
    r0 *= r0;
    return r0 + (1.0 - r0) * pow(1.0 - cosine, 5);
}

/* main.cpp:69-97 */
static void dielectric_A(const recA *rec, rngA *r, v3 *ro, v3 *rd)
{
    const double refraction_index = 2.0;
    double ratio = rec->front ? (1.0 / refraction_index) : refraction_index;
    v3 ud = vnorm(rec->d);
    double x = vdot(vmul(ud, -1.0), rec->n);
    double ct = 1.0 < x ? 1.0 : x; /* std::min(x, 1.0) */
    double st = sqrt(1.0 - ct * ct);
    int cannot = ratio * st > 1.0;
    if (cannot || reflectance_A(ct, ratio) > drawA(r)) { /* short-circuit: no draw on TIR */
        specular_A(rec, r, ro, rd);
        return;
    }
    v3 perp = vmul(vadd(ud, vmul(rec->n, ct)), ratio);
    v3 par = vmul(rec->n, -sqrt(fabs(1.0 - vdot(perp, perp))));
    *ro = rec->p;
    *rd = vadd(perp, par);
}

#define BRDF_WRAPPER(name, fn)                                                                     \
    int name(const double rec[10], const double o[3], const double d[3], po_mt19937 *g, double ro[3], \
             double rd[3])                                                                         \
    {                                                                                              \
        rngA r = {g, 0, 0};                                                                        \
        recA h = rec_from(rec, o, d);                                                              \
        v3 a, b;                                                                                   \
        fn(&h, &r, &a, &b);                                                                        \
        st3(ro, a);                                                                                \
        st3(rd, b);                                                                                \
        return r.draws;                                                                            \
    }
BRDF_WRAPPER(po_diffuse_ray_mt, diffuse_A)
BRDF_WRAPPER(po_specular_ray_mt, specular_A)
BRDF_WRAPPER(po_dielectric_ray_mt, dielectric_A)

/* main.cpp:104-158; *segs = number of scene scans */
static v3 radiance_A(const po_sphere *s, int n, v3 o, v3 d, rngA *r, int *segs)
{
    v3 E = mk(0, 0, 0), T = mk(1, 1, 1);
    *segs = 0;
    for (int depth = 0; depth < PO_DEPTH_LIMIT; ++depth) {
        double t = 0.0;
        int id = 0;
        (*segs)++;
        if (!intersect_A(s, n, o, d, &t, &id)) {
            v3 ud = vnorm(d);
            double tt = 0.5 * (ud.y + 1.0);
            v3 bg = vadd(vmul(mk(1, 1, 1), 1.0 - tt), vmul(mk(0.5, 0.7, 1.0), tt));
            return vadd(E, vblend(T, bg));
        }
        const po_sphere *obj = &s[id];
        recA rec = hit_record_A(obj, o, d, t);
        v3 color = ld3(obj->color);
        E = vadd(E, vblend(T, ld3(obj->emission)));
        double p = color.x;
        if (p < color.y) p = color.y;
        if (p < color.z) p = color.z; /* std::max({x,y,z}) */
        if (depth > PO_RR_THRESHOLD) {
            if (drawA(r) < p)
                color = vmul(color, 1.0 / p);
            else
                return E;
        }
        T = vblend(T, color);
        switch (obj->material) {
        case 0: diffuse_A(&rec, r, &o, &d); break;
        case 1: specular_A(&rec, r, &o, &d); break;
        default: dielectric_A(&rec, r, &o, &d); break;
        }
    }
    return E;
}

int po_radiance_mt(const po_sphere *s, int n, const double o[3], const double d[3], po_mt19937 *g, double out[3])
{
    rngA r = {g, 0, 0};
    int segs = 0;
    v3 c = radiance_A(s, n, ld3(o), ld3(d), &r, &segs);
    st3(out, c);
    return segs;
}

/* main.cpp:179-197 for one sub-pixel; *r supplies the draws */
static v3 subpixel_A(const po_sphere *s, int n, const po_camera *cam, int W, int H, int samps, int nsub, int x,
                     int y, int sx, int sy, rngA *r, uint64_t key, uint64_t *segs)
{
    v3 acc = mk(0, 0, 0);
    for (int k = 0; k < samps; ++k) {
        if (!r->mt)
            r->xs = po_sample_state(key, (uint32_t)k);
        double sl = 1.0 / nsub;
        double xin = (x + sx * sl + drawA_between(r, 0.0, sl));
        double yin = (y + sy * sl + drawA_between(r, 0.0, sl));
        v3 o, d;
        cam_get_ray_A(cam, xin / W, yin / H, r, &o, &d);
        int sg = 0;
        v3 c = radiance_A(s, n, o, d, r, &sg);
        *segs += (uint64_t)sg;
        acc = vadd(acc, vmul(c, 1.0 / samps));
    }
    return acc;
}

static int check_args(int n, int W, int H, int samps, int nsub)
{
    return n < 0 || W <= 0 || H <= 0 || samps < 0 || nsub <= 0;
}

/* main.cpp:214-236 with the reference's row seeding (main.cpp:222-223) */
int po_render_mt(const po_sphere *s, int n, const po_camera *cam, int W, int H, int samps, int nsub,
                 uint32_t rd_value, int y0, int y1, int ystep, int nthreads, double *image)
{
    if (check_args(n, W, H, samps, nsub) || ystep <= 0)
        return -1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
    for (int y = y0; y < y1; y += ystep) {
        unsigned short seed = (unsigned short)(y * y * y);
        po_mt19937 g;
        po_mt_seed(&g, rd_value * (uint32_t)seed);
        rngA r = {&g, 0, 0};
        uint64_t segs = 0;
        for (int x = 0; x < W; ++x)
            for (int sy = 0; sy < nsub; ++sy)
                for (int sx = 0; sx < nsub; ++sx) {
                    v3 a = subpixel_A(s, n, cam, W, H, samps, nsub, x, y, sx, sy, &r, 0, &segs);
                    size_t row = (size_t)(H - y - 1) * (size_t)W + (size_t)x;
                    double *px = image + 3 * row;
                    double q = 1.0 / (nsub * nsub);
                    px[0] = px[0] + po_clamp(a.x) * q;
                    px[1] = px[1] + po_clamp(a.y) * q;
                    px[2] = px[2] + po_clamp(a.z) * q;
                }
    }
    return 0;
}

int po_render_xs_f64(const po_sphere *s, int n, const po_camera *cam, int W, int H, int samps, int nsub,
                     uint64_t seed, int y0, int y1, int ystep, int nthreads, double *image, uint64_t *segments)
{
    if (check_args(n, W, H, samps, nsub) || ystep <= 0)
        return -1;
    uint64_t total = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : total)
    for (int y = y0; y < y1; y += ystep) {
        for (int x = 0; x < W; ++x)
            for (int sy = 0; sy < nsub; ++sy)
                for (int sx = 0; sx < nsub; ++sx) {
                    uint64_t ps = ((uint64_t)y * (uint64_t)W + (uint64_t)x) * (uint64_t)(nsub * nsub) +
                                  (uint64_t)(sy * nsub + sx);
                    rngA r = {NULL, 0, 0};
                    uint64_t segs = 0;
                    v3 a = subpixel_A(s, n, cam, W, H, samps, nsub, x, y, sx, sy, &r, po_key_hash(seed, ps),
                                      &segs);
                    total += segs;
                    size_t row = (size_t)(H - y - 1) * (size_t)W + (size_t)x;
                    double *px = image + 3 * row;
                    double q = 1.0 / (nsub * nsub);
                    px[0] = px[0] + po_clamp(a.x) * q;
                    px[1] = px[1] + po_clamp(a.y) * q;
                    px[2] = px[2] + po_clamp(a.z) * q;
                }
    }
    if (segments)
        *segments = total;
    return 0;
}

/* ========================================================================= */
/* Mode B: the float op sequence of the GPU megakernel (DESIGN.md "Mode B")   */
/* ========================================================================= */
#define BIG_RADIUS 1000.0
#define TRIG_BITS 7 /* sin/cos table of 2^TRIG_BITS entries (sincos2pi_B) */
#define TRIG_ENTRIES (1 << TRIG_BITS)
#define LINEAR_MAX_PREP 64 /* = LINEAR_MAX: scenes scanned linearly on the GPU */
#define EPSF 1e-4f
#define INFF 1e20f

/* Mode B' (error decomposition, tests/test_error_budget.py): each flag swaps one
 * of Mode B's deliberate approximations for the accurate fp32 operation, so the
 * fp32-vs-fp64 difference can be split into "approximations" and "fp32 as
 * such".  0 = Mode B (the GPU's op sequence). */
#define PO_BV_IEEE_SQRT 1   /* sqrtf / 1.0f/sqrtf instead of the Newton/Goldschmidt sequences */
#define PO_BV_IEEE_DIV 2    /* n / d instead of the Newton reciprocal */
#define PO_BV_LIBM_TRIG 4   /* (float)cos/sin(2 pi u) in double instead of the table */
#define PO_BV_RENORM 8      /* normal = norm(p - C), diffuse direction re-normalised (main.cpp:55) */
#define PO_BV_FULL_SCAN 16  /* every sphere tested in index order (no wall pairs / box mode) */
#define PO_BV_LEX 32        /* every candidate divided, lowest index wins ties (main.cpp:35) */
#define PO_BV_DISC_NAIVE 64 /* small spheres' discriminant as hb^2 - a c (round 1) instead of a R^2 - |e x d|^2 */
/* small spheres' roots as (-hb -+ sqrt(disc)) / a (sphere.cpp:18-25's form) instead of c / q, q / a:
 * round 4 measured it (C3 box_mirror, 16 rows at 256 samples per sub-pixel, RMSE vs Mode A/xs
 * 5.0e-5 -> 4.5e-4, all of it from the near root -hb - sqrt(disc) -- its cancellation where a ray
 * meets a sphere close to its origin, e.g. in the crevice where the mirror and glass spheres touch
 * the floor); the fast kernel with these roots was 4 % faster and was not kept */
#define PO_BV_NAIVE_ROOTS 128
static int g_bvar = 0;
void po_set_mode_b_variant(int flags) { g_bvar = flags; }
int po_get_mode_b_variant(void) { return g_bvar; }
/* Anchored ("huge") form: R >= 1000, or R more than 16 times the camera's
 * distance to the surface (+1).  The kernel's host side: ptg_render.hip
 * is_huge. */
static int is_huge_B(const po_sphere *sp, const po_camera *cam)
{
    if (sp->radius >= BIG_RADIUS)
        return 1;
    double d2 = 0.0;
    for (int c = 0; c < 3; ++c)
        d2 += (cam->position[c] - sp->position[c]) * (cam->position[c] - sp->position[c]);
    return sp->radius > 16.0 * (fabs(sqrt(d2) - sp->radius) + 1.0);
}

typedef struct { float x, y, z; } f3;
static f3 fk(float x, float y, float z) { f3 r = {x, y, z}; return r; }
static float fcomp(f3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }
static float fdot(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
/* Deterministic reciprocal square root (DESIGN.md "fp32 math"): bit-trick seed
 * + two Newton steps written with explicit fmaf, so CPU and GPU agree bit for
 * bit; about 2 ulp, x > 0. */
static float rsqrt_B(float x)
{
    if (g_bvar & PO_BV_IEEE_SQRT)
        return 1.0f / sqrtf(x);
    uint32_t i;
    memcpy(&i, &x, 4);
    i = 0x5f375a86u - (i >> 1);
    float y;
    memcpy(&y, &i, 4);
    float h = 0.5f * x;
    for (int k = 0; k < 3; ++k) { /* three Newton steps: ~1.7 ulp (two left ~5e-6, 40 ulp) */
        float t = y * y;
        t = fmaf(-h, t, 1.5f);
        y = y * t;
    }
    return y;
}
/* Deterministic square root for x >= 0 (x = +0 gives 0): the rsqrt_B seed,
 * two coupled Goldschmidt steps on g ~ sqrt(x), h ~ 1/(2 sqrt(x)), then one
 * Newton residual step g + (x - g^2) h -- within 1 ulp (0.63 ulp measured;
 * the two steps alone leave ~5e-6, about 40 ulp, which was the largest
 * single part of the fp32-vs-fp64 image difference after the discriminant
 * form: DESIGN.md "error budget").  Kernel: pt_device.hpp sqrt_gs. */
static float sqrt_gs_B(float x)
{
    if (g_bvar & PO_BV_IEEE_SQRT)
        return sqrtf(x);
    uint32_t i;
    memcpy(&i, &x, 4);
    i = 0x5f375a86u - (i >> 1);
    float y;
    memcpy(&y, &i, 4);
    float g = x * y;
    float h = 0.5f * y;
    float r = fmaf(-g, h, 0.5f);
    g = fmaf(g, r, g);
    h = fmaf(h, r, h);
    r = fmaf(-g, h, 0.5f);
    g = fmaf(g, r, g);
    return fmaf(fmaf(-g, g, x), h, g);
}
/* the scan's square root (the discriminant): the same sequence */
static float sqrt_scan_B(float x) { return sqrt_gs_B(x); }
/* sqrt for any x: 0 for x <= 0 (clamped as an integer max, like the kernel) */
static float sqrt_B(float x)
{
    int32_t i;
    memcpy(&i, &x, 4);
    i = i > 0 ? i : 0;
    memcpy(&x, &i, 4);
    return sqrt_gs_B(x);
}
/* Deterministic n / d for d > 0: bit-trick reciprocal seed, two Newton steps,
 * one residual correction of the quotient.  Kernel: pt_device.hpp div_d. */
static float div_B(float n, float d)
{
    if (g_bvar & PO_BV_IEEE_DIV)
        return n / d;
    uint32_t i;
    memcpy(&i, &d, 4);
    i = 0x7EF311C3u - i;
    float r;
    memcpy(&r, &i, 4);
    r = fmaf(r, fmaf(-d, r, 1.0f), r);
    r = fmaf(r, fmaf(-d, r, 1.0f), r);
    float t = n * r;
    return fmaf(fmaf(-d, t, n), r, t);
}
static f3 fnorm(f3 a)
{
    float inv = rsqrt_B(fdot(a, a));
    return fk(a.x * inv, a.y * inv, a.z * inv);
}
static f3 fcross(f3 a, f3 b)
{
    return fk(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}

typedef struct {
    f3 P, N;          /* anchor point and anchor normal (big) or centre and 0 */
    float R, R2x, negR2, invR;
    int big;
    f3 C;             /* centre (float) for normals */
    f3 emis, col, col_rr;
    float prob;
    int mat;
    int axis;         /* huge sphere anchored on axis 0..2, else -1 (choose_anchor_B) */
    int visit;        /* linear scan: the sphere visited at scan position (this element's index) */
    int pair;         /* wall pair member (pair_walls_B): +1 the + wall, -1 the - wall, 0 none */
    float plo, phi;   /* on the + wall: the pair's origin bounds; box mode: a single wall's bound */
    int box;          /* box mode (box_mode_B), the same on every element */
} sphB;

typedef struct {
    f3 pos, base, X, Y; /* base = float(llc - pos) */
    float lens, invW, invH;
    float trig[2 * TRIG_ENTRIES]; /* sincos2pi_B table */
} camB;

/* Anchor of a huge sphere (DESIGN.md "Huge spheres"): P = C + R n0 on the
 * sphere, n0 its outward normal there.  Default n0: unit vector from C to the
 * camera.  If the point C + s R e_k of the dominant axis direction of that n0
 * lies within max(diagonal, 1) of the box around the camera and the non-huge
 * spheres, it is the anchor instead (both are exact anchors; the kernel then
 * reads e_k, d_k instead of two dot products).  Returns k, or -1.  Same
 * choice as the kernel's host side (ptg_render.hip: choose_anchor). */
typedef struct { double lo[3], hi[3], diag; } boxB;

static int choose_anchor_B(const po_sphere *sp, const po_camera *cam, const boxB *box, double P[3], double N[3])
{
    double R = sp->radius, v[3], len2 = 0.0;
    for (int c = 0; c < 3; ++c) {
        v[c] = cam->position[c] - sp->position[c];
        len2 += v[c] * v[c];
    }
    double len = sqrt(len2);
    for (int c = 0; c < 3; ++c)
        N[c] = len > 0.0 ? v[c] / len : (c == 1 ? 1.0 : 0.0);
    int k = 0;
    for (int c = 1; c < 3; ++c)
        if (fabs(N[c]) > fabs(N[k]))
            k = c;
    double sg = N[k] >= 0.0 ? 1.0 : -1.0, out2 = 0.0;
    for (int c = 0; c < 3; ++c) {
        double pa = sp->position[c] + (c == k ? sg * R : 0.0);
        double o = pa < box->lo[c] ? box->lo[c] - pa : (pa > box->hi[c] ? pa - box->hi[c] : 0.0);
        out2 += o * o;
    }
    int snap = sqrt(out2) <= (box->diag > 1.0 ? box->diag : 1.0);
    for (int c = 0; c < 3; ++c) {
        if (snap)
            N[c] = c == k ? sg : 0.0;
        P[c] = sp->position[c] + R * N[c];
    }
    return snap ? k : -1;
}

/* box around the camera and every non-huge sphere, and its diagonal */
static boxB scene_box_B(const po_sphere *s, int n, const po_camera *cam)
{
    boxB b;
    double d2 = 0.0;
    for (int c = 0; c < 3; ++c)
        b.lo[c] = b.hi[c] = cam->position[c];
    for (int i = 0; i < n; ++i) {
        if (is_huge_B(&s[i], cam))
            continue;
        for (int c = 0; c < 3; ++c) {
            double a = s[i].position[c] - s[i].radius, e = s[i].position[c] + s[i].radius;
            b.lo[c] = a < b.lo[c] ? a : b.lo[c];
            b.hi[c] = e > b.hi[c] ? e : b.hi[c];
        }
    }
    for (int c = 0; c < 3; ++c)
        d2 += (b.hi[c] - b.lo[c]) * (b.hi[c] - b.lo[c]);
    b.diag = sqrt(d2);
    return b;
}

static void trig_table_B(float *tab);

/* Wall pairs (DESIGN.md "wall pairs"; the kernel's host side:
 * ptg_render.hip pair_walls): on each axis k the first axis-anchored huge
 * sphere with its centre on the + side of its anchor (N = -e_k) and the first
 * on the - side.  A ray whose origin has pair_lo <= o_k <= pair_hi (the
 * tangent planes x_k = a_minus, a_plus widened by 1e-4 max(1, diagonal)) tests
 * only the wall it moves toward (d_k >= 0: the + wall): each sphere lies
 * entirely beyond its tangent plane. */
/* A wall may be paired / take part in box mode only if no ray origin can lie
 * genuinely inside it (the kernel's host side: ptg_render.hip wall_clear): not
 * dielectric, the camera on the room side by more than the margin. */
static int wall_clear_B(const po_sphere *s, int i, int k, int plus_side, const po_camera *cam, const boxB *box)
{
    if (s[i].material == 2)
        return 0;
    const double margin = 1e-4 * (box->diag > 1.0 ? box->diag : 1.0);
    const double a = plus_side ? s[i].position[k] - s[i].radius : s[i].position[k] + s[i].radius;
    return plus_side ? cam->position[k] < a - margin : cam->position[k] > a + margin;
}

static void pair_walls_B(const po_sphere *s, int n, const po_camera *cam, const boxB *box, sphB *out)
{
    const double margin = 1e-4 * (box->diag > 1.0 ? box->diag : 1.0);
    for (int k = 0; k < 3; ++k) {
        int plus = -1, minus = -1;
        for (int i = 0; i < n; ++i) {
            if (!out[i].big || out[i].axis != k)
                continue;
            const float nk = k == 0 ? out[i].N.x : (k == 1 ? out[i].N.y : out[i].N.z);
            if (nk < 0.0f && plus < 0)
                plus = i;
            if (nk > 0.0f && minus < 0)
                minus = i;
        }
        if (plus < 0 || minus < 0 || !wall_clear_B(s, plus, k, 1, cam, box) ||
            !wall_clear_B(s, minus, k, 0, cam, box))
            continue;
        out[plus].pair = 1;
        out[minus].pair = -1;
        out[plus].plo = (float)(s[minus].position[k] + s[minus].radius - margin);
        out[plus].phi = (float)(s[plus].position[k] - s[plus].radius + margin);
    }
}

/* Box mode (DESIGN.md "box mode"; the kernel's host side: ptg_render.hip
 * box_mode_of): every axis-anchored wall is one of its axis's pair or the
 * only wall of its axis, some axis has a pair, no other huge sphere.  A
 * single wall's room bound (margin as pair_walls_B) goes into its own
 * plo (- side wall) or phi (+ side wall). */
static void box_mode_B(const po_sphere *s, int n, const po_camera *cam, const boxB *box, sphB *out)
{
    int cnt[3] = {0, 0, 0}, pairs[3] = {0, 0, 0}, general = 0;
    for (int i = 0; i < n; ++i) {
        out[i].box = 0;
        if (!out[i].big)
            continue;
        if (out[i].axis < 0)
            ++general;
        else
            ++cnt[out[i].axis];
        if (out[i].pair == 1)
            pairs[out[i].axis] = 1;
    }
    int ok = general == 0 && (pairs[0] || pairs[1] || pairs[2]);
    for (int k = 0; k < 3; ++k)
        ok = ok && (pairs[k] ? cnt[k] == 2 : cnt[k] <= 1);
    for (int i = 0; i < n && ok; ++i) /* single walls too (the pairs' members are clear) */
        if (out[i].big && out[i].axis >= 0)
            ok = wall_clear_B(s, i, out[i].axis, fcomp(out[i].N, out[i].axis) < 0.0f, cam, box);
    if (!ok)
        return;
    const double margin = 1e-4 * (box->diag > 1.0 ? box->diag : 1.0);
    for (int i = 0; i < n; ++i) {
        out[i].box = 1;
        if (out[i].big && out[i].pair == 0) { /* single wall */
            const int k = out[i].axis;
            const float nk = k == 0 ? out[i].N.x : (k == 1 ? out[i].N.y : out[i].N.z);
            if (nk < 0.0f)
                out[i].phi = (float)(s[i].position[k] - s[i].radius + margin);
            else
                out[i].plo = (float)(s[i].position[k] + s[i].radius - margin);
        }
    }
}

/* sphB array + a compact copy of the lex scan's hot fields behind it: per
 * sphere {P, -R^2} (NaN for huge spheres: never rejected early), 16 B, so a
 * 10,000-sphere scan streams 160 KB instead of the whole records */
static sphB *malloc_sphB(int n)
{
    const size_t m = (size_t)(n > 0 ? n : 1);
    return (sphB *)malloc(sizeof(sphB) * m + 4 * sizeof(float) * m);
}
static float *hot_B(const sphB *s, int n) { return (float *)(s + (n > 0 ? n : 1)); }

static void prep_B(const po_sphere *s, int n, const po_camera *cam, sphB *out, camB *cb)
{
    boxB box = scene_box_B(s, n, cam);
    for (int i = 0; i < n; ++i) {
        const po_sphere *sp = &s[i];
        sphB *b = &out[i];
        double R = sp->radius;
        b->big = is_huge_B(sp, cam);
        b->R = (float)R;
        b->R2x = (float)(2.0 * R);
        b->negR2 = (float)(-(R * R));
        b->invR = (float)(1.0 / R);
        b->axis = -1;
        b->pair = 0;
        b->plo = b->phi = 0.0f;
        b->box = 0;
        if (b->big) {
            double P[3], N[3];
            b->axis = choose_anchor_B(sp, cam, &box, P, N);
            b->P = fk((float)P[0], (float)P[1], (float)P[2]);
            b->N = fk((float)N[0], (float)N[1], (float)N[2]);
        } else {
            b->P = fk((float)sp->position[0], (float)sp->position[1], (float)sp->position[2]);
            b->N = fk(0.0f, 0.0f, 0.0f);
        }
        b->C = fk((float)sp->position[0], (float)sp->position[1], (float)sp->position[2]);
        b->emis = fk((float)sp->emission[0], (float)sp->emission[1], (float)sp->emission[2]);
        b->col = fk((float)sp->color[0], (float)sp->color[1], (float)sp->color[2]);
        float p = b->col.x;
        if (p < b->col.y) p = b->col.y;
        if (p < b->col.z) p = b->col.z;
        b->prob = p;
        if (p > 0.0f) {
            float inv = 1.0f / p;
            b->col_rr = fk(b->col.x * inv, b->col.y * inv, b->col.z * inv);
        } else {
            b->col_rr = fk(0.0f, 0.0f, 0.0f);
        }
        b->mat = sp->material;
    }
    /* linear scan order (the kernel's record order, ptg_render.hip
     * prepare_scan_order): x-, y-, z-axis-anchored huge spheres (each axis
     * led by its wall pair, + wall first), the other huge spheres, the small
     * ones; each group otherwise in index order */
    if (n <= LINEAR_MAX_PREP) {
        pair_walls_B(s, n, cam, &box, out);
        box_mode_B(s, n, cam, &box, out);
        int j = 0;
        for (int k = 0; k < 3; ++k) {
            for (int i = 0; i < n; ++i)
                if (out[i].big && out[i].axis == k && out[i].pair == 1)
                    out[j++].visit = i;
            for (int i = 0; i < n; ++i)
                if (out[i].big && out[i].axis == k && out[i].pair == -1)
                    out[j++].visit = i;
            for (int i = 0; i < n; ++i)
                if (out[i].big && out[i].axis == k && out[i].pair == 0)
                    out[j++].visit = i;
        }
        for (int i = 0; i < n; ++i)
            if (out[i].big && out[i].axis < 0)
                out[j++].visit = i;
        for (int i = 0; i < n; ++i)
            if (!out[i].big)
                out[j++].visit = i;
    } else {
        for (int i = 0; i < n; ++i)
            out[i].visit = i;
    }
    cb->pos = fk((float)cam->position[0], (float)cam->position[1], (float)cam->position[2]);
    cb->base = fk((float)(cam->lower_left_corner[0] - cam->position[0]),
                  (float)(cam->lower_left_corner[1] - cam->position[1]),
                  (float)(cam->lower_left_corner[2] - cam->position[2]));
    cb->X = fk((float)cam->cam_x_axis[0], (float)cam->cam_x_axis[1], (float)cam->cam_x_axis[2]);
    cb->Y = fk((float)cam->cam_y_axis[0], (float)cam->cam_y_axis[1], (float)cam->cam_y_axis[2]);
    cb->lens = (float)cam->lens_radius;
    trig_table_B(cb->trig);
    cb->invW = 0.0f;
    cb->invH = 0.0f;
    float *hot = hot_B(out, n);
    for (int i = 0; i < n; ++i) {
        hot[4 * i + 0] = out[i].P.x;
        hot[4 * i + 1] = out[i].P.y;
        hot[4 * i + 2] = out[i].P.z;
        hot[4 * i + 3] = out[i].big ? NAN : out[i].negR2;
    }
}

/* sin/cos of 2*pi*u, u = m * 2^-24 with m the draw's 24-bit integer (replaces
 * libm in main.cpp:55 so host and device agree bit-for-bit): table entry
 * {cos, sin}(2*pi*k/128) for k = m >> 17, rotated by dl = 2*pi*(m mod 2^17)*2^-24
 * with sin dl = dl (1 - dl^2/6), cos dl = 1 - dl^2/2 + dl^4/24 (truncation
 * < 3e-9).  Kernel: pt_device.hpp sincos2pi_tab. */

static void sincos2pi_B(uint32_t m, const float *tab, float *c, float *s)
{
    if (g_bvar & PO_BV_LIBM_TRIG) {
        const double a = 2.0 * PO_PI * ((double)m * 0x1p-24);
        *c = (float)cos(a);
        *s = (float)sin(a);
        return;
    }
    const float *cs = tab + 2 * (m >> (24 - TRIG_BITS));
    float dl = (float)(m & ((1u << (24 - TRIG_BITS)) - 1u)) * 0x1.921fb6p-22f;
    float d2 = dl * dl;
    float sd = dl * fmaf(d2, -0x1.555556p-3f, 1.0f);
    float cd = fmaf(d2, fmaf(d2, 0x1.555556p-5f, -0.5f), 1.0f);
    *c = fmaf(cs[0], cd, -(cs[1] * sd));
    *s = fmaf(cs[1], cd, cs[0] * sd);
}

/* The table: Taylor series in double on the first octant (fixed operation
 * order, no libm), exact symmetries elsewhere, rounded to float. */
static void trig_table_B(float *tab)
{
    const double pi = 3.14159265358979323846;
    enum { OCT = TRIG_ENTRIES / 8, QUAD = TRIG_ENTRIES / 4 };
    double bc[OCT + 1], bs[OCT + 1];
    for (int r = 0; r <= OCT; ++r) {
        double a = 2.0 * pi / (double)TRIG_ENTRIES * (double)r, a2 = a * a;
        double ts = a, ss = a, tc = 1.0, sc = 1.0;
        for (int n = 1; n <= 12; ++n) {
            ts = -ts * a2 / (double)((2 * n) * (2 * n + 1));
            ss = ss + ts;
            tc = -tc * a2 / (double)((2 * n - 1) * (2 * n));
            sc = sc + tc;
        }
        bc[r] = sc;
        bs[r] = ss;
    }
    for (int k = 0; k < TRIG_ENTRIES; ++k) {
        int q = k / QUAD, r = k % QUAD;
        double c0 = r <= OCT ? bc[r] : bs[QUAD - r], s0 = r <= OCT ? bs[r] : bc[QUAD - r];
        double c = q == 0 ? c0 : (q == 1 ? -s0 : (q == 2 ? -c0 : s0));
        double s = q == 0 ? s0 : (q == 1 ? c0 : (q == 2 ? -s0 : -c0));
        tab[2 * k] = (float)c;
        tab[2 * k + 1] = (float)s;
    }
}

/* Scene scan, Mode B (main.cpp:30-42 + sphere.cpp:6-30 with the stable
 * quadratic roots; huge spheres use the anchored form).  With
 * q = -(hb + sign(hb) sqrt(disc)) the roots are c/q and q/a, and c/q is the
 * nearer one whenever hb < 0; the nearest root >= eps is therefore c/q, else
 * (hb < 0 only) q/a.  Two exact culls skip spheres that provably cannot win
 * (they never change the result: DESIGN.md "scene scan"). */
#define CULL_MARGIN 0x1.00001p+0f /* 1 + 2^-20 */
/* one candidate: the nearest root >= eps of sphere i, if nearer than bn/bq */
static void test_B(const sphB *sp, int i, f3 o, f3 d, float a, float *bn, float *bq, int *id)
{
    f3 e = fk(o.x - sp->P.x, o.y - sp->P.y, o.z - sp->P.z);
    float ed = fdot(e, d);
    float ee = fdot(e, e);
    float hb, c;
    if (sp->big) {
        hb = fmaf(sp->R, fdot(sp->N, d), ed);
        c = fmaf(sp->R2x, fdot(e, sp->N), ee);
    } else {
        hb = ed;
        c = ee + sp->negR2;
    }
    if (hb >= 0.0f && c >= 0.0f)
        return; /* both roots <= 0: num = -c <= 0 is rejected below (exact) */
    /* small spheres: Lagrange's identity hb^2 - a c = a R^2 - |e x d|^2
     * (no cancellation between two terms of size a|e|^2); the kernel's
     * scene_scan, DESIGN.md "error budget" */
    float disc = fmaf(hb, hb, -(a * c));
    if (!sp->big && !(g_bvar & PO_BV_DISC_NAIVE)) {
        f3 x = fcross(e, d);
        disc = fmaf(a, -sp->negR2, -fdot(x, x));
    }
    if (disc < 0.0f)
        return;
    float sq = sqrt_scan_B(disc); /* disc >= 0 here */
    float num, den;
    if (!sp->big && (g_bvar & PO_BV_NAIVE_ROOTS)) {
        const float tn = -hb - sq;
        num = tn < EPSF * a ? sq - hb : tn;
        den = a;
        if (num < EPSF * a)
            return;
    } else if (hb < 0.0f) {
        float q = sq - hb; /* > 0; roots c/q (near) and q/a (far) */
        num = c;
        den = q;
        if (c < EPSF * q) { /* near root < eps */
            num = q;
            den = a;
            if (q < EPSF * a)
                return;
        }
    } else {
        float qn = hb + sq; /* > 0 here (c < 0): root c/-qn */
        num = -c;
        den = qn;
        if (num < EPSF * den)
            return;
    }
    if (num * *bq < *bn * den) {
        *bn = num;
        *bq = den;
        *id = i;
    }
}

#define FAR_PLANE 1e30f
#define PLANE_MARGIN 0x1.ffep-1f /* 1 - 2^-12 */

/* Box mode walls (the kernel's scene_scan): the wall of the nearest tangent
 * plane the ray moves toward first; another wall only where its plane is not
 * safely beyond that root, or every wall for an origin outside the room.
 * Returns the number of scan positions consumed (the walls). */
static int box_walls_B(const sphB *s, int n, f3 o, f3 d, float a, float *bn, float *bq, int *id)
{
    int rec_plus[3] = {-1, -1, -1}, rec_minus[3] = {-1, -1, -1};
    /* a missing wall's plane is at +-inf: never the nearest, never needed */
    float plane_plus[3] = {INFINITY, INFINITY, INFINITY}, plane_minus[3] = {-INFINITY, -INFINITY, -INFINITY};
    float lo[3] = {-FAR_PLANE, -FAR_PLANE, -FAR_PLANE}, hi[3] = {FAR_PLANE, FAR_PLANE, FAR_PLANE};
    int nw = 0;
    while (nw < n && s[s[nw].visit].big && s[s[nw].visit].axis >= 0) { /* the walls lead the scan order */
        const int i = s[nw].visit, k = s[i].axis;
        const float nk = fcomp(s[i].N, k);
        if (nk < 0.0f) {
            rec_plus[k] = i;
            plane_plus[k] = fcomp(s[i].P, k);
            if (s[i].pair == 1) {
                lo[k] = s[i].plo;
                hi[k] = s[i].phi;
            } else {
                hi[k] = s[i].phi;
            }
        } else {
            rec_minus[k] = i;
            plane_minus[k] = fcomp(s[i].P, k);
            if (s[i].pair == 0)
                lo[k] = s[i].plo;
        }
        ++nw;
    }
    const int in_room = o.x >= lo[0] && o.x <= hi[0] && o.y >= lo[1] && o.y <= hi[1] && o.z >= lo[2] &&
                        o.z <= hi[2];
    float u[3], v[3];
    int ci[3];
    for (int k = 0; k < 3; ++k) {
        const float dk = fcomp(d, k);
        const int pos = dk >= 0.0f;
        u[k] = pos ? plane_plus[k] - fcomp(o, k) : fcomp(o, k) - plane_minus[k];
        v[k] = fabsf(dk);
        ci[k] = pos ? rec_plus[k] : rec_minus[k];
    }
    float un = u[0], vn = v[0];
    int in = ci[0], kn = 0;
    for (int k = 1; k < 3; ++k)
        if (u[k] * vn < un * v[k]) {
            un = u[k];
            vn = v[k];
            in = ci[k];
            kn = k;
        }
    /* in < 0 only when no existing wall the ray moves toward has v > 0: no
     * wall can be hit from inside the room (the kernel masks the test) */
    if (in >= 0)
        test_B(&s[in], in, o, d, a, bn, bq, id);
    const float bqm = *bq * PLANE_MARGIN;
    int need[3];
    for (int k = 0; k < 3; ++k) /* a missing wall: u = inf, never needed; guarded as well */
        need[k] = k != kn && ci[k] >= 0 && !(*bn * v[k] < u[k] * bqm);
    for (int k = 0; k < 3; ++k)
        if (need[k])
            test_B(&s[ci[k]], ci[k], o, d, a, bn, bq, id);
    /* a wall the ray moves away from can be hit only from beyond its tangent
     * plane (outside the room's bound on that side: after a bounce off a
     * curved wall far from its tangent point); those are tested last */
    for (int k = 0; k < 3; ++k) {
        const float ok = fcomp(o, k);
        const int pos = fcomp(d, k) >= 0.0f;
        const int w = pos ? rec_minus[k] : rec_plus[k];
        const int beyond = pos ? !(ok >= lo[k]) : !(ok <= hi[k]);
        if (w >= 0 && beyond)
            test_B(&s[w], w, o, d, a, bn, bq, id);
    }
    (void)in_room;
    return nw;
}

static int intersect_B(const sphB *s, int n, f3 o, f3 d, float *tout, int *idout)
{
    /* nearest root kept as a fraction bn/bq (bq > 0): candidates are compared
     * by cross-multiplication and only the winner is divided */
    float a = fdot(d, d);
    float bn = INFF, bq = 1.0f;
    int id = -1;
    int j0 = 0;
    if (g_bvar & PO_BV_FULL_SCAN) {
        for (int i = 0; i < n; ++i)
            test_B(&s[i], i, o, d, a, &bn, &bq, &id);
        *tout = id >= 0 ? div_B(bn, bq) : INFF;
        *idout = id;
        return id >= 0;
    }
    if (n > 0 && s[0].box)
        j0 = box_walls_B(s, n, o, d, a, &bn, &bq, &id);
    for (int j = j0; j < n; ++j) {
        const int i = s[j].visit; /* scan order: first visited wins exact ties */
        if (s[i].pair == 1) { /* wall pair: + wall at j, - wall at j + 1 */
            const int im = s[j + 1].visit, k = s[i].axis;
            const float dk = k == 0 ? d.x : (k == 1 ? d.y : d.z), ok = k == 0 ? o.x : (k == 1 ? o.y : o.z);
            const int first = dk >= 0.0f ? i : im, second = dk >= 0.0f ? im : i;
            test_B(&s[first], first, o, d, a, &bn, &bq, &id);
            if (!(ok >= s[i].plo) || !(ok <= s[i].phi)) /* origin outside the room: both */
                test_B(&s[second], second, o, d, a, &bn, &bq, &id);
            j += 1;
            continue;
        }
        test_B(&s[i], i, o, d, a, &bn, &bq, &id);
    }
    *tout = id >= 0 ? div_B(bn, bq) : INFF;
    *idout = id;
    return id >= 0;
}

/* Scenes with more than LINEAR_MAX spheres (the GPU walks a BVH there): the
 * reference's own rule -- every candidate root divided, t = fl(num/den), the
 * smallest t wins, lowest index on ties (main.cpp:35 strict < in index order).
 * Per-sphere arithmetic as intersect_B; the cull compares against tb. */
#define LINEAR_MAX 64
/* The discriminant of sphere sp (the kernel's forms; hb, c as above). */
static float disc_B_lex(const sphB *sp, f3 e, f3 d, float a, float hb, float c)
{
    float disc = fmaf(hb, hb, -(a * c));
    if (!sp->big && !(g_bvar & PO_BV_DISC_NAIVE)) {
        /* Lagrange form, limited to hb^2 for an origin outside (c >= 0:
         * exactly disc <= hb^2) so that the cull below stays exact */
        f3 x = fcross(e, d);
        disc = fmaf(a, -sp->negR2, -fdot(x, x));
        disc = c >= 0.0f ? fminf(disc, hb * hb) : disc;
    }
    return disc;
}

static int intersect_B_lex(const sphB *s, int n, f3 o, f3 d, float *tout, int *idout)
{
    float a = fdot(d, d);
    float tb = INFF;
    int id = -1;
    /* Blocks of 64 spheres: first the rejections that do not depend on tb
     * (both roots behind, no real root: the same disc as below), branch-free
     * from a compact copy of the records, then the full test of the
     * survivors in index order.  Every rejection is a pure "skip", so the
     * result is that of testing every sphere in order (only faster: the
     * unpredictable branches ran for all 10,000 spheres of C5). */
    const float *hot = hot_B(s, n);
    const int naive = (g_bvar & PO_BV_DISC_NAIVE) != 0;
    int cand[64];
    for (int b0 = 0; b0 < n; b0 += 64) {
        const int b1 = b0 + 64 < n ? b0 + 64 : n;
        int nc = 0;
        for (int i = b0; i < b1; ++i) {
            const float *h = hot + 4 * i;
            const f3 e = fk(o.x - h[0], o.y - h[1], o.z - h[2]);
            const float hb = fdot(e, d), c = fdot(e, e) + h[3];  /* huge spheres: NaN, kept */
            float disc;
            if (naive) {
                disc = fmaf(hb, hb, -(a * c));
            } else {
                const f3 x = fcross(e, d);
                disc = fmaf(a, -h[3], -fdot(x, x));
                /* = fminf(disc, m) (NaN operands included) without the libm call */
                const float m = hb * hb;
                disc = c >= 0.0f ? (disc < m ? disc : (m != m ? disc : m)) : disc;
            }
            cand[nc] = i;
            nc += !((hb >= 0.0f) & (c >= 0.0f)) & !(disc < 0.0f);
        }
        for (int k = 0; k < nc; ++k) {
            const int i = cand[k];
            const sphB *sp = &s[i];
            f3 e = fk(o.x - sp->P.x, o.y - sp->P.y, o.z - sp->P.z);
            float ed = fdot(e, d);
            float ee = fdot(e, e);
            float hb, c;
            if (sp->big) {
                hb = fmaf(sp->R, fdot(sp->N, d), ed);
                c = fmaf(sp->R2x, fdot(e, sp->N), ee);
            } else {
                hb = ed;
                c = ee + sp->negR2;
            }
            if (hb >= 0.0f && c >= 0.0f)
                continue;
            if (hb < 0.0f && c > 0.0f && c >= (tb * (-2.0f * hb)) * CULL_MARGIN)
                continue;
            float disc = disc_B_lex(sp, e, d, a, hb, c);
            if (disc < 0.0f)
                continue;
            float sq = sqrt_scan_B(disc);
            float num, den;
            if (hb < 0.0f) {
                float q = sq - hb;
                num = c;
                den = q;
                if (c < EPSF * q) {
                    num = q;
                    den = a;
                    if (q < EPSF * a)
                        continue;
                }
            } else {
                float qn = hb + sq;
                num = -c;
                den = qn;
                if (num < EPSF * den)
                    continue;
            }
            float t = num / den;
            if (t < tb) {
                tb = t;
                id = i;
            }
        }
    }
    *tout = tb;
    *idout = id;
    return id >= 0;
}

static f3 sample_B(const sphB *s, int n, const camB *cam, int nsub, int x, int y, int sx, int sy,
                   uint32_t st, int *segs)
{
    float sl = 1.0f / (float)nsub;
    float u1 = po_xs_f32(&st);
    float u2 = po_xs_f32(&st);
    float xin = fmaf(sl, u1, (float)x + (float)sx * sl);
    float yin = fmaf(sl, u2, (float)y + (float)sy * sl);
    float fs = xin * cam->invW, ft = yin * cam->invH; /* main.cpp:190 x/W, y/H as x * (1/W) */
    float px, py;
    for (;;) {
        px = fmaf(2.0f, po_xs_f32(&st), -1.0f);
        py = fmaf(2.0f, po_xs_f32(&st), -1.0f);
        if (fmaf(py, py, px * px) >= 1.0f)
            continue;
        break;
    }
    float sst = fs + ft;
    float ox = (px * cam->lens) * sst, oy = (py * cam->lens) * sst;
    f3 o = fk(cam->pos.x + ox, cam->pos.y + oy, cam->pos.z);
    f3 d = fk(fmaf(cam->Y.x, ft, fmaf(cam->X.x, fs, cam->base.x)) - ox,
              fmaf(cam->Y.y, ft, fmaf(cam->X.y, fs, cam->base.y)) - oy,
              fmaf(cam->Y.z, ft, fmaf(cam->X.z, fs, cam->base.z)));
    f3 E = fk(0, 0, 0), T = fk(1, 1, 1);
    *segs = 0;
    for (int depth = 0; depth < PO_DEPTH_LIMIT; ++depth) {
        float t;
        int id;
        (*segs)++;
        if (!(n > LINEAR_MAX || (g_bvar & PO_BV_LEX) ? intersect_B_lex(s, n, o, d, &t, &id)
                                                     : intersect_B(s, n, o, d, &t, &id))) {
            f3 ud = fnorm(d);
            float tt = 0.5f * (ud.y + 1.0f);
            float it = 1.0f - tt;
            E = fk(fmaf(T.x, fmaf(tt, 0.5f, it), E.x), fmaf(T.y, fmaf(tt, 0.7f, it), E.y),
                   fmaf(T.z, fmaf(tt, 1.0f, it), E.z));
            return E;
        }
        const sphB *sp = &s[id];
        f3 p = fk(fmaf(d.x, t, o.x), fmaf(d.y, t, o.y), fmaf(d.z, t, o.z));
        /* hit_record.cpp:6: (p - C).norm(), as (p - C) * (1/R): p lies on the sphere */
        f3 on = fk((p.x - sp->C.x) * sp->invR, (p.y - sp->C.y) * sp->invR, (p.z - sp->C.z) * sp->invR);
        if (g_bvar & PO_BV_RENORM)
            on = fnorm(fk(p.x - sp->C.x, p.y - sp->C.y, p.z - sp->C.z));
        int front = fdot(on, d) < 0.0f;
        f3 nn = front ? on : fk(-on.x, -on.y, -on.z);
        E = fk(fmaf(T.x, sp->emis.x, E.x), fmaf(T.y, sp->emis.y, E.y), fmaf(T.z, sp->emis.z, E.z));
        f3 col = sp->col;
        if (depth > PO_RR_THRESHOLD) {
            if (po_xs_f32(&st) < sp->prob)
                col = sp->col_rr;
            else
                return E;
        }
        T = fk(T.x * col.x, T.y * col.y, T.z * col.z);
        int reflect = 0;
        if (sp->mat == 0) { /* diffuse, main.cpp:44-58 */
            uint32_t m_phi = po_xorshift32(&st) >> 8;
            float ra = po_xs_f32(&st);
            float cp, sp_;
            sincos2pi_B(m_phi, cam->trig, &cp, &sp_);
            float sth = sqrt_B(ra);
            float cth = sqrt_B(1.0f - ra);
            f3 w = nn;
            f3 uu = fabsf(w.x) > 0.1f ? fk(w.z, 0.0f, -w.x) : fk(0.0f, -w.z, w.y);
            uu = fnorm(uu);
            f3 vv = fcross(w, uu);
            float cs = cp * sth, ss = sp_ * sth;
            f3 nd = fk(fmaf(w.x, cth, fmaf(vv.x, ss, uu.x * cs)), fmaf(w.y, cth, fmaf(vv.y, ss, uu.y * cs)),
                       fmaf(w.z, cth, fmaf(vv.z, ss, uu.z * cs)));
            if (g_bvar & PO_BV_RENORM)
                nd = fnorm(nd);
            o = p; /* main.cpp:55 normalises u*cos*sin + v*sin*sin + w*cos, a unit vector by construction */
            d = nd;
            continue;
        } else if (sp->mat == 2) { /* dielectric, main.cpp:69-97 */
            float ratio = front ? 0.5f : 2.0f;
            f3 ud = fnorm(d);
            float x0 = -fdot(ud, nn);
            float cth = 1.0f < x0 ? 1.0f : x0;
            float sth = sqrt_B(fmaf(-cth, cth, 1.0f));
            int cannot = ratio * sth > 1.0f;
            if (cannot) {
                reflect = 1;
            } else {
                const float r0 = 0x1.c71c74p-4f; /* ((1-ratio)/(1+ratio))^2 for ratio 0.5 and 2 */
                float xm = 1.0f - cth;
                float x2 = xm * xm;
                float x5 = (x2 * x2) * xm;
                float R = fmaf(1.0f - r0, x5, r0);
                reflect = R > po_xs_f32(&st);
            }
            if (!reflect) {
                f3 perp = fk(fmaf(nn.x, cth, ud.x) * ratio, fmaf(nn.y, cth, ud.y) * ratio,
                             fmaf(nn.z, cth, ud.z) * ratio);
                float sq = sqrt_B(fabsf(1.0f - fdot(perp, perp)));
                o = p;
                d = fk(fmaf(nn.x, -sq, perp.x), fmaf(nn.y, -sq, perp.y), fmaf(nn.z, -sq, perp.z));
                continue;
            }
        }
        /* specular (main.cpp:60-67), also the dielectric's reflection */
        {
            float k = fdot(on, d);
            k = k + k;
            (void)po_xs_f32(&st); /* fuzz draw: consumed, times 0 */
            o = p;
            d = fk(fmaf(-k, on.x, d.x), fmaf(-k, on.y, d.y), fmaf(-k, on.z, d.z));
        }
    }
    return E;
}

/* Exact, order-independent sample accumulation (include/ptgpu.h "Sample
 * accumulation"): q(c) = trunc(c * 2^32), c clamped to [0, 2^30]; the
 * sub-pixel mean is (float)((double)sum * 2^-32 / samps) (main.cpp:192). */
static uint64_t quant_B(float c)
{
    if (!(c >= 0.0f))
        return 0;
    if (c > 0x1p30f)
        c = 0x1p30f;
    return (uint64_t)((double)c * 0x1p32);
}

static float mean_B(uint64_t sum, int samps)
{
    return samps > 0 ? (float)(((double)sum * 0x1p-32) / (double)samps) : 0.0f;
}

/* quant_B is exact on [0, 2^30]; other values (NaN, negative, larger) are
 * clipped -- counted by po_render_xs_f32_ex (the kernel's
 * PTG_FLAG_COUNT_NONFINITE) */
static int in_quant_range_B(float c) { return c >= 0.0f && c <= 0x1p30f; }

static f3 subpixel_B(const sphB *s, int n, const camB *cam, int samps, int nsub, int x, int y,
                     int sx, int sy, uint64_t key, uint64_t *segs, uint64_t *bad)
{
    uint64_t ax = 0, ay = 0, az = 0;
    for (int k = 0; k < samps; ++k) {
        int sg = 0;
        f3 c = sample_B(s, n, cam, nsub, x, y, sx, sy, po_sample_state(key, (uint32_t)k), &sg);
        *segs += (uint64_t)sg;
        *bad += !(in_quant_range_B(c.x) && in_quant_range_B(c.y) && in_quant_range_B(c.z));
        ax += quant_B(c.x);
        ay += quant_B(c.y);
        az += quant_B(c.z);
    }
    return fk(mean_B(ax, samps), mean_B(ay, samps), mean_B(az, samps));
}

static float clampf_B(float v) { return v < 0.0f ? 0.0f : (1.0f < v ? 1.0f : v); }

int po_render_xs_f32(const po_sphere *s, int n, const po_camera *cam, int W, int H, int samps, int nsub,
                     uint64_t seed, int y0, int y1, int ystep, int nthreads, float *image, uint64_t *segments)
{
    return po_render_xs_f32_ex(s, n, cam, W, H, samps, nsub, seed, y0, y1, ystep, nthreads, image, segments, NULL);
}

int po_render_xs_f32_ex(const po_sphere *s, int n, const po_camera *cam, int W, int H, int samps, int nsub,
                        uint64_t seed, int y0, int y1, int ystep, int nthreads, float *image, uint64_t *segments,
                        uint64_t *out_of_range)
{
    if (check_args(n, W, H, samps, nsub) || ystep <= 0)
        return -1;
    sphB *sb = malloc_sphB(n);
    camB cb;
    prep_B(s, n, cam, sb, &cb);
    cb.invW = 1.0f / (float)W;
    cb.invH = 1.0f / (float)H;
    uint64_t total = 0, nbad = 0;
    float q = 1.0f / (float)(nsub * nsub);
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : total, nbad)
    for (int y = y0; y < y1; y += ystep) {
        for (int x = 0; x < W; ++x) {
            f3 pix = fk(0, 0, 0);
            for (int sy = 0; sy < nsub; ++sy)
                for (int sx = 0; sx < nsub; ++sx) {
                    uint64_t ps = ((uint64_t)y * (uint64_t)W + (uint64_t)x) * (uint64_t)(nsub * nsub) +
                                  (uint64_t)(sy * nsub + sx);
                    uint64_t segs = 0, bad = 0;
                    f3 a = subpixel_B(sb, n, &cb, samps, nsub, x, y, sx, sy, po_key_hash(seed, ps), &segs, &bad);
                    total += segs;
                    nbad += bad;
                    pix = fk(fmaf(clampf_B(a.x), q, pix.x), fmaf(clampf_B(a.y), q, pix.y),
                             fmaf(clampf_B(a.z), q, pix.z));
                }
            size_t row = (size_t)(H - y - 1) * (size_t)W + (size_t)x;
            image[3 * row + 0] = pix.x;
            image[3 * row + 1] = pix.y;
            image[3 * row + 2] = pix.z;
        }
    }
    free(sb);
    if (segments)
        *segments = total;
    if (out_of_range)
        *out_of_range = nbad;
    return 0;
}

/* Rectangle renders (tests at the BASELINE sample counts): pixels
 * x in [x0, x1) of rows y = y0, y0 + ystep, ... < y1, parallel over PIXELS
 * (the row renders above are parallel over rows, so one row runs on one
 * thread).  Same per-pixel arithmetic as po_render_xs_f64 / _f32; pixels
 * outside the rectangle are left untouched. */
int po_render_xs_f64_rect(const po_sphere *s, int n, const po_camera *cam, int W, int H, int samps, int nsub,
                          uint64_t seed, int x0, int x1, int y0, int y1, int ystep, int nthreads, double *image,
                          uint64_t *segments)
{
    if (check_args(n, W, H, samps, nsub) || ystep <= 0 || x0 < 0 || x1 > W || x0 > x1 || y0 < 0 || y1 > H)
        return -1;
    const long nx = x1 - x0, ny = y1 > y0 ? (y1 - y0 + ystep - 1) / ystep : 0;
    uint64_t total = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : total)
    for (long i = 0; i < nx * ny; ++i) {
        const int y = y0 + (int)(i / nx) * ystep, x = x0 + (int)(i % nx);
        for (int sy = 0; sy < nsub; ++sy)
            for (int sx = 0; sx < nsub; ++sx) {
                uint64_t ps = ((uint64_t)y * (uint64_t)W + (uint64_t)x) * (uint64_t)(nsub * nsub) +
                              (uint64_t)(sy * nsub + sx);
                rngA r = {NULL, 0, 0};
                uint64_t segs = 0;
                v3 a = subpixel_A(s, n, cam, W, H, samps, nsub, x, y, sx, sy, &r, po_key_hash(seed, ps), &segs);
                total += segs;
                double *px = image + 3 * ((size_t)(H - y - 1) * (size_t)W + (size_t)x);
                double q = 1.0 / (nsub * nsub);
                px[0] = px[0] + po_clamp(a.x) * q;
                px[1] = px[1] + po_clamp(a.y) * q;
                px[2] = px[2] + po_clamp(a.z) * q;
            }
    }
    if (segments)
        *segments = total;
    return 0;
}

int po_render_xs_f32_rect(const po_sphere *s, int n, const po_camera *cam, int W, int H, int samps, int nsub,
                          uint64_t seed, int x0, int x1, int y0, int y1, int ystep, int nthreads, float *image,
                          uint64_t *segments)
{
    if (check_args(n, W, H, samps, nsub) || ystep <= 0 || x0 < 0 || x1 > W || x0 > x1 || y0 < 0 || y1 > H)
        return -1;
    sphB *sb = malloc_sphB(n);
    camB cb;
    prep_B(s, n, cam, sb, &cb);
    cb.invW = 1.0f / (float)W;
    cb.invH = 1.0f / (float)H;
    const long nx = x1 - x0, ny = y1 > y0 ? (y1 - y0 + ystep - 1) / ystep : 0;
    uint64_t total = 0;
    float q = 1.0f / (float)(nsub * nsub);
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : total)
    for (long i = 0; i < nx * ny; ++i) {
        const int y = y0 + (int)(i / nx) * ystep, x = x0 + (int)(i % nx);
        f3 pix = fk(0, 0, 0);
        for (int sy = 0; sy < nsub; ++sy)
            for (int sx = 0; sx < nsub; ++sx) {
                uint64_t ps = ((uint64_t)y * (uint64_t)W + (uint64_t)x) * (uint64_t)(nsub * nsub) +
                              (uint64_t)(sy * nsub + sx);
                uint64_t segs = 0, bad = 0;
                f3 a = subpixel_B(sb, n, &cb, samps, nsub, x, y, sx, sy, po_key_hash(seed, ps), &segs, &bad);
                total += segs;
                pix = fk(fmaf(clampf_B(a.x), q, pix.x), fmaf(clampf_B(a.y), q, pix.y), fmaf(clampf_B(a.z), q, pix.z));
            }
        const size_t row = (size_t)(H - y - 1) * (size_t)W + (size_t)x;
        image[3 * row + 0] = pix.x;
        image[3 * row + 1] = pix.y;
        image[3 * row + 2] = pix.z;
    }
    free(sb);
    if (segments)
        *segments = total;
    return 0;
}

void po_mode_b_math(const float *a, const float *b, size_t n, float *quot, float *root)
{
    for (size_t i = 0; i < n; ++i) {
        quot[i] = div_B(a[i], b[i]);
        root[i] = sqrt_B(a[i]);
    }
}

void po_mode_b_roots(const float *a, size_t n, float *sq_scan, float *rsq)
{
    for (size_t i = 0; i < n; ++i) {
        sq_scan[i] = sqrt_scan_B(a[i]);
        rsq[i] = rsqrt_B(a[i]);
    }
}

void po_sincos2pi(const uint32_t *m, size_t n, float *out)
{
    float tab[2 * TRIG_ENTRIES];
    trig_table_B(tab);
    for (size_t i = 0; i < n; ++i)
        sincos2pi_B(m[i] & 0xFFFFFFu, tab, &out[2 * i], &out[2 * i + 1]);
}

int po_scan_layout(const po_sphere *s, int n, const po_camera *cam, int32_t *axis, int32_t *order)
{
    if (n < 0)
        return -1;
    sphB *sb = malloc_sphB(n);
    camB cb;
    prep_B(s, n, cam, sb, &cb);
    for (int i = 0; i < n; ++i) {
        axis[i] = sb[i].pair != 0 ? sb[i].axis + 3 : sb[i].axis; /* 3..5: paired wall */
        order[i] = sb[i].visit;
    }
    free(sb);
    return 0;
}

int po_sample_f32(const po_sphere *s, int n, const po_camera *cam, int W, int H, int nsub, uint64_t seed, int x,
                  int y, int sx, int sy, uint32_t sample, float out[3])
{
    sphB *sb = malloc_sphB(n);
    camB cb;
    prep_B(s, n, cam, sb, &cb);
    cb.invW = 1.0f / (float)W;
    cb.invH = 1.0f / (float)H;
    uint64_t ps = ((uint64_t)y * (uint64_t)W + (uint64_t)x) * (uint64_t)(nsub * nsub) + (uint64_t)(sy * nsub + sx);
    int segs = 0;
    f3 c = sample_B(sb, n, &cb, nsub, x, y, sx, sy, po_sample_state(po_key_hash(seed, ps), sample), &segs);
    out[0] = c.x;
    out[1] = c.y;
    out[2] = c.z;
    free(sb);
    return segs;
}

/* ========================================================================= */
/* Scenes: values of simple_scene.hpp:18-49, box_scene.hpp:16-69,             */
/* box_mirror_scene.hpp:16-69, computed with the same double expressions.     */
/* ========================================================================= */
static void put(po_sphere *s, double r, double px, double py, double pz, double ex, double ey, double ez, double cx,
                double cy, double cz, int m)
{
    memset(s, 0, sizeof(*s));
    s->radius = r;
    s->position[0] = px; s->position[1] = py; s->position[2] = pz;
    s->emission[0] = ex; s->emission[1] = ey; s->emission[2] = ez;
    s->color[0] = cx; s->color[1] = cy; s->color[2] = cz;
    s->material = m;
}

static void cfg_defaults(po_camera_config *c)
{
    memset(c, 0, sizeof(*c));
    c->up[1] = 1.0;                      /* camera.hpp:15 */
    c->aspect_ratio = 16.0 / 9.0;        /* camera.hpp:16 */
    c->vertical_fov_radians = 0.785398163; /* camera.hpp:17 */
    c->focal_length = 1.0;               /* camera.hpp:18 */
}

int po_scene(int id, int w, int h, po_sphere *out, int cap, po_camera_config *cfg)
{
    po_sphere tmp[8];
    int n = 0;
    cfg_defaults(cfg);
    if (id == 0) { /* simple_scene.hpp:14-52 */
        put(&tmp[n++], 100.0, 0.0, -100.5, -1.0, 0, 0, 0, 0.8, 0.8, 0.0, 0);
        put(&tmp[n++], 0.5, 1.0, 0.0, -1.0, 0, 0, 0, 0.999, 0.999, 0.999, 1);
        put(&tmp[n++], 0.5, -1.0, 0.0, -1.0, 0, 0, 0, 0.999, 0.999, 0.999, 2);
        put(&tmp[n++], 0.5, 0.0, 0.0, -1.0, 0.1, 0.1, 0.9, 0.0, 0.7, 0.1, 0);
        put(&tmp[n++], 1.0, 1.0, 3.1, -1.0, 30.0, 30.0, 30.0, 0.0, 0.0, 0.0, 0);
        cfg->position[0] = -2.0; cfg->position[1] = 2.0; cfg->position[2] = 1.0;
        cfg->direction[0] = 0.0; cfg->direction[1] = 0.0; cfg->direction[2] = -1.0;
        cfg->vertical_fov_radians = 1.2;
    } else if (id == 1 || id == 2) { /* box_scene.hpp:14-72 / box_mirror_scene.hpp:14-72 */
        const double big = 1E6, off = 0.4, y = 0.0, z = -1.0;
        int wall = id == 1 ? 0 : 1;
        put(&tmp[n++], big, -big - off, y, z, 0, 0, 0, 0.9, 0.1, 0.2, wall);
        put(&tmp[n++], big, big + off, y, z, 0, 0, 0, 0.3, 0.1, 0.9, wall);
        put(&tmp[n++], big, 0.0, 0.0, z - big, 0, 0, 0, 0.1, 0.7, 0.2, wall);
        put(&tmp[n++], big, 0.0, big + off, z, 0, 0, 0, 0.3, 0.7, 0.2, wall);
        put(&tmp[n++], big, 0.0, -big - off, z, 0, 0, 0, 0.9, 0.9, 0.9, wall);
        if (id == 1) {
            put(&tmp[n++], off / 2.0, 0.0, 0.0 + off / 4.0, z - off / 2.5, 9.0, 9.0, 9.0, 1.8, 1.8, 1.8, 0);
            put(&tmp[n++], off / 2.0, off / 2.0, -off / 2.0, z + off * 1.5, 0, 0, 0, 1.0, 1.0, 1.0, 1);
            put(&tmp[n++], off / 2.0, -off / 2.0, -off / 2.0, z + off * 1.5, 0, 0, 0, 1.0, 1.0, 1.0, 2);
            cfg->vertical_fov_radians = 0.5;
        } else {
            put(&tmp[n++], off / 2.0, 0.0, 0.0 + off / 4.0, z + off * 1.5, 1.92, 1.91, 1.9, 1.92, 1.91, 1.9, 0);
            put(&tmp[n++], off / 2.0, off / 2.0, -off / 2.0, z + off, 0, 0, 0, 1.0, 1.0, 1.0, 1);
            put(&tmp[n++], off / 2.0, -off / 2.0, -off / 2.0, z + off, 0, 0, 0, 1.0, 1.0, 1.0, 2);
            cfg->vertical_fov_radians = 0.75;
        }
        cfg->position[2] = 2.0;
        cfg->direction[2] = z + off * 1.5;
    } else {
        return -1;
    }
    cfg->aspect_ratio = (w * 1.0) / (h * 1.0);
    cfg->aperture = 0.2;
    double diff[3] = {cfg->position[0] - cfg->direction[0], cfg->position[1] - cfg->direction[1],
                      cfg->position[2] - cfg->direction[2]};
    cfg->focus_distance = po_vec_length(diff);
    if (n > cap)
        return -1;
    memcpy(out, tmp, sizeof(po_sphere) * (size_t)n);
    return n;
}

/* Synthetic scene (BASELINE.json configs[4]; the reference has none, the
 * generator is defined in DESIGN.md "Synthetic scene"). */
int po_scene_synthetic(int n, int w, int h, uint32_t gen_seed, po_sphere *out, po_camera_config *cfg)
{
    if (n < 2)
        return -1;
    po_mt19937 g;
    po_mt_seed(&g, gen_seed);
    cfg_defaults(cfg);
    put(&out[0], 1000.0, 0.0, -1000.0, 0.0, 0, 0, 0, 0.5, 0.5, 0.5, 0);
    put(&out[1], 2.0, 0.0, 8.0, 0.0, 8.0, 8.0, 8.0, 0.8, 0.8, 0.8, 0);
    for (int i = 2; i < n; ++i) {
        double r = 0.05 + 0.1 * po_mt_generate(&g);
        double x = -10.0 + 20.0 * po_mt_generate(&g);
        double z = -10.0 + 20.0 * po_mt_generate(&g);
        double m = po_mt_generate(&g);
        double cr = 0.2 + 0.75 * po_mt_generate(&g);
        double cg = 0.2 + 0.75 * po_mt_generate(&g);
        double cbl = 0.2 + 0.75 * po_mt_generate(&g);
        int mat = m < 0.80 ? 0 : (m < 0.95 ? 1 : 2);
        put(&out[i], r, x, r, z, 0, 0, 0, cr, cg, cbl, mat);
    }
    cfg->position[0] = 0.0; cfg->position[1] = 2.0; cfg->position[2] = 12.0;
    cfg->vertical_fov_radians = 0.8;
    cfg->aspect_ratio = (w * 1.0) / (h * 1.0);
    cfg->aperture = 0.0;
    double diff[3] = {cfg->position[0] - cfg->direction[0], cfg->position[1] - cfg->direction[1],
                      cfg->position[2] - cfg->direction[2]};
    cfg->focus_distance = po_vec_length(diff);
    return n;
}
