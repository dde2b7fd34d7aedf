// ref64.hpp -- the reference-arithmetic mode of the render loop
// (PTG_FLAG_REFERENCE_F64): the reference's per-pixel algorithm in double
// precision on the GPU, operation for operation.
//
// The fp32 megakernel (ptg_render.hip) restates the reference with fp32
// reformulations (anchored walls, Lagrange discriminant, fraction compares,
// deterministic sqrt/rsqrt sequences: DESIGN.md section 2).  This mode runs
// instead the reference's own double arithmetic as src/main.cpp and the pt
// library write it -- vec.cpp's evaluation order (x*x + y*y + z*z, norm as
// v * (1 / sqrt(v.v))), sphere.cpp:6-30's quadratic with its (-hb -+ sq) / a
// roots, the strict-< linear scan of main.cpp:30-42, camera.cpp:19-38 with the
// rejection-sampled disk, the samplers of main.cpp:44-97 with libm-style
// sin/cos/pow/sqrt, radiance main.cpp:104-158, and render_subpixel's
// sequential `r += c * (1/samps)` and clamp (main.cpp:179-197) -- compiled
// without FMA contraction (the reference's x86-64 build has none).  The only
// substitution is the north star's: the draws come from the counter RNG
// (u = m * 2^-24 of the same xorshift32 stream the fp32 kernel uses), so the
// oracle's Mode A/xs (oracle/pt_oracle.c, the same restatement on the CPU) is
// its exact counterpart: IEEE division and square root are correctly rounded
// on both sides, and only sin/cos/pow may differ from glibc's in the last ulp.
//
// One lane per sub-pixel, its samples in order (the reference's loop);
// 16 pixels x 4 sub-pixels per wave; a pixel's 4 lanes combine their clamped
// means in (sy, sx) order like main.cpp:196.  A parity mode, not the
// benchmark: fp64 VALU runs at half the fp32 rate on MI355X and the scan is
// the reference's linear one.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ptgpu.h"
#include "pt_device.hpp"

namespace ptg {
namespace ref64 {

constexpr double kEps = 1e-4;    // constants.hpp:7
constexpr double kPi = 3.14159265358979323846;  // constants.hpp:8
constexpr double kInf = 1e20;    // constants.hpp:9

struct d3 {
    double x, y, z;
};
__device__ inline d3 mk(double x, double y, double z) { return d3{x, y, z}; }
__device__ inline d3 add(d3 a, d3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }    // vec.cpp:15-18
__device__ inline d3 sub(d3 a, d3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }    // vec.cpp:20-23
__device__ inline d3 mul(d3 a, double s) { return mk(a.x * s, a.y * s, a.z * s); }     // vec.cpp:25-28
__device__ inline d3 blend(d3 a, d3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); } // vec.cpp:30-33
__device__ inline double dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } // vec.cpp:40-43
__device__ inline d3 norm(d3 a) { return mul(a, 1 / sqrt(a.x * a.x + a.y * a.y + a.z * a.z)); }  // vec.cpp:35-38
__device__ inline d3 cross(d3 a, d3 b)                                                  // vec.cpp:45-48
{
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ inline d3 ld(const double *p) { return mk(p[0], p[1], p[2]); }

// random_state.cpp:9-17 with the counter RNG's draws
__device__ inline double draw(uint32_t &st) { return (double)draw_bits(st) * 0x1p-24; }
__device__ inline double between(uint32_t &st, double lo, double hi) { return lo + (hi - lo) * draw(st); }

// sphere.cpp:6-30
__device__ inline double intersect(const ptg_sphere &s, d3 o, d3 d)
{
    const d3 oc = sub(o, ld(s.position));
    const double a = dot(d, d);
    const double hb = dot(oc, d);
    const double c = dot(oc, oc) - s.radius * s.radius;
    const double disc = hb * hb - a * c;
    if (disc < 0)
        return 0.0;
    const double sq = sqrt(disc);
    double root = (-hb - sq) / a;
    if (root < kEps) {
        root = (-hb + sq) / a;
        if (root < kEps)
            return 0.0;
    }
    return root;
}

struct Hit {
    d3 p, on, n;
    bool front;
};

// main.cpp:30-42: strict < keeps the lowest index on ties
__device__ inline int scene_intersect(const ptg_sphere *s, int n, d3 o, d3 d, double &t)
{
    t = kInf;
    int id = -1;
    for (int i = 0; i < n; ++i) {
        const double dd = intersect(s[i], o, d);
        if (dd > 0 && dd < t) {
            t = dd;
            id = i;
        }
    }
    return id;
}

// hit_record.cpp:3-12
__device__ inline Hit hit_record(const ptg_sphere &s, d3 o, d3 d, double t)
{
    Hit h;
    h.p = add(o, mul(d, t));  // ray.cpp:3-6
    h.on = norm(sub(h.p, ld(s.position)));
    h.front = dot(h.on, d) < 0;
    h.n = h.front ? h.on : mul(h.on, -1);
    return h;
}

// main.cpp:60-67 (the fuzz draw is consumed and multiplied by 0)
__device__ inline void specular(const Hit &h, d3 d, uint32_t &st, d3 &ro, d3 &rd)
{
    const d3 refl = sub(d, mul(mul(h.on, 2.0), dot(h.on, d)));
    const double f = draw(st) * 0.0;
    ro = h.p;
    rd = add(refl, mk(f, f, f));
}

// main.cpp:104-158 for the path starting at (o, d); segs += scene scans
__device__ inline d3 radiance(const ptg_sphere *s, int n, d3 o, d3 d, uint32_t &st, int &segs)
{
    d3 E = mk(0, 0, 0), T = mk(1, 1, 1);
    for (int depth = 0; depth < kDepthLimit; ++depth) {
        double t = 0.0;
        segs += 1;
        const int id = scene_intersect(s, n, o, d, t);
        if (id < 0) {  // main.cpp:115-120
            const d3 ud = norm(d);
            const double tt = 0.5 * (ud.y + 1.0);
            const d3 bg = add(mul(mk(1, 1, 1), 1.0 - tt), mul(mk(0.5, 0.7, 1.0), tt));
            return add(E, blend(T, bg));
        }
        const ptg_sphere &obj = s[id];
        const Hit h = hit_record(obj, o, d, t);
        d3 color = ld(obj.color);
        E = add(E, blend(T, ld(obj.emission)));  // main.cpp:126
        double p = color.x;                        // main.cpp:128: std::max({x, y, z})
        if (p < color.y)
            p = color.y;
        if (p < color.z)
            p = color.z;
        if (depth > kRRThreshold) {  // main.cpp:130-137
            if (draw(st) < p)
                color = mul(color, 1.0 / p);
            else
                return E;
        }
        T = blend(T, color);
        if (obj.material == PTG_DIFFUSE) {  // main.cpp:44-58
            const double phi = 2 * kPi * draw(st);
            const double ra = draw(st);
            const double sth = sqrt(ra), cth = sqrt(1.0 - ra);
            const d3 w = h.n;
            const d3 u = norm(cross(fabs(w.x) > 0.1 ? mk(0, 1, 0) : mk(1, 0, 0), w));
            const d3 v = cross(w, u);
            d = norm(add(add(mul(mul(u, cos(phi)), sth), mul(mul(v, sin(phi)), sth)), mul(w, cth)));
            o = h.p;
        } else if (obj.material == PTG_SPECULAR) {
            specular(h, d, st, o, d);
        } else {  // main.cpp:69-97
            const double ratio = h.front ? (1.0 / 2.0) : 2.0;
            const d3 ud = norm(d);
            const double x = dot(mul(ud, -1.0), h.n);
            const double ct = 1.0 < x ? 1.0 : x;  // std::min(x, 1.0)
            const double sth = sqrt(1.0 - ct * ct);
            bool refl = ratio * sth > 1.0;
            if (!refl) {  // main.cpp:89: || short-circuits the Fresnel draw
                double r0 = (1.0 - ratio) / (1.0 + ratio);  // main.cpp:82-87
                r0 *= r0;
                refl = r0 + (1.0 - r0) * pow(1.0 - ct, 5.0) > draw(st);  // C: pow(double, double)
            }
            if (refl) {
                specular(h, d, st, o, d);
            } else {
                const d3 perp = mul(add(ud, mul(h.n, ct)), ratio);
                const d3 par = mul(h.n, -sqrt(fabs(1.0 - dot(perp, perp))));
                o = h.p;
                d = add(perp, par);
            }
        }
    }
    return E;
}

struct Args {
    const ptg_sphere *spheres;
    int n;
    ptg_camera cam;
    int W, H, samps, nsub, lanes_per_pixel, pixels_per_wave, waves_per_row;
    int slab_rows, band_rows, shard_rank, shard_count;
    unsigned long long seed;
    double *out64;  // slab of doubles (ptg_render) or
    float *out32;   // floats (ptg_render_device)
    unsigned long long *segments;
};

// One lane per sub-pixel: render_subpixel (main.cpp:179-197) for all samples.
__global__ __launch_bounds__(256) void render_kernel(Args A)
{
    const int lane = threadIdx.x & 63;
    const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int slab_row = (int)(wave / A.waves_per_row);
    if (slab_row >= A.slab_rows)
        return;  // whole wave
    const int x0 = (int)(wave - (long long)slab_row * A.waves_per_row) * A.pixels_per_wave;
    const int band = slab_row / A.band_rows;
    const int r = (band * A.shard_count + A.shard_rank) * A.band_rows + (slab_row - band * A.band_rows);
    const int px = x0 + lane / A.lanes_per_pixel;
    const int subi = lane % A.lanes_per_pixel;
    const bool valid = r < A.H && px < A.W && lane < A.pixels_per_wave * A.lanes_per_pixel;
    const int y = A.H - 1 - r;  // main.cpp:181
    const int sy = subi / A.nsub, sx = subi - sy * A.nsub;
    d3 acc = mk(0, 0, 0);
    int segs = 0;
    if (valid) {
        const uint64_t key = key_hash(A.seed, ((uint64_t)y * (uint64_t)A.W + (uint64_t)px) * (uint64_t)A.lanes_per_pixel +
                                                  (uint64_t)subi);
        const ptg_camera &C = A.cam;
        for (int k = 0; k < A.samps; ++k) {
            uint32_t st = sample_state(key, (uint32_t)k);
            const double sl = 1.0 / A.nsub;
            const double xin = (px + sx * sl + between(st, 0.0, sl));  // main.cpp:186-187
            const double yin = (y + sy * sl + between(st, 0.0, sl));   // main.cpp:188
            const double s = xin / A.W, t = yin / A.H;                  // main.cpp:190
            d3 pd;
            for (;;) {  // camera.cpp:19-30
                const double ax = between(st, -1.0, 1.0);
                const double ay = between(st, -1.0, 1.0);
                pd = mk(ax, ay, 0.0);
                if (dot(pd, pd) >= 1.0)
                    continue;
                break;
            }
            // camera.cpp:32-38 (offset = rd*s + rd*t, the reference's lens quirk)
            const d3 rdk = mul(pd, C.lens_radius);
            const d3 off = add(mul(rdk, s), mul(rdk, t));
            const d3 dir = sub(sub(add(add(ld(C.lower_left_corner), mul(ld(C.cam_x_axis), s)), mul(ld(C.cam_y_axis), t)),
                                   ld(C.position)),
                               off);
            const d3 c = radiance(A.spheres, A.n, add(ld(C.position), off), dir, st, segs);
            acc = add(acc, mul(c, 1.0 / A.samps));  // main.cpp:192
        }
    }
    // main.cpp:195-196: clamp, then the pixel's sub-pixels added in (sy, sx)
    // order with weight 1/nsub^2, from zero
    const double q = 1.0 / (A.nsub * A.nsub);
    auto clampd = [](double v) { return v < 0.0 ? 0.0 : (1.0 < v ? 1.0 : v); };  // utils.cpp:6-9
    const d3 mine = mk(clampd(acc.x) * q, clampd(acc.y) * q, clampd(acc.z) * q);
    const int first = lane - subi;
    d3 pix = mk(0, 0, 0);
    for (int j = 0; j < A.lanes_per_pixel; ++j) {
        const int src = first + j;
        pix = add(pix, mk(__shfl(mine.x, src, 64), __shfl(mine.y, src, 64), __shfl(mine.z, src, 64)));
    }
    if (valid && subi == 0) {
        const size_t o = ((size_t)slab_row * A.W + px) * 3;
        if (A.out64) {
            A.out64[o] = pix.x;
            A.out64[o + 1] = pix.y;
            A.out64[o + 2] = pix.z;
        } else {
            A.out32[o] = (float)pix.x;
            A.out32[o + 1] = (float)pix.y;
            A.out32[o + 2] = (float)pix.z;
        }
    }
    if (A.segments) {
        unsigned long long ws = valid ? (unsigned long long)segs : 0ull;
        for (int off = 32; off > 0; off >>= 1)
            ws += __shfl_xor(ws, off, 64);
        if (lane == 0 && ws)
            atomicAdd(A.segments, ws);
    }
}

}  // namespace ref64
}  // namespace ptg
