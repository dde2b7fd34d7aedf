// pt_device.hpp -- device-side math of the MI355X render loop (gfx950).
//
// fp32 restatement of the reference's hot path, written so that every value
// is produced by a fixed sequence of IEEE-754 operations (explicit fmaf,
// correctly-rounded division, a Newton rsqrt, a polynomial sin/cos), which
// the oracle's Mode B (oracle/pt_oracle.c) executes on the host in the same
// order -- the GPU image equals the CPU image bit-for-bit.  Compiled with
// -ffp-contract=off: nothing fuses unless fmaf is written.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ptg {

// constants.hpp:7-10, main.cpp:106
constexpr float kEps = 1e-4f;
constexpr float kInf = 1e20f;
constexpr int kDepthLimit = 100;
constexpr int kRRThreshold = 4;

struct f3 {
    float x, y, z;
};

__device__ __forceinline__ f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ float dot3(f3 a, f3 b) { return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x)); }
__device__ __forceinline__ f3 sub3(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
// Deterministic reciprocal square root: bit-trick seed + three Newton steps
// in explicit fmaf (11 VALU ops, ~1 ulp, instead of the ~28 of IEEE sqrt +
// division); the oracle's rsqrt_B executes the same operations, so results
// agree bit for bit.  (Two steps leave ~5e-6, about 40 ulp.)
__device__ __forceinline__ float rsqrt_d(float x)
{
    float y = __uint_as_float(0x5f375a86u - (__float_as_uint(x) >> 1));
    const float h = 0.5f * x;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float t = y * y;
        t = __builtin_fmaf(-h, t, 1.5f);
        y = y * t;
    }
    return y;
}
// Deterministic square root for x >= 0 (x = +0 gives 0): the same bit-trick
// seed y ~ 1/sqrt(x), two coupled Goldschmidt steps on g ~ sqrt(x) and
// h ~ 1/(2 sqrt(x)), then one Newton residual step g + (x - g^2) h -- 11 VALU,
// within 1 ulp (0.63 measured), no special case for 0.  (The two steps alone
// leave ~5e-6, about 40 ulp: after the discriminant form, the largest single
// part of the fp32-vs-fp64 image difference, DESIGN.md "error budget".)
// The oracle's sqrt_gs_B executes the same operations.
__device__ __forceinline__ float sqrt_gs(float x)
{
    const float y = __uint_as_float(0x5f375a86u - (__float_as_uint(x) >> 1));
    float g = x * y;
    float h = 0.5f * y;
    float r = __builtin_fmaf(-g, h, 0.5f);
    g = __builtin_fmaf(g, r, g);
    h = __builtin_fmaf(h, r, h);
    r = __builtin_fmaf(-g, h, 0.5f);
    g = __builtin_fmaf(g, r, g);
    return __builtin_fmaf(__builtin_fmaf(-g, g, x), h, g);
}
// the scan's square root (ray-sphere discriminant): the same sequence
__device__ __forceinline__ float sqrt_scan(float x) { return sqrt_gs(x); }
// sqrt for any x: 0 for x <= 0 (the clamp as an integer max: negative floats
// are negative integers; one VALU, no canonicalisation)
__device__ __forceinline__ float sqrt_d(float x) { return sqrt_gs(__int_as_float(max(__float_as_int(x), 0))); }
// Deterministic n / d for d > 0 (normal): bit-trick reciprocal seed, two
// Newton steps (error ~2e-4), then one residual correction of the quotient
// (error ~1 ulp) -- 8 VALU instead of the IEEE division's 10 with a
// transcendental.  The oracle's div_B executes the same operations.
__device__ __forceinline__ float div_d(float n, float d)
{
    float r = __uint_as_float(0x7EF311C3u - __float_as_uint(d));
    r = __builtin_fmaf(r, __builtin_fmaf(-d, r, 1.0f), r);
    r = __builtin_fmaf(r, __builtin_fmaf(-d, r, 1.0f), r);
    const float t = n * r;
    return __builtin_fmaf(__builtin_fmaf(-d, t, n), r, t);
}
// vec.cpp:35-38: x * (1 / sqrt(x.x))
__device__ __forceinline__ f3 norm3(f3 a)
{
    float inv = rsqrt_d(dot3(a, a));
    return mk3(a.x * inv, a.y * inv, a.z * inv);
}
__device__ __forceinline__ f3 cross3(f3 a, f3 b)
{
    return mk3(__builtin_fmaf(a.y, b.z, -(a.z * b.y)), __builtin_fmaf(a.z, b.x, -(a.x * b.z)),
               __builtin_fmaf(a.x, b.y, -(a.y * b.x)));
}

// ---- counter RNG: replaces pt::rand_state (random_state.cpp:3-17) ----------
__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t key_hash(uint64_t seed, uint64_t pixel_sub)
{
    return mix64(seed ^ mix64(pixel_sub + 1ull));
}
__device__ __forceinline__ uint32_t sample_state(uint64_t key, uint32_t sample)
{
    uint32_t st = (uint32_t)(mix64(key + ((uint64_t)sample + 1ull) * 0x9E3779B97F4A7C15ull) >> 32);
    return st ? st : 0x6D2B79F5u;
}
// one draw: xorshift32 (13,17,5); its top 24 bits m give U[0,1) = m * 2^-24
__device__ __forceinline__ uint32_t draw_bits(uint32_t &st)
{
    st ^= st << 13;
    st ^= st >> 17;
    st ^= st << 5;
    return st >> 8;
}
__device__ __forceinline__ float draw(uint32_t &st) { return (float)draw_bits(st) * 0x1p-24f; }

// sin/cos of 2*pi*u (replaces libm at main.cpp:55) for u = m * 2^-24, m the
// draw's 24-bit integer: a 128-entry table of cos/sin(2*pi*k/128) (LDS,
// trig_table below) indexed by the top 7 bits, rotated by the remaining angle
// dl = 2*pi*(m mod 2^17)*2^-24 < 2*pi/128 with sin dl = dl (1 - dl^2/6) and
// cos dl = 1 - dl^2/2 + dl^4/24 (truncation < 3e-9).  14 VALU instead of the
// ~30 of a quadrant-split degree-13 polynomial.
constexpr int kTrigBits = 7;
constexpr int kTrigEntries = 1 << kTrigBits;
__device__ __forceinline__ void sincos2pi_tab(uint32_t m, const float2 *tab, float &c, float &s)
{
    const float2 cs = tab[m >> (24 - kTrigBits)];
    const float dl = (float)(m & ((1u << (24 - kTrigBits)) - 1u)) * 0x1.921fb6p-22f;  // 2*pi*2^-24
    const float d2 = dl * dl;
    const float sd = dl * __builtin_fmaf(d2, -0x1.555556p-3f, 1.0f);
    const float cd = __builtin_fmaf(d2, __builtin_fmaf(d2, 0x1.555556p-5f, -0.5f), 1.0f);
    c = __builtin_fmaf(cs.x, cd, -(cs.y * sd));
    s = __builtin_fmaf(cs.y, cd, cs.x * sd);
}

// Two arithmetic modes of the render kernels (template parameter kExact):
//  * exact (PTG_FLAG_EXACT_MATH): the deterministic sequences above -- the
//    image equals the oracle's Mode B (oracle/pt_oracle.c) bit for bit;
//  * fast (the default): the hardware's transcendental instructions,
//    v_sqrt_f32 / v_rsq_f32 / v_rcp_f32 / v_sin_f32 / v_cos_f32, one
//    instruction (issue cost of two plain VALU) instead of 8-14 -- about as
//    accurate (~1 ulp; sin/cos of 2 pi u with v_sin/v_cos taking revolutions),
//    but not reproducible on a CPU, so the image is tied to the reference
//    by the north star's RMSE bar instead (DESIGN.md "arithmetic modes").
// Everything else (draw order, the scan, the BRDFs, the exact u64 sums) is
// the same in both modes, and a frame is deterministic in either: it does
// not depend on sharding, unit sizes or GPU count.
template <bool kExact>
struct Math {
    __device__ static __forceinline__ float rsqrt(float x) { return rsqrt_d(x); }
    __device__ static __forceinline__ float sqrt(float x) { return sqrt_gs(x); }  // x >= 0 (or rejected later)
    __device__ static __forceinline__ float sqrt0(float x) { return sqrt_d(x); }   // 0 for x <= 0
    __device__ static __forceinline__ float div(float n, float d) { return div_d(n, d); }
    __device__ static __forceinline__ void sincos2pi(uint32_t m, const float2 *tab, float &c, float &s)
    {
        sincos2pi_tab(m, tab, c, s);
    }
};
template <>
struct Math<false> {
    __device__ static __forceinline__ float rsqrt(float x) { return __builtin_amdgcn_rsqf(x); }
    __device__ static __forceinline__ float sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
    __device__ static __forceinline__ float sqrt0(float x)
    {
        return __builtin_amdgcn_sqrtf(__int_as_float(max(__float_as_int(x), 0)));
    }
    // n / d for d > 0: hardware reciprocal, one residual correction (~1 ulp)
    __device__ static __forceinline__ float div(float n, float d)
    {
        const float r = __builtin_amdgcn_rcpf(d);
        const float t = n * r;
        return __builtin_fmaf(__builtin_fmaf(-d, t, n), r, t);
    }
    // u = m 2^-24 in [0, 1): v_cos_f32 / v_sin_f32 take revolutions
    __device__ static __forceinline__ void sincos2pi(uint32_t m, const float2 *, float &c, float &s)
    {
        const float u = (float)m * 0x1p-24f;
        c = __builtin_amdgcn_cosf(u);
        s = __builtin_amdgcn_sinf(u);
    }
};
template <bool kExact>
__device__ __forceinline__ f3 norm3m(f3 a)
{
    const float inv = Math<kExact>::rsqrt(dot3(a, a));
    return mk3(a.x * inv, a.y * inv, a.z * inv);
}

// Host: the table, {cos, sin}(2*pi*k/128) rounded to float.  Taylor series in
// double on the first octant (fixed operation order, no libm) and exact
// symmetries elsewhere, so the oracle's copy (oracle/pt_oracle.c:
// trig_table_B) is the same bit for bit on any IEEE-754 host.
inline void trig_table(float *tab /* 2 * kTrigEntries */)
{
    const double pi = 3.14159265358979323846;
    constexpr int kOct = kTrigEntries / 8, kQuad = kTrigEntries / 4;
    double bc[kOct + 1], bs[kOct + 1];
    for (int r = 0; r <= kOct; ++r) {
        const double a = 2.0 * pi / (double)kTrigEntries * (double)r, a2 = a * a;
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
    for (int k = 0; k < kTrigEntries; ++k) {
        const int q = k / kQuad, r = k % kQuad;
        const double c0 = r <= kOct ? bc[r] : bs[kQuad - r], s0 = r <= kOct ? bs[r] : bc[kQuad - r];
        const double c = q == 0 ? c0 : (q == 1 ? -s0 : (q == 2 ? -c0 : s0));
        const double s = q == 0 ? s0 : (q == 1 ? c0 : (q == 2 ? -s0 : -c0));
        tab[2 * k] = (float)c;
        tab[2 * k + 1] = (float)s;
    }
}

// Scene records prepared on the host (ptg_render.hip: prepare_scene).
// Geometry, 32 B per sphere, read with wave-uniform (scalar) loads:
//   g0 = {P.x, P.y, P.z, k1}, g1 = {N.x, N.y, N.z, k2}
//   huge sphere (R >= 1000): P = C + R*n0 on the surface facing the camera,
//     N = n0, k1 = R, k2 = 2R  -> hb = e.d + R (n0.d), c = e.e + 2R (e.n0)
//     (exact algebraic rewrite of |o + t d - C| = R, fp32-safe at R = 1e6)
//   otherwise: P = C, N = 0, k1 = -1 (flag), k2 = -R^2 -> hb = e.d, c = e.e - R^2
// Shading, 64 B per sphere, gathered by hit id:
//   s0 = {C.xyz, prob}, s1 = {emission.xyz, material}, s2 = {color.xyz, 1/R}, s3 = {color/prob .xyz, 0}
struct GeoRec {
    float4 g0, g1;
};
struct ShadeRec {
    float4 s0, s1, s2, s3;
};
// Linear scenes: one 96-B record per sphere in scan order (geometry, then
// shading), plus a sentinel record at index n that stands for "no hit": the
// scan tracks the winner by its record address (the LDS address it already
// holds for the broadcast reads) instead of by an index.
struct LinRec {
    GeoRec g;
    ShadeRec s;
};

}  // namespace ptg
