// ptg_render.hip -- the MI355X render-loop megakernel and its C ABI (include/ptgpu.h).
//
// Replaces the reference's per-pixel hot path (src/main.cpp:214-236 and
// below).  Mapping onto CDNA4:
//  * one lane per (pixel, sub-pixel): lanes 4p..4p+3 of a wave are the
//    2x2 sub-pixels of pixel p (main.cpp:226-232), 16 pixels per wave64;
//  * each lane runs its `samples` paths back to back in ONE flat loop whose
//    iteration is one bounce segment: a lane whose path ends (miss, Russian
//    roulette, depth cap) accumulates it and immediately starts its next
//    sample (per-lane path regeneration), so the wave keeps ~all lanes busy
//    despite the geometric path-length tail;
//  * sphere geometry records are staged in LDS once per workgroup and read
//    with uniform-address (broadcast) LDS loads in the scan (up to 256
//    spheres; measured 1.5 % faster than scalar loads, 7 % faster than
//    software-prefetched scalar loads); larger scenes use wave-uniform scalar
//    loads (s_load into SGPRs) from L2/HBM;
//  * per-wave segment counts via ballot popcount, one atomic per wave;
//  * sub-pixel combine by in-register cross-lane reads, then coalesced
//    192-B stores (three lanes of each pixel write R, G, B).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/ptgpu.h"
#include "bvh_build.hpp"
#include "pt_device.hpp"
#include "ref64.hpp"

using namespace ptg;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg)
{
    g_last_error = msg;
    return code;
}

#define PTG_HIP(call)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return fail(PTG_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));           \
    } while (0)
// inside ptg_context_create, once `ctx` exists: release it on failure
#define PTG_HIP_OR_DESTROY(call)                                                                   \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            ptg_context_destroy(ctx);                                                              \
            return fail(PTG_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));           \
        }                                                                                          \
    } while (0)

#ifndef PTG_BLOCK
#define PTG_BLOCK 256  // linear-scene render kernel workgroup size
#endif
constexpr int kBlock = PTG_BLOCK;
constexpr int kMaxLevels = 4;     // unit levels: head + up to 3 split-tail levels
// samples per sub-pixel in one work unit, at most: a unit's paths are indexed
// it < 64 * chunk <= 2^22, where render_kernel's float-reciprocal divmod_nv is
// exact (fill_launch caps every level's chunk)
constexpr int kMaxChunk = 1 << 16;
constexpr int kTraceBlock = 256;  // parity probe kernel
#ifndef PTG_MAX_LDS_SPHERES
#define PTG_MAX_LDS_SPHERES 64
#endif
// scenes up to 64 spheres keep geometry (32 B) and shading (64 B) records in
// dynamically sized LDS: box_scene needs 17.4 KB + 768 B per workgroup, so 8
// workgroups fit a CU (measured: shading in LDS +1.3 % over geometry-only
// staging, which itself beat scalar loads by 1.5 %)
constexpr int kMaxLdsSpheres = PTG_MAX_LDS_SPHERES;
// nearest-hit rule and scan: <= kLinearMax spheres -> linear scan from LDS with
// fraction comparisons; more -> BVH with the reference's per-candidate
// division rule (DESIGN.md "scene scan"); the oracle switches at the same n
#ifndef PTG_LINEAR_MAX
#define PTG_LINEAR_MAX 64
#endif
constexpr int kLinearMax = PTG_LINEAR_MAX;
static_assert(kLinearMax <= kMaxLdsSpheres, "linear scenes must fit in LDS");
#ifndef PTG_REFILL_BATCH
#define PTG_REFILL_BATCH 40  // measured: 40 beats 32 by 0.35 % (box) / 0.6 % (box_mirror), ties 48-56; 24 is 1.2 % slower
#endif
#ifndef PTG_LEAF_FRAC
#define PTG_LEAF_FRAC 4  // BVH: leaf phase once 4/8 of the walking lanes hold a leaf (re-swept after the walk clean-up: 4 and 3 beat 5 by 0.6 %, 6 +1.5 %)
#endif
#ifndef PTG_LEAF_SPLIT
#define PTG_LEAF_SPLIT 2  // BVH leaf phase: lanes without a leaf test part of another lane's leaf (1: one helper per leaf, 2: up to two)
#endif
#ifndef PTG_LONG_LEAF
#define PTG_LONG_LEAF 5  // BVH leaf phase: leaves of at least this many spheres get helpers first (and a second one; 5 beats 4 by 0.9 %, 3 and 6 worse)
#endif
#ifndef PTG_BVH_UNIT_MULT
#define PTG_BVH_UNIT_MULT 2  // BVH scenes below the split-tail threshold: this many times more work units (8-way C5 shards: 2 beats 1 and 4 by 2-5 %)
#endif
#ifndef PTG_TAIL_CHUNKS
#define PTG_TAIL_CHUNKS 8  // split-tail units per pixel group of the last rows (1: off)
#endif
#ifndef PTG_TAIL_LEVELS
// split-tail levels, each with twice the chunks of the one before (<= 3);
// measured: 2 or 3 levels (chunks 4/8/16) within 1 % of 1 level on the bench
// frame, its 2-8-way shards and box 1024x768
#define PTG_TAIL_LEVELS 1
#endif
#ifndef PTG_TAIL_CHUNKS_MANY
// ... with at least 5 rounds of wave slots (measured: box 1024x768x256 spp
// 2 % faster with 4 than with 8, the 1920x1080 frame the same; 2-8-way shards
// of that frame, 2-4 rounds, keep 8)
#define PTG_TAIL_CHUNKS_MANY 4
#endif
#ifndef PTG_BVH_TAIL_CHUNKS_MANY
// ... and for BVH scenes, whose pixel-split tail units carry every sample of
// their pixels (no HBM accumulation either way): 8 units of 2 pixels per
// group (C5 -0.85 % against 4, A/B 244.4-244.7 vs 246.3-247.1 ms; the box
// scenes keep 4, the cooperative LDS-reduced level)
#define PTG_BVH_TAIL_CHUNKS_MANY 8
#endif
#ifndef PTG_LIN_TAIL_HALF_ROUNDS
#define PTG_LIN_TAIL_HALF_ROUNDS 2  // linear scenes: split-tail rows, in half rounds of the device's wave slots
#endif
#ifndef PTG_BVH_TAIL_HALF_ROUNDS
#define PTG_BVH_TAIL_HALF_ROUNDS 2  // BVH scenes: split-tail rows, in half rounds of the device's wave slots
#endif
#ifndef PTG_TAIL_MIN_HALF_ROUNDS
// linear scenes: split tail from 1.5 rounds of wave slots on (measured with
// tools/shard_sim.py: 2/4/8-way shards of the bench frame 1.6/1.8/1.4 %
// faster than with their samples split into ~96k units)
#define PTG_TAIL_MIN_HALF_ROUNDS 3
#endif
#ifndef PTG_BVH_STACK
#define PTG_BVH_STACK 3  // wide walk: per-lane stack entries before the continuation fallback (3: C5 -0.7 % vs 2, A/B 258.3 vs 260.1 ms)
#endif
#ifndef PTG_BVH_TAIL_MIN_HALF_ROUNDS
#define PTG_BVH_TAIL_MIN_HALF_ROUNDS 6  // BVH scenes: split tail from 3 rounds of wave slots on
#endif
#ifndef PTG_BVH_HEAD_CHUNK
#define PTG_BVH_HEAD_CHUNK 128  // BVH scenes below the split-tail threshold: head rows in chunks of this many samples (0: off; C5 8-way shard 50.4 -> 48.1 ms; 64/96 within 0.5 %, whole pixels +45 %)
#endif
#ifndef PTG_BVH_HEAD_TAIL_HALF_ROUNDS
#define PTG_BVH_HEAD_TAIL_HALF_ROUNDS 1  // ... and the last rows, this many half rounds of wave slots, in the auto chunk (1 beats 2 by 2.5 %, 3 by 5 %)
#endif
#ifndef PTG_BVH_TAIL_CHUNK
#define PTG_BVH_TAIL_CHUNK 0  // ... in chunks of this many samples (0: the auto chunk, 20 at C5 8-way; 10: +0.8 %, 32: +5 %)
#endif
#ifndef PTG_READY_FRAC
#define PTG_READY_FRAC 6  // BVH: stop walking and shade once 6/8 of the active lanes have finished their scan
                          // (measured with octant layouts + SAH: 6 beats 4 by 7 %, 5 and 7 by 1-2 %)
#endif
#ifndef PTG_BLOCK_STATS
#define PTG_BLOCK_STATS 0  // debug builds only: wave-level execution counts of the linear kernel's blocks (ptg_dbg_stats)
#endif
#if PTG_BLOCK_STATS
// [0] main-loop iterations, [1] scans, [2] small-sphere root parts, [3] extra box-mode walls,
// [4] diffuse/dielectric blocks, [5] mirror blocks, [6] refill batches, [7] small-sphere pre-tests
__device__ unsigned long long ptg_dbg_stats[256 * 16];
// PTG_BLOCK_STATS == 3: wave cycles inside the linear kernel's refill batch --
// [0] batches, [1] flush + park of finished paths, [2] camera rays (ray_of),
// [3] begin / store_pre
__device__ unsigned long long ptg_dbg_stats2[256 * 16];
#define PTG_SUB_T(var) const unsigned long long var = clock64()
#define PTG_SUB_ADD(i, v)                                                                              \
    do {                                                                                               \
        if (__lane_id() == __ffsll((long long)__ballot(1)) - 1)                                        \
            atomicAdd(&ptg_dbg_stats2[(blockIdx.x & 255) * 16 + (i)], (v));                           \
    } while (0)
#define PTG_STAT(i)                                                                                    \
    do {                                                                                               \
        if (__lane_id() == __ffsll((long long)__ballot(1)) - 1)                                        \
            atomicAdd(&ptg_dbg_stats[(blockIdx.x & 255) * 16 + (i)], 1ull);                            \
    } while (0)
// BVH kernel, PTG_BLOCK_STATS=2: wave cycles (s_memtime) per phase of the
// main loop in [8..13]: scan starts, node steps, leaf phases, shading,
// refills, loop control
#if PTG_BLOCK_STATS == 2
#define PTG_PHASE(i)                                                                                   \
    do {                                                                                               \
        if constexpr (kBvh) {                                                                          \
            const unsigned long long t_ = clock64();                                                   \
            ph_cyc[i] += t_ - ph_t;                                                                    \
            ph_t = t_;                                                                                 \
        }                                                                                              \
    } while (0)
#else
#define PTG_PHASE(i) ((void)0)
#endif
#else
#define PTG_STAT(i) ((void)0)
#define PTG_PHASE(i) ((void)0)
#endif
#ifndef PTG_UNIT_TRACE
#define PTG_UNIT_TRACE 0  // debug builds only: per-unit start / end wall clock and hardware id (tools/unit_trace.py)
#endif
#if PTG_UNIT_TRACE
constexpr int kTraceUnits = 1 << 19;
// unit u: [3u] start, [3u + 1] end (s_memrealtime, 100 MHz), [3u + 2] XCC id << 32 | HW_ID
__device__ unsigned long long ptg_unit_trace[3 * kTraceUnits];
#define PTG_TRACE_END()                                                                                \
    do {                                                                                               \
        if (__lane_id() == 0 && unit < kTraceUnits) {                                                  \
            ptg_unit_trace[3 * unit] = trace_t0;                                                       \
            ptg_unit_trace[3 * unit + 1] = wall_clock64();                                             \
            ptg_unit_trace[3 * unit + 2] = ((unsigned long long)__builtin_amdgcn_s_getreg(0xF814) << 32) | \
                                           (unsigned long long)__builtin_amdgcn_s_getreg(0xF804);     \
        }                                                                                              \
    } while (0)
#else
#define PTG_TRACE_END() ((void)0)
#endif
#ifndef PTG_WAVE_STATS
#define PTG_WAVE_STATS 0  // debug builds only: count wave-level BVH iterations instead of per-lane tests
#endif
#ifndef PTG_MIN_WAVES_PER_EU
#define PTG_MIN_WAVES_PER_EU 8  // 8 waves per SIMD: <= 64 VGPRs and <= 80 SGPRs (8 blocks of 256 per CU)
#endif
#ifndef PTG_BVH_BLOCK
#define PTG_BVH_BLOCK 64  // BVH render kernel: one wave per workgroup, so a wave slot frees as soon as its unit ends
                          // (units of the 10,000-sphere scene differ widely in length: 64 beats 256 by 10 %, 128 by 6 %)
#endif
template <bool kBvh>
constexpr int kBlockOf = kBvh ? PTG_BVH_BLOCK : kBlock;
constexpr double kBigRadius = 1000.0;
// A sphere takes the anchored form ("huge", DESIGN.md "huge spheres") when its
// radius is >= 1000 or more than 16 times the camera's distance to its
// surface (+1): locally plane-like for the scene, where c = |o - C|^2 - R^2
// cancels in fp32 (simple_scene's R = 100 ground: RMSE vs fp64 1.5e-3 ->
// 3.3e-4).  The oracle's is_huge_B applies the same rule.
inline bool is_huge(const ptg_sphere &sp, const ptg_camera *cam)
{
    if (sp.radius >= kBigRadius)
        return true;
    double d2 = 0.0;
    for (int c = 0; c < 3; ++c)
        d2 += (cam->position[c] - sp.position[c]) * (cam->position[c] - sp.position[c]);
    return sp.radius > 16.0 * (std::fabs(std::sqrt(d2) - sp.radius) + 1.0);
}

struct KArgs {
    const LinRec *lin;      // linear scenes (<= kLinearMax): n records in scan order + sentinel
    const ShadeRec *shade;  // BVH scenes: shading records in scene index order
    int n;
    // linear scenes: records in SCAN order (prepare_scan_order), grouped by
    // kind: [0, end_ax[0]) huge spheres anchored on the x axis, then y, then z
    // ([end_ax[k-1], end_ax[k])), then general huge spheres up to end_big,
    // then the small spheres up to n
    int end_ax[3];
    int end_big;
    int box_walls_out;  // box mode's walls: no ray starts inside any (outside_only); else the fast mode scans generically
    // wall pairs (pair_walls): axis k's group starts with a pair when
    // pairs[k] = 1 -- its wall on the + side, then its wall on the - side; a
    // lane whose origin lies in [pair_lo[k], pair_hi[k]] tests only the wall
    // its direction moves toward (d_k >= 0: the + wall)
    int pairs[3];
    float pair_lo[3], pair_hi[3];
    // box mode (scan_order_of: every axis-anchored wall belongs to the one
    // pair or is the one single wall of its axis, at least one pair, no
    // other huge sphere): per axis the + and - walls' records (-1: none) and
    // tangent planes (+-inf: none); pair_lo/hi bound the room on every
    // axis (+-kFarPlane where open)
    int box_mode;
    int rec_plus[3], rec_minus[3];  // byte offsets of the records
    float plane_plus[3], plane_minus[3];
    // box mode: -m, m > 0 the smallest gap between a wall's tangent plane and
    // its room bound (pair_lo/hi) less a rounding margin: an origin whose
    // plane distances up/um (scene_scan) are all >= -m lies inside the room
    // bounds (room_neg_margin); +inf where there is no such gap
    float room_nmr;
    // scenes with more than kLinearMax spheres: BVH (bvh_build.hpp)
    // the 4-wide tree (bvh_build.hpp wide_bvh): 8 near-plane-first layouts,
    // one per ray-direction octant, interleaved node by node (node j of
    // layout k at node 8 j + k), 4 records of 16 B per node
    const uint4 *bvh_qnodes;
    float q_lo[3], q_scale[3];  // box grid: plane = q_lo + value * q_scale (binary16 values)
    const float4 *bvh_sph;    // leaf-ordered spheres {C, -R^2} (BVH leaves hold only non-huge spheres)
    const int *bvh_id;        // leaf-ordered scene indices
    const GeoRec *big_geo;    // huge spheres, tested linearly
    const int *big_id;
    int n_nodes, n_big;
    const int *bvh_cont;  // per wide node (first record / 4) its continuation (bvh_build.hpp wide_conts)
    const float2 *trig;  // {cos, sin}(2 pi k / 128), staged in LDS (sincos2pi_tab)
    // camera (camera.cpp:32-38): pos, base = llc - pos, X, Y, lens_radius
    float pos_x, pos_y, pos_z;
    float base_x, base_y, base_z;
    float X_x, X_y, X_z;
    float Y_x, Y_y, Y_z;
    float lens;
    // image / sampling
    int W, H, samps, nsub, lanes_per_pixel, pixels_per_wave, waves_per_row;
    int slab_rows, band_rows, shard_rank, shard_count;
    float invW, invH, inv_samps, sub_len, inv_sub2;
    unsigned long long seed;
    int chunk, n_groups, single_chunk;
    // unit levels (fill_launch): level l covers pixel groups [lvl_group[l],
    // lvl_group[l + 1]) in chunks of lvl_chunk[l] samples, chunk-major, as
    // units [lvl_unit[l], lvl_unit[l + 1]); level 0 is the head, levels >= 1
    // the split tail (accumulated, then resolve_kernel from slab row
    // resolve_row0).  lvl_group[n_levels] = n_groups.
    int n_levels;
    int lvl_group[kMaxLevels + 1], lvl_chunk[kMaxLevels];
    // cooperative level (linear kernel's split tail with as many chunks as a
    // workgroup has waves): the waves of one workgroup take the chunks of one
    // pixel group, the last wave to finish adds the others' LDS sums and
    // resolves -- no HBM accumulator (lvl_unit[l] is a multiple of the
    // waves per workgroup)
    int lvl_coop[kMaxLevels];
    // pixel-split level (the BVH kernel's split tail): each pixel group in
    // lvl_psplit[l] units, unit k taking the group's pixels k, k + ps, k + 2ps,
    // ... (interleaved, so the units of a group cost about the same) with
    // every sample (lvl_inwave: resolved in the wave, nothing accumulated in
    // HBM); 1 elsewhere
    int lvl_psplit[kMaxLevels];
    int lvl_inwave[kMaxLevels];  // the level's units hold every sample of their pixels
    int needs_resolve;  // some level accumulates in HBM: resolve_kernel from resolve_row0
    long long lvl_unit[kMaxLevels + 1];
    int resolve_row0;
    int sample_begin, sample_end;  // samples [begin, end) of every sub-pixel in this launch
    int keep_acc;                  // resolve without re-zeroing (progressive previews)
    int count_tests;               // PTG_FLAG_COUNT_TESTS: segments[1..2] += sphere tests, box tests
    int count_nonfinite;           // PTG_FLAG_COUNT_NONFINITE: segments[3] += paths quant() would clip
    int exact_math;                // PTG_FLAG_EXACT_MATH: the kernels' exact arithmetic (pt_device.hpp Math)
    long long n_units;
    float *out;
    unsigned long long *acc;  // slab_rows * W * lanes_per_pixel * 3 exact sums
    unsigned long long *segments;
};

struct Lane {
    int x, y, sx, sy;
    uint64_t key;
};

// camera constants as 4 float4: {pos, lens}, {base, sub_len}, {X, 1/W},
// {Y, 1/H}.  The render kernel stages them in LDS and reads them in each
// refill (camera_ray runs only there): kept in registers for the whole unit
// they took 16 VGPRs, half of them spilled to scratch (measured).
struct CamC {
    float4 p, b, X, Y;
};

__host__ __device__ inline CamC cam_of(const KArgs &A)
{
    return CamC{make_float4(A.pos_x, A.pos_y, A.pos_z, A.lens), make_float4(A.base_x, A.base_y, A.base_z, A.sub_len),
                make_float4(A.X_x, A.X_y, A.X_z, A.invW), make_float4(A.Y_x, A.Y_y, A.Y_z, A.invH)};
}

__device__ __forceinline__ void camera_ray(const CamC &C, const Lane &L, uint32_t sample, uint32_t &st, f3 &o,
                                           f3 &d)
{
    st = sample_state(L.key, sample);
    // main.cpp:186-190: jitter inside the sub-pixel cell
    float u1 = draw(st);
    float u2 = draw(st);
    float xin = __builtin_fmaf(C.b.w, u1, (float)L.x + (float)L.sx * C.b.w);
    float yin = __builtin_fmaf(C.b.w, u2, (float)L.y + (float)L.sy * C.b.w);
    float fs = xin * C.X.w;  // main.cpp:190 x/W as x * (1/W)
    float ft = yin * C.Y.w;
    // camera.cpp:19-30: rejection sample of the unit disk (2 draws per try)
    float px, py;
    do {
        px = __builtin_fmaf(2.0f, draw(st), -1.0f);
        py = __builtin_fmaf(2.0f, draw(st), -1.0f);
    } while (__builtin_fmaf(py, py, px * px) >= 1.0f);
    // camera.cpp:34-37 (offset = rd*s + rd*t, the reference's lens quirk)
    float sst = fs + ft;
    float ox = (px * C.p.w) * sst;
    float oy = (py * C.p.w) * sst;
    o = mk3(C.p.x + ox, C.p.y + oy, C.p.z);
    d = mk3(__builtin_fmaf(C.Y.x, ft, __builtin_fmaf(C.X.x, fs, C.b.x)) - ox,
            __builtin_fmaf(C.Y.y, ft, __builtin_fmaf(C.X.y, fs, C.b.y)) - oy,
            __builtin_fmaf(C.Y.z, ft, __builtin_fmaf(C.X.z, fs, C.b.z)));
}

// main.cpp:30-42 + sphere.cpp:6-30: closest root >= eps over all spheres,
// strict < so the first record in scan order wins exact ties.  Sphere records
// are read from LDS at wave-uniform addresses (broadcast reads).
// Scan order groups the records by kind (host: prepare_scan_order), so every
// loop below runs one straight-line test: huge spheres whose anchor normal is
// a coordinate axis (the box walls) need e_k and d_k instead of two dot
// products (-6 VALU per wall); the oracle's generic form gives the same bits
// (a dot product with +-e_k is exactly +-x_k).
// Roots: with qq = sq + |hb| they are c/-qq (hb >= 0) or c/qq (near) and
// qq/a (far) (hb < 0); the far root matters only when the near one is < eps.
// Roots stay fractions num/den (den > 0): "root < eps" is num < eps*den,
// "nearer" is num*bq < bn*den, and one division per segment turns the winner
// into t.  The test is straight-line code (selects, no per-lane branches):
// the oracle's two culls (hb >= 0 && c >= 0; near root provably not nearer,
// DESIGN.md "scene scan") are exact early-outs that never let a wave skip the
// sqrt in practice, so they are left out here (-15 % frame time, same bits).
constexpr float kCullMargin = 0x1.00001p+0f;  // 1 + 2^-20 (BVH leaf test)
constexpr float kFarPlane = 1e30f;             // box mode: the room bound of an open side
constexpr float kPlaneMargin = 0x1.ffep-1f;    // 1 - 2^-12: box mode's wall skip test

enum : int { kAxX = 0, kAxY = 1, kAxZ = 2, kBig = 3, kSmall = 4, kAxAny = 5, kAxSel = 6, kAxAnyOut = 7 };

#ifndef PTG_UNIT_ROUNDS
#define PTG_UNIT_ROUNDS 2  // linear scenes below the split-tail size: work units for this many rounds of wave slots (2 beats 4 by 5 %, 12 by 12 % on C1)
#endif




__device__ __forceinline__ float comp(f3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

// Returns the winner's record, or the sentinel recs + n (no hit).
// Tests a scan executed (counting kernels only).  BVH scenes: sphere tests
// (huge + leaf spheres) and box tests of the walk; linear scenes: sphere
// tests executed (walls + small spheres, each lane's own -- box mode tests
// one wall for most rays, not all of them) and, of those, the wall tests.
struct ScanCount {
    uint32_t spheres = 0, boxes = 0;
};

template <bool kExact, bool kCount = false>
__device__ __forceinline__ const LinRec *scene_scan(const KArgs &A, const LinRec *recs, f3 o, f3 d, float &tbest,
                                                   ScanCount &cnt)
{
    // the nearest root is kept as a fraction bn/bq (bq > 0); candidates are
    // compared by cross-multiplication, only the winner is divided
    float a = dot3(d, d);
    float bn = kInf, bq = 1.0f;
    // the winner as a byte offset from the sentinel (0: the sentinel, no
    // hit): no multiply by the record size per segment
    constexpr int kRecB = (int)sizeof(LinRec);
    int bi = 0;
    auto ri_of = [&](const LinRec *r) { return ((int)(r - recs) - A.n) * kRecB; };
    // r: the record's index relative to the sentinel
    auto test_geo = [&](const auto r, const float4 g0, const float4 g1, auto kind_tag, const float un = 0.0f,
                        const float vn = 0.0f, const bool valid = true, const int ks = 0) {
        constexpr int kKind = decltype(kind_tag)::value;
        if constexpr (kCount) {
            cnt.spheres += valid ? 1u : 0u;
            if constexpr (kKind != kSmall)
                cnt.boxes += valid ? 1u : 0u;  // (linear scenes: the wall tests)
        }
        // r is wave-uniform, except for a pair's walls / box mode
        f3 e = mk3(o.x - g0.x, o.y - g0.y, o.z - g0.z);
        float ed = dot3(e, d);
        float ee = dot3(e, e);
        float hb, c;
        if constexpr (kKind <= kAxZ) {  // huge sphere anchored on axis k: g0.w = +-R, g1.w = +-2R
            hb = __builtin_fmaf(g0.w, comp(d, kKind), ed);
            c = __builtin_fmaf(g1.w, comp(e, kKind), ee);
        } else if constexpr (kKind == kAxAny || kKind == kAxAnyOut) {
            // the same, for the wall the ray moves toward on a per-lane axis
            // k: g0.w d_k = -R |d_k| = -|g0.w| vn and g1.w e_k = 2R u = |g1.w| un
            // (un: the plane distance numerator, the same subtraction as e_k
            // up to sign), the products' bits are unchanged
            hb = __builtin_fmaf(-__builtin_fabsf(g0.w), vn, ed);
            c = __builtin_fmaf(__builtin_fabsf(g1.w), un, ee);
        } else if constexpr (kKind == kAxSel) {
            // the same as kAxX..kAxZ for a per-lane axis ks (box mode's extra
            // walls).  Exact cull: with hb >= 0 the only candidate root is
            // -c / qq, qq = sq + hb >= hb, so -c < eps hb (or c >= 0) means
            // it fails "num < eps den" below -- the common case here, a lane
            // that just left this convex wall; the wave skips the root when
            // every lane is culled
            hb = __builtin_fmaf(g0.w, comp(d, ks), ed);
            c = __builtin_fmaf(g1.w, comp(e, ks), ee);
            const bool live = valid & !((hb >= 0.0f) & ((c >= 0.0f) | (-c < kEps * hb)));
#if PTG_BLOCK_STATS == 1  // [13] lanes with an extra wall in a pass, [14] of them not culled, [15] passes not skipped
            {
                const unsigned long long mv = __ballot(valid), ml = __ballot(live);
                if (__lane_id() == __ffsll((long long)__ballot(1)) - 1) {
                    unsigned long long *st = &ptg_dbg_stats[(blockIdx.x & 255) * 16];
                    atomicAdd(st + 13, (unsigned long long)__popcll(mv));
                    atomicAdd(st + 14, (unsigned long long)__popcll(ml));
                    atomicAdd(st + 15, ml ? 1ull : 0ull);
                }
            }
#endif
            if (__ballot(live) == 0ull)
                return;
        } else if constexpr (kKind == kBig) {  // general anchored form
            hb = __builtin_fmaf(g0.w, dot3(mk3(g1.x, g1.y, g1.z), d), ed);
            c = __builtin_fmaf(g1.w, dot3(e, mk3(g1.x, g1.y, g1.z)), ee);
        } else {
            hb = ed;
            // fast mode: -R^2 folded into the first product of e.e (one add
            // fewer; another rounding order of the same sum)
            if constexpr (!kExact)
                c = __builtin_fmaf(e.z, e.z, __builtin_fmaf(e.y, e.y, __builtin_fmaf(e.x, e.x, g0.w)));
            else
            c = ee + g0.w;  // g0.w = g1.w = -R^2
        }
        float disc;
        if constexpr (kKind == kSmall) {
            // Lagrange's identity: hb^2 - a c = a R^2 - |e x d|^2.  hb^2 - a c
            // cancels to ~1e-3 relative for a sphere of radius r at distance
            // D >> r (two terms of size a D^2 for a difference of size a r^2);
            // this form keeps the rounding at the scale of a r^2 (DESIGN.md
            // "error budget": box_mirror 1920x1080x1024 RMSE vs fp64 1.9e-3 ->
            // 5e-5).  Huge spheres keep hb^2 - a c: there the anchored hb, c
            // are accurate and a R^2 would be ~1e12.
            const f3 x = cross3(e, d);
            disc = __builtin_fmaf(a, -g0.w, -dot3(x, x));
        } else {
            disc = __builtin_fmaf(hb, hb, -(a * c));
        }
        // a small sphere no lane's ray line meets cannot win: the wave skips
        // the root (exact: "win" below requires disc >= 0)
        if constexpr (kKind == kSmall) {
            PTG_STAT(7);
            if (__ballot(!(disc < 0.0f)) == 0ull)
                return;
            PTG_STAT(2);
        }
        // disc < 0 is rejected below whatever sq is: no clamp
        const float sq = Math<kExact>::sqrt(disc);
        const bool neg = hb < 0.0f;
        // sq - hb (hb < 0) and hb + sq (hb >= 0) are the same IEEE add
        const float qq = sq + __builtin_fabsf(hb);
        float num, den;
        if constexpr (kKind == kAxAnyOut) {
            // a box wall, origin outside it (box_walls_out): the near root
            // c/qq (hb < 0) or nothing (hb >= 0: -c/qq <= 0 fails the eps
            // test; `win` below requires hb < 0).  The far root qq/a -- the
            // wall sphere's other side, ~2R away -- is dropped: the
            // reference takes it only for an origin within eps of the wall
            // moving toward it (a surface touching the wall); the bench
            // frame's quality rows are unchanged up to single roundings
            // (profiles/r04_kernel_ab.txt 13).  The same for the small
            // spheres moved paths there (item 12): not done.
            num = c;
            den = qq;
        } else {
            const bool near_lt = c < kEps * qq;
            num = neg ? (near_lt ? qq : c) : -c;
            den = (neg & near_lt) ? a : qq;
        }
        // one eps test covers all three cases (for the near root it repeats
        // near_lt, which is false there)
        bool win = valid & (!kExact || !(disc < 0.0f)) & !(num < kEps * den) &
                   (num * bq < bn * den);
        if constexpr (kKind == kAxAnyOut)
            win = win & neg;
        bn = win ? num : bn;
        bq = win ? den : bq;
        bi = win ? r : bi;
    };
    auto test_rec = [&](const LinRec *r, auto kind_tag, const float un = 0.0f, const float vn = 0.0f,
                        const bool valid = true, const int ks = 0) {
        test_geo(ri_of(r), r->g.g0, r->g.g1, kind_tag, un, vn, valid, ks);
    };
    auto test = [&](const int i, auto kind_tag) { test_rec(recs + i, kind_tag); };
    // scan order: axis-anchored walls (x, y, z), general huge spheres, small
    // spheres (host: prepare_scan_order)
    int i = 0;
    // a wall pair: the + wall at i, the - wall at i + 1.  A ray whose origin
    // is on the room side of both walls' tangent planes (within a margin) can
    // only hit the wall it moves toward (DESIGN.md "wall pairs"); other lanes
    // (origins outside the room, rare) test both, the one moved toward first
    auto axis_group = [&](auto kind_tag) {
        constexpr int k = decltype(kind_tag)::value;
        if (A.pairs[k]) {
            const bool pos = comp(d, k) >= 0.0f;
            test(pos ? i : i + 1, kind_tag);
            const float ok = comp(o, k);
            const bool outside = !(ok >= A.pair_lo[k]) | !(ok <= A.pair_hi[k]);
            if (__ballot(outside) != 0ull) {
                if (outside)
                    test(pos ? i + 1 : i, kind_tag);
            }
            i += 2;
        }
        for (; i < A.end_ax[k]; ++i)
            test(i, kind_tag);
    };
#ifndef PTG_ASSUME_BOX_MODE
#define PTG_ASSUME_BOX_MODE 0  // analysis builds only (tools/isa_breakdown.py): box mode on, the other scan compiled out
#endif
    // the first small sphere's geometry (the records after the huge ones;
    // always in bounds: the sentinel follows the last record)
    const float4 pf_g0 = recs[A.end_big].g.g0, pf_g1 = recs[A.end_big].g.g1;
    const float4 pf2_g0 = recs[A.end_big + 1].g.g0;  // (in bounds: the sentinel and the wall table follow)
    const float4 pf3_g0 = recs[A.end_big + 2].g.g0;  // (all three read at the start)
    // the small spheres [i, n) (i = n after)
    auto small_spheres = [&](int &i) {
        // three small spheres (the box scenes): straight-line code on one LDS
        // base address (the records at constant offsets), no loop control
        if (A.n - i == 3) {
            // the three records' geometry read at the scan's start (pf_g0,
            // pf2_g0, pf3_g0: their LDS latency behind the walls' tests)
            test_geo(-3 * kRecB, pf_g0, pf_g1, std::integral_constant<int, kSmall>{});
            const float4 a2 = pf3_g0;
            test_geo(-2 * kRecB, pf2_g0, pf_g1, std::integral_constant<int, kSmall>{});
            test_geo(-1 * kRecB, a2, pf_g1, std::integral_constant<int, kSmall>{});
            i = A.n;
        }
        for (; i < A.n; ++i)
            test(i, std::integral_constant<int, kSmall>{});
    };
    if (PTG_ASSUME_BOX_MODE || A.box_mode) {
        // Box mode (DESIGN.md "box mode"): per axis the wall the ray moves
        // toward and the distance u/v to its tangent plane; the wall of the
        // nearest plane is tested first.  Every wall lies beyond its tangent
        // plane, so another wall can only win if its plane is nearer than the
        // winner's root (checked with a 2^-12 margin, far above the roots'
        // rounding): those walls are tested only where that check fails
        // (rare: rays hitting near an edge); a wall the ray moves away from
        // only from beyond its tangent plane (below).
        // wall table after the sentinel: byte offsets of the records of axis
        // k's + wall (2k) and - wall (2k + 1), -1 where missing
        [[maybe_unused]] const int *walls = reinterpret_cast<const int *>(recs + A.n + 1);
        float u[3], v[3];
        bool posk[3];
        float umin = 0.0f;  // the smallest of the six plane distances (room bound check below)
        for (int k = 0; k < 3; ++k) {
            // the uniform plane / record values stay in SGPRs: select values,
            // not kernel-argument addresses (that became per-lane loads)
            float pp = A.plane_plus[k], pm = A.plane_minus[k];
            asm volatile("" : "+s"(pp), "+s"(pm));
            const float dk = comp(d, k);
            const bool pos = dk >= 0.0f;

            // (o - pm) is the same IEEE subtraction as -(pm - o).  A missing
            // wall's plane is at +-inf: u = inf is never the nearest (inf * v
            // is inf or NaN, and NaN compares false) and never needed below
            const float up = pp - comp(o, k), um = comp(o, k) - pm;
            umin = k == 0 ? __builtin_fminf(up, um) : __builtin_fminf(__builtin_fminf(umin, up), um);
            u[k] = pos ? up : um;
            v[k] = __builtin_fabsf(dk);
            posk[k] = pos;
        }
        // the nearest plane, kept as the lane masks n1, n2 (axis 1, axis 2
        // nearer) and the wall table's byte offset of the selected wall (8 k,
        // + 4 for the - wall), not as an axis index re-compared and
        // re-multiplied
        float un = u[0], vn = v[0];
        int offn = posk[0] ? 0 : 4;
        const bool n1 = u[1] * vn < un * v[1];
        un = n1 ? u[1] : un;
        vn = n1 ? v[1] : vn;
        offn = n1 ? (posk[1] ? 8 : 12) : offn;
        const bool n2 = u[2] * vn < un * v[2];
        un = n2 ? u[2] : un;
        vn = n2 ? v[2] : vn;
        offn = n2 ? (posk[2] ? 16 : 20) : offn;
        [[maybe_unused]] auto rec_at = [&](int off) { return reinterpret_cast<const LinRec *>(reinterpret_cast<const char *>(recs) + off); };
        // (fast mode: box mode runs only when no ray starts inside a wall --
        // KArgs::box_walls_out -- so the outside-only roots apply)
        {
            // 32-B geometry entries, entry 2 k + side at 8 offn bytes
            const GeoRec *wg = reinterpret_cast<const GeoRec *>(recs + A.n + 2);
            const GeoRec &g = *reinterpret_cast<const GeoRec *>(reinterpret_cast<const char *>(wg) + 8 * offn);
            const float4 g0 = g.g0, g1 = g.g1;
            test_geo(__float_as_int(g1.x), g0, g1,
                     std::integral_constant<int, !kExact ? kAxAnyOut : kAxAny>{}, un, vn);
        }
        const float bqm = bq * kPlaneMargin;
        // need[k]: wall k is not the selected one and its plane is not safely
        // beyond the winner's root.  Formed as wave masks by the scalar unit
        // from the selection's masks and one compare per plane (as per-lane
        // logic, !n1 and !n2 had been emitted as two more compares).  A
        // missing wall is never needed: its u is +inf, so the compare holds
        // unless bn v is NaN, and the pass below masks a missing wall's test
        // by its NaN geometry -- the same results
        bool need[3];
        const unsigned long long b1 = __ballot(n1), b2 = __ballot(n2);
        const unsigned long long nm[3] = {__ballot(!(bn * v[0] < u[0] * bqm)) & (b1 | b2),
                                          __ballot(!(bn * v[1] < u[1] * bqm)) & (~b1 | b2),
                                          __ballot(!(bn * v[2] < u[2] * bqm)) & ~b2};
        for (int k = 0; k < 3; ++k)
            need[k] = __builtin_amdgcn_inverse_ballot_w64(nm[k]);
        // a wall the ray moves away from can be hit only from beyond its
        // tangent plane (outside the room's bound on that side -- after a
        // bounce off a curved wall far from its tangent point, frequent in
        // box_mirror's mirror tube).  in_room: inside every bound, from the
        // plane distances already formed (host room_neg_margin: it implies
        // the six bound compares; a lane for which only those hold takes the
        // pass below, which checks the exact bounds -- the same tests run)
        const bool in_room = umin >= A.room_nmr;
        if ((__ballot(!in_room) | nm[0] | nm[1] | nm[2]) != 0ull) {
            PTG_STAT(3);
#if PTG_BLOCK_STATS == 3  // debug: wave cycles of the extra-wall block in [15]
            const unsigned long long xw_t0 = clock64();
#endif
#if PTG_BLOCK_STATS == 1  // [9] waves with a lane outside the room, [10] with a lane needing a wall toward; [11], [12] such lanes
            {
                const unsigned long long mo = __ballot(!in_room), mn = __ballot(need[0] | need[1] | need[2]);
                if (__lane_id() == __ffsll((long long)__ballot(1)) - 1) {
                    unsigned long long *st = &ptg_dbg_stats[(blockIdx.x & 255) * 16];
                    atomicAdd(st + 9, mo ? 1ull : 0ull);
                    atomicAdd(st + 10, mn ? 1ull : 0ull);
                    atomicAdd(st + 11, (unsigned long long)__popcll(mo));
                    atomicAdd(st + 12, (unsigned long long)__popcll(mn));
                }
            }
#endif
            // each lane's extra walls in the order of the scan below (toward
            // x, y, z, then away x, y, z): one wall per lane per pass, so a
            // wave pays one test per pass, not one per axis any lane needs
            unsigned m = (need[0] ? 1u : 0u) | (need[1] ? 2u : 0u) | (need[2] ? 4u : 0u);
            if (__ballot(!in_room) != 0ull) {
                for (int k = 0; k < 3; ++k) {
                    float pp = A.plane_plus[k], pm = A.plane_minus[k], lo = A.pair_lo[k], hi = A.pair_hi[k];
                    asm volatile("" : "+s"(pp), "+s"(pm), "+s"(lo), "+s"(hi));
                    const float ok = comp(o, k);
                    const bool pos = comp(d, k) >= 0.0f;
                    // (the wall's existence checked by value as well: a NaN
                    // origin must not select a missing wall's record)
                    // (mask logic, not a select: the select became two exec-mask blocks)
                    const bool away = (pos & !(ok >= lo) & (pm > -HUGE_VALF)) | (!pos & !(ok <= hi) & (pp < HUGE_VALF));
                    m |= away ? 8u << k : 0u;
                }
            }
            while (__ballot(m != 0u) != 0ull) {
                const int j = __builtin_ctz(m | 64u);  // 6: none left
                m &= m - 1u;
                const int k = j < 3 ? j : (j < 6 ? j - 3 : 0);
                const bool toward = j < 3;
                // the wall's geometry entry (axis, side) of the table above:
                // one dependent LDS read; a missing wall's NaN geometry never
                // passes the cull's compares' win
                const int side = (comp(d, k) >= 0.0f) == toward ? 0 : 1;
                const GeoRec &gx = reinterpret_cast<const GeoRec *>(recs + A.n + 2)[2 * k + side];
                const float4 x0 = gx.g0, x1 = gx.g1;
                test_geo(__float_as_int(x1.x), x0, x1, std::integral_constant<int, kAxSel>{}, 0.0f, 0.0f,
                         j < 6, k);
            }
#if PTG_BLOCK_STATS == 3
            {
                const unsigned long long xw_t1 = clock64();
                if (__lane_id() == __ffsll((long long)__ballot(1)) - 1)
                    atomicAdd(&ptg_dbg_stats[(blockIdx.x & 255) * 16 + 15], xw_t1 - xw_t0);
            }
#endif
        }
        i = A.end_ax[2];
    } else {
        axis_group(std::integral_constant<int, kAxX>{});
        axis_group(std::integral_constant<int, kAxY>{});
        axis_group(std::integral_constant<int, kAxZ>{});
    }
    for (; i < A.end_big; ++i)
        test(i, std::integral_constant<int, kBig>{});
    small_spheres(i);
    tbest = bi != 0 ? Math<kExact>::div(bn, bq) : kInf;
    return reinterpret_cast<const LinRec *>(reinterpret_cast<const char *>(recs + A.n) + bi);
}

// Scenes with more than kLinearMax spheres: the huge
// spheres linearly, then a stackless walk of the BVH.  The nearest-hit rule
// here is the reference's own -- every candidate root is divided,
// t = fl(num/den), and the winner is the smallest t, lowest scene index on
// ties (main.cpp:35 strict <, in index order) -- which does not depend on the
// visiting order, so the oracle reproduces it with a linear scan.  Box tests
// only cull: boxes are padded (bvh_build.hpp) and use fast reciprocals.

// Root of one sphere under the reference's rule (the root >= eps nearest to
// the origin, t = fl(num/den)); NaN when rejected or provably not below tb
// (the two exact culls of DESIGN.md "scene scan").  kBig: anchored form with
// g0 = {P0, R}, g1 = {n0, 2R} (huge spheres); else g0 = {C, -R^2}.
constexpr float kReject = __builtin_nanf("");  // every comparison with it is false

// the cull's scaled culling distance: tb * -2 (1 + 2^-20), exact constant
constexpr float kCullScale = -2.0f * kCullMargin;

template <bool kBig, bool kExact>
__device__ __forceinline__ float root_lex(const float4 g0, const float4 g1, const f3 o, const f3 d, const float a,
                                          const float tb, const float tbm)
{
    f3 e = mk3(o.x - g0.x, o.y - g0.y, o.z - g0.z);
    float ed = dot3(e, d);
    float ee = dot3(e, e);
    float hb, c;
    if constexpr (kBig) {
        hb = __builtin_fmaf(g0.w, dot3(mk3(g1.x, g1.y, g1.z), d), ed);
        c = __builtin_fmaf(g1.w, dot3(e, mk3(g1.x, g1.y, g1.z)), ee);
    } else {
        hb = ed;
        c = ee + g0.w;  // g0.w = -R^2
    }
    // the two culls and the discriminant test as one early-out (bitwise: the
    // && chains had been evaluated as nested exec-masked blocks; C5 -1.1 %)
    // The two culls as one compare: behind (hb >= 0, c >= 0) and beyond (hb
    // < 0, near root > tb: c >= 2 |hb| tb (1 + 2^-20); the margin covers the q
    // bound's 3u and the two roundings) are c >= max(hb tbm, 0) with tbm = tb
    // * kCullScale < 0 from the caller (once per change of tb): hb tbm <= 0
    // for hb >= 0 (NaN for hb = 0, tb = inf: fmax gives 0), > 0 for hb < 0.
    // (As two sign-selected compares the choice was materialised: 5 VALU.)
    const bool culled = c >= __builtin_fmaxf(hb * tbm, 0.0f);
    float disc;
    if constexpr (kBig) {
        disc = __builtin_fmaf(hb, hb, -(a * c));
    } else {
        // Lagrange form (scene_scan), limited to hb^2 for an origin outside
        // (c >= 0: exactly disc <= hb^2), which keeps q <= 2|hb|(1 + 3u)
        // and so the cull above exact
        const f3 x = cross3(e, d);
        disc = __builtin_fmaf(a, -g0.w, -dot3(x, x));
        disc = c >= 0.0f ? __builtin_fminf(disc, hb * hb) : disc;
    }
    if (culled | (disc < 0.0f))
        return kReject;
    const float sq = Math<kExact>::sqrt(disc);  // disc >= 0 here
    // the near root c/q (hb < 0, q = sq - hb), else the far root q/a, or -c/qn
    // (hb >= 0, qn = hb + sq) -- as selects (scene_scan's form: sq - hb and
    // hb + sq are the IEEE add sq + |hb|; one eps test covers the three cases),
    // not two divergent branches that a wave with both signs ran one after
    // the other
    const bool neg = hb < 0.0f;
    const float qq = sq + __builtin_fabsf(hb);
    const bool near_lt = c < kEps * qq;
    const float num = neg ? (near_lt ? qq : c) : -c;
    const float den = (neg & near_lt) ? a : qq;
    if (num < kEps * den)
        return kReject;
    if constexpr (kExact)
        return num / den;  // IEEE: the oracle's intersect_B_lex
    else
        return Math<false>::div(num, den);
}

// The BVH scan's winner is its scene index (-1: none).  Ties of t go to the
// lowest scene index (main.cpp:35: strict < in index order), which makes the
// result independent of the visiting order: the oracle's linear scan
// (intersect_B_lex) gives the same bits.
__device__ __forceinline__ void update_lex(const float t, const int sid, float &tb, int &best)
{
    // a NaN t (rejected) fails both compares; (unsigned) -1 orders after every
    // index.  Selects, not a short-circuit && / || (exec-masked blocks)
    const bool win = (t < tb) | ((t == tb) & ((unsigned)sid < (unsigned)best));
    tb = win ? t : tb;
    best = win ? sid : best;
}

// Per-lane BVH scan state.  The render kernel keeps it across iterations of
// its main loop (resumable scan): lanes whose scan ends early shade and start
// their next segment while the wave keeps walking for the long rays -- a
// wave otherwise waits for its slowest ray (measured 93 wave-level node
// steps for 33 per ray on the 10,000-sphere scene).
// global (address space 1) pointers: kernel-argument pointers pinned in
// SGPRs lose their address space, and generic (flat) loads also wait on LDS
template <class T>
using gptr = const T __attribute__((address_space(1))) *;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));  // a compact node record, loadable from gptr

struct BvhTrav {
    int ni;    // binary: next node in depth-first order; wide: see below
    int pend;  // parked leaf (first | count << 24) or -1
    float tb;  // nearest root so far
    int best;  // winner's scene index or -1
    // wide walk: ni = the next position (a wide node's first record + the
    // slot to resume from, >= 0), -1 (walk finished), or -- only while a leaf
    // is parked -- kPopLater (-2: pop the stack after the leaf phase) or a
    // leaf word (parked after the leaf phase).  A two-entry stack (top first, -1 empty)
    // of positions / leaf words still to visit; when it overflows it is
    // cleared and the walk continues, once it runs dry, from the resume
    // position `res` and its continuation chain (bvh_build.hpp wide_conts:
    // everything after it in depth-first order, culled by tb), so any tree
    // depth is walked correctly with three registers.
    int s0, s1;
#if PTG_BVH_STACK >= 3
    int s2;
#endif
    int res;
};

__device__ __forceinline__ bool bvh_done(const KArgs &, const BvhTrav &tr) { return (tr.ni == -1) & (tr.pend < 0); }
__device__ __forceinline__ int bvh_pop(gptr<int> cont, BvhTrav &tr)
{
    const int v = tr.s0;
    tr.s0 = tr.s1;
#if PTG_BVH_STACK >= 3
    tr.s1 = tr.s2;
    tr.s2 = -1;
#else
    tr.s1 = -1;
#endif
    if (v != -1)
        return v;
    const int r = tr.res;  // stack dry: the resume position, then its continuation
    if (r != -1)
        tr.res = cont[r >> 2];
    return r;
}

// Start a scan: the huge spheres (tested linearly, first), then the BVH in
// the layout of the ray's direction octant.
template <bool kCount, bool kExact>
__device__ __forceinline__ void bvh_start(const KArgs &A, f3 o, f3 d, BvhTrav &tr, ScanCount &cnt)
{
    const float a = dot3(d, d);
    tr.tb = kInf;
    tr.best = -1;
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    typedef const __attribute__((address_space(4))) f32x4 *cvec_t;
    typedef const __attribute__((address_space(4))) int *cint_t;
    const cvec_t bgeo = (cvec_t)A.big_geo;  // GeoRec k: words 2 k, 2 k + 1
    const cint_t bid = (cint_t)A.big_id;
    for (int k = 0; k < A.n_big; ++k) {
        const f32x4 v0 = bgeo[2 * k], v1 = bgeo[2 * k + 1];
        const float4 g0 = make_float4(v0.x, v0.y, v0.z, v0.w), g1 = make_float4(v1.x, v1.y, v1.z, v1.w);
        update_lex(root_lex<true, kExact>(g0, g1, o, d, a, tr.tb, tr.tb * kCullScale), bid[k], tr.tb, tr.best);
    }
    if constexpr (kCount)
        cnt.spheres += A.n_big;
    // the wide layouts store each box near-plane first for their octant:
    // all 8 layouts exist
    const unsigned oct = (__float_as_uint(d.x) >> 31) | ((__float_as_uint(d.y) >> 30) & 2u) |
                         ((__float_as_uint(d.z) >> 29) & 4u);
    tr.ni = A.n_nodes > 0 ? (int)(oct << 2) : -1;  // layout k's root: interleaved node k
    tr.s0 = -1;
    tr.s1 = -1;
#if PTG_BVH_STACK >= 3
    tr.s2 = -1;
#endif
    tr.res = -1;
    tr.pend = -1;
}

// Slab-test constants of a ray in the compact nodes' grid units (culling
// only: fast reciprocals, boxes padded and rounded outward):
// t = q * (scale / d) + (lo - o) / d.
struct SlabRay {
    float sx, sy, sz, bx, by, bz;
};
__device__ __forceinline__ SlabRay slab_ray(const KArgs &A, f3 o, f3 d)
{
    const float ix = d.x != 0.0f ? __builtin_amdgcn_rcpf(d.x) : __builtin_copysignf(1e30f, d.x);
    const float iy = d.y != 0.0f ? __builtin_amdgcn_rcpf(d.y) : __builtin_copysignf(1e30f, d.y);
    const float iz = d.z != 0.0f ? __builtin_amdgcn_rcpf(d.z) : __builtin_copysignf(1e30f, d.z);
    SlabRay r;
    r.sx = A.q_scale[0] * ix;
    r.sy = A.q_scale[1] * iy;
    r.sz = A.q_scale[2] * iz;
    r.bx = (A.q_lo[0] - o.x) * ix;
    r.by = (A.q_lo[1] - o.y) * iy;
    r.bz = (A.q_lo[2] - o.z) * iz;
    return r;
}


// Box test of a wide-layout record: binary16 planes on the wide grid, stored
// near-plane first for the ray's octant (bvh_build.hpp WideGrid), each read
// by one v_fma_mix_f32.  No slab margin: the boxes are padded far beyond the
// rounding of the slab times (bvh_build.hpp); tcap keeps the 1e-4 margin
// over the nearest root.
// binary16 halves of a word as float: folded into v_fma_mix_f32 operands.
// (A __builtin_bit_cast of the word to a 2 x _Float16 vector miscompiles
// here: every plane was read from the record's first word.)
__device__ __forceinline__ float lo_half(unsigned w) { return (float)__builtin_bit_cast(_Float16, (unsigned short)(w & 0xFFFFu)); }
__device__ __forceinline__ float hi_half(unsigned w) { return (float)__builtin_bit_cast(_Float16, (unsigned short)(w >> 16)); }
__device__ __forceinline__ bool box_hit_sorted(const u32x4 q, const SlabRay &r, const float tcap)
{
    const float tnx = __builtin_fmaf(lo_half(q.x), r.sx, r.bx);
    const float tny = __builtin_fmaf(hi_half(q.x), r.sy, r.by);
    const float tnz = __builtin_fmaf(lo_half(q.y), r.sz, r.bz);
    const float tfx = __builtin_fmaf(hi_half(q.y), r.sx, r.bx);
    const float tfy = __builtin_fmaf(lo_half(q.z), r.sy, r.by);
    const float tfz = __builtin_fmaf(hi_half(q.z), r.sz, r.bz);
    const float t_in = __builtin_fmaxf(__builtin_fmaxf(tnx, tny), __builtin_fmaxf(tnz, 0.0f));
    // tcap by its own compare: as a min operand it came from outside the
    // node step's block, so the compiler re-canonicalised it (v_max x, x) in
    // every step; the slab times are fresh v_fma_mix results
    const float t_out = __builtin_fminf(__builtin_fminf(tfx, tfy), tfz);
    return !(t_in > t_out) & !(t_in > tcap);
}

// One wide node step at position ni (node + first slot): the node's 4
// records (one 64-B line) in one go.  Slots are in near-first order for the
// layout's octant.  The nearest hit child is visited next -- or, when it is a
// leaf, parked in tr.pend and the second hit visited next; of the hits after
// that one goes on the stack as itself, several as the position of the first
// (the node is re-tested from there, with the culling distance of then).
// With no successor the stack is popped -- at most once per step, and not
// when a leaf was parked: ni = kPopLater then, and the leaf phase pops.
// Selections are branch-free (v_cndmask).
constexpr int kPopLater = -2;
__device__ __forceinline__ int bvh_pop_sel(gptr<int> cont, BvhTrav &tr, const bool need, const int keep);
template <bool kCount>
__device__ __forceinline__ void bvh_node_step(gptr<int> cont, gptr<u32x4> qnodes, const SlabRay &r_in, BvhTrav &tr,
                                              ScanCount &cnt)
{
    const int base = tr.ni & ~3;
    u32x4 q0, q1, q2, q3;
    const SlabRay &r = r_in;
    {
        // a 32-bit byte offset on the uniform base: the load's saddr form
        // (no 64-bit address arithmetic per lane)
        gptr<u32x4> q = (gptr<u32x4>)((const __attribute__((address_space(1))) char *)qnodes + ((unsigned)base << 4));
        q0 = q[0];
        q1 = q[1];
        q2 = q[2];
        q3 = q[3];
    }
    if constexpr (kCount)
        cnt.boxes += 4 - (tr.ni & 3);
    const float tcap = tr.tb * 1.0001f;
    // slots before the walk's position (ni & 3) are not tested again
    const int s = tr.ni & 3;
    const bool h0 = box_hit_sorted(q0, r, tcap) & (s == 0), h1 = box_hit_sorted(q1, r, tcap) & (s <= 1),
               h2 = box_hit_sorted(q2, r, tcap) & (s <= 2), h3 = box_hit_sorted(q3, r, tcap);
    // the words of the first three hits in slot order (-1: none) and the
    // slots of the second and third, shifted in from the last slot: every
    // step is a v_cndmask on its box test's lane mask (the hit mask with
    // lowest-set-bit lookups took 10-16 VALU more per node step: C5 +4.8 %)
    int w1 = h3 ? (int)q3.w : -1, w2 = -1, w3 = -1;
    w2 = h2 ? w1 : w2;
    w1 = h2 ? (int)q2.w : w1;
    w3 = h1 ? w2 : w3;
    w2 = h1 ? w1 : w2;
    w1 = h1 ? (int)q1.w : w1;
    w3 = h0 ? w2 : w3;
    w2 = h0 ? w1 : w2;
    w1 = h0 ? (int)q0.w : w1;
    int i2 = 3, i3 = 3;  // (meaningful only where the hit exists)
    i3 = h1 ? i2 : i3;
    i2 = h1 ? (h2 ? 2 : 3) : i2;
    i3 = h0 ? i2 : i3;
    i2 = h0 ? (h1 ? 1 : h2 ? 2 : 3) : i2;
    const bool leaf = w1 < kPopLater;  // the first hit is a leaf: parked (no hit: w1 = -1)
    int next = leaf ? (w2 != -1 ? w2 : kPopLater) : w1;
    tr.pend = leaf ? (w1 & 0x7FFFFFFF) : tr.pend;
    // the hits left after next: from the second (an inner first hit) or the
    // third (a parked leaf); one goes on the stack as its word, several as
    // the position of the first of them
    // (each select on one lane mask: a select between two conditions was
    // materialised as 5 VALU)
    const bool push = leaf ? w3 != -1 : w2 != -1;
    const int pos = base + (leaf ? i3 : i2);
    const int e = leaf ? ((h0 & h1 & h2 & h3) ? pos : w3) : (w3 != -1 ? pos : w2);
#if PTG_BVH_STACK >= 3
    const bool full = tr.s2 != -1;
    tr.res = (push & full) ? pos : tr.res;
    const int s0 = tr.s0, s1 = tr.s1;
    tr.s0 = push ? (full ? -1 : e) : s0;
    tr.s1 = push ? (full ? -1 : s0) : s1;
    tr.s2 = push ? (full ? -1 : s1) : tr.s2;
#else
    const bool full = tr.s1 != -1;
    tr.res = (push & full) ? pos : tr.res;
    const int s0 = tr.s0;
    tr.s0 = push ? (full ? -1 : e) : s0;
    tr.s1 = push ? (full ? -1 : s0) : tr.s1;
#endif
    if (next == -1) {
        next = bvh_pop(cont, tr);
        if (next < kPopLater) {  // a leaf from the stack
            tr.pend = next & 0x7FFFFFFF;
            next = kPopLater;
        }
    }
    tr.ni = next;
}

// The render kernel's leaf completion (bvh_leaf_done) and its pop, executed
// by every lane of the wave: lanes without a tested leaf (act false) keep
// their state through selects.  As nested divergent branches the update
// merged the traversal state through exec-masked copies (39 v_mov per leaf
// phase in the ISA); same values, C5 -0.5 %.
//
// Pop where need (else return keep): the stack top, or once it runs dry the
// resume position and its continuation -- the one load stays behind a branch
// (rare: the two-entry stack overflowed earlier).
__device__ __forceinline__ int bvh_pop_sel(gptr<int> cont, BvhTrav &tr, const bool need, const int keep)
{
    const int v = tr.s0, r = tr.res;
    const bool dry = v == -1;
    int nres = r;
    if (need & dry & (r != -1))
        nres = cont[r >> 2];
    tr.s0 = need ? tr.s1 : v;
#if PTG_BVH_STACK >= 3
    tr.s1 = need ? tr.s2 : tr.s1;
    tr.s2 = need ? -1 : tr.s2;
#else
    tr.s1 = need ? -1 : tr.s1;
#endif
    tr.res = nres;
    return need ? (dry ? r : v) : keep;
}

// bvh_leaf_done for the lanes whose parked leaf was tested (act)
__device__ __forceinline__ void bvh_leaf_done_sel(gptr<int> cont, BvhTrav &tr, const bool act)
{
    tr.pend = act ? -1 : tr.pend;
    int next = bvh_pop_sel(cont, tr, act & (tr.ni == kPopLater), tr.ni);
    const bool lf = act & (next < kPopLater);  // a leaf word (popped, or waiting in ni)
    tr.pend = lf ? (next & 0x7FFFFFFF) : tr.pend;
    next = lf ? kPopLater : next;
    tr.ni = act ? next : tr.ni;
}

// Spheres [f, f + cnt) of the leaf order against one ray: compact records
// {C, -R^2}; (tb, best) updated by the lex rule.
template <bool kCount, bool kExact>
__device__ __forceinline__ void leaf_spheres(const KArgs &A, int f, int cnt, f3 o, f3 d, float &tb, int &best,
                                             ScanCount &sc)
{
    const float a = dot3(d, d);
    if constexpr (kCount)
        sc.spheres += cnt;
    // 32-bit byte offsets on the uniform bases (saddr loads)
    const char *sph = (const char *)A.bvh_sph;
    const char *ids = (const char *)A.bvh_id;
    float tbm = tb * kCullScale;
    for (int j = 0; j < cnt; ++j) {
        const unsigned off = (unsigned)(f + j) << 4;
        const float4 rec = *(const float4 *)(sph + off);
        const float t = root_lex<false, kExact>(rec, float4{}, o, d, a, tb, tbm);
        if (t <= tb) {  // the scene index is read only for a candidate that wins or ties
            update_lex(t, *(const int *)(ids + (off >> 2)), tb, best);
            tbm = tb * kCullScale;
        }
    }
}

// After the parked leaf's spheres: wide walk -- a leaf word waiting in tr.ni
// is parked next, or the pop deferred by the node step happens.
__device__ __forceinline__ void bvh_leaf_done(gptr<int> cont, BvhTrav &tr)
{
    tr.pend = -1;
    if (tr.ni < -1) {  // kPopLater, or the leaf the node step moved to after parking one
        int next = tr.ni == kPopLater ? bvh_pop(cont, tr) : tr.ni;
        if (next < kPopLater) {  // a leaf: parked for the next leaf phase
            tr.pend = next & 0x7FFFFFFF;
            next = kPopLater;
        }
        tr.ni = next;
    }
}

// The parked leaf's spheres, all by this lane.
template <bool kCount, bool kExact>
__device__ __forceinline__ void bvh_leaf(const KArgs &A, gptr<int> cont, f3 o, f3 d, BvhTrav &tr, ScanCount &cnt)
{
    const int first = tr.pend & 0xFFFFFF, nl = tr.pend >> 24;
    const int take = nl;
    leaf_spheres<kCount, kExact>(A, first, take, o, d, tr.tb, tr.best, cnt);
    if (take < nl) {
        tr.pend = (first + take) | ((nl - take) << 24);
        return;
    }
    bvh_leaf_done(cont, tr);
}

// Leaf phase with helpers (PTG_LEAF_SPLIT; called by the whole wave): lanes
// with no leaf to test are assigned, by rank, to lanes holding a leaf of >= 2
// spheres -- one helper per such leaf, longest leaves (>= PTG_LONG_LEAF spheres: they set
// the wave's loop length) first, then a second helper per long leaf while
// idle lanes remain.  A helper tests its part of the leaf with the owner's
// ray and culling distance (ds_bpermute) and the owner merges the helpers'
// nearest roots by the same lex rule -- order-independent, so the result is
// the one-lane result bit for bit.  pair: 2 x 64 bytes of LDS (owner lane by
// owner rank, helper lane by helper rank).
template <bool kCount, bool kExact>
__device__ __forceinline__ void bvh_leaf_split(const KArgs &A, gptr<int> cont, f3 o, f3 d, bool has,
                                               unsigned long long mhas, BvhTrav &tr, ScanCount &cnt,
                                               uint8_t (*pair)[64])
{
    const int lane = (int)__lane_id();
    const int nl = has ? (tr.pend >> 24) : 0;
    const bool own = nl >= 2, hlp = !has;
    auto rank = [](unsigned long long m) {
        return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
    };
    const bool longl = nl >= PTG_LONG_LEAF;
    // (mhas = ballot(has), the whole wave active: ballots of single compares only)
    const unsigned long long ml = __ballot(longl), ms = __ballot(own) & ~ml, mh = ~mhas;
    const int nlong = (int)__popcll(ml), nown = nlong + (int)__popcll(ms), nhelp = (int)__popcll(mh);
    const int np1 = min(nown, nhelp);  // owners (by rank) with a first helper
#if PTG_LEAF_SPLIT >= 2
    const int np2 = max(0, min(nlong, nhelp - nown));  // long-leaf owners with a second helper
#else
    const int np2 = 0;
#endif
    const int ro = longl ? rank(ml) : nlong + rank(ms);
    const int rh = rank(mh);
    const bool po = own & (ro < np1), ph = hlp & (rh < np1 + np2);
    if (po)
        pair[0][ro] = (uint8_t)lane;
    if (ph)
        pair[1][rh] = (uint8_t)lane;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int orank = rh < np1 ? rh : rh - np1;  // a helper's owner, and which helper it is
    const int part = rh < np1 ? 1 : 2;
    const int partner = po ? (int)pair[1][ro] : ph ? (int)pair[0][orank] : lane;
    const int partner2 = (po & (ro < np2)) ? (int)pair[1][np1 + ro] : lane;
    auto bpf = [](int who, float v) {
        return __int_as_float(__builtin_amdgcn_ds_bpermute(who << 2, __float_as_int(v)));
    };
    auto bpi = [](int who, int v) { return __builtin_amdgcn_ds_bpermute(who << 2, v); };
    // helpers take the owner's ray, culling distance and leaf
    const f3 po3 = mk3(bpf(partner, o.x), bpf(partner, o.y), bpf(partner, o.z));
    const f3 pd3 = mk3(bpf(partner, d.x), bpf(partner, d.y), bpf(partner, d.z));
    const float ptb = bpf(partner, tr.tb);
    const int ppend = bpi(partner, tr.pend);
    const f3 ro3 = ph ? po3 : o, rd3 = ph ? pd3 : d;
    const int pendl = ph ? ppend : tr.pend;
    const int first = pendl & 0xFFFFFF, nll = pendl >> 24;
    // the leaf's parts: one helper -> [0, ceil(n/2)), [ceil(n/2), n); two
    // helpers -> [0, n/3), [n/3, 2n/3), [2n/3, n) (n <= 12: x/3 = x*11 >> 5)
    const int k = ph ? 1 + (orank < np2) : po ? 1 + (ro < np2) : 0;
    const int b1 = k == 2 ? (nll * 11) >> 5 : (nll + 1) >> 1;
    const int b2 = k == 2 ? (2 * nll * 11) >> 5 : nll;
    const int lo = !ph ? 0 : part == 1 ? b1 : b2;
    const int hi = !ph ? (po ? b1 : (has ? nll : 0)) : part == 1 ? b2 : nll;
    const int f = first + lo, c = hi - lo;
    float tb = ph ? ptb : tr.tb;
    int best = ph ? -1 : tr.best;
#if PTG_WAVE_STATS == 1  // debug: the wave's loop length
    {
        int mx = c;
        for (int off = 32; off > 0; off >>= 1)
            mx = max(mx, __shfl_xor(mx, off, 64));
        const bool first_lane = lane == __ffsll((long long)__ballot(1)) - 1;
        cnt.spheres += first_lane ? (uint32_t)mx : 0u;
    }
#endif
    leaf_spheres<kCount && !PTG_WAVE_STATS, kExact>(A, f, c, ro3, rd3, tb, best, cnt);
    // owners merge their helpers' nearest roots
    const float htb = bpf(partner, tb), htb2 = bpf(partner2, tb);
    const int hbest = bpi(partner, best), hbest2 = bpi(partner2, best);
    if (po) {
        update_lex(htb, hbest, tb, best);
        update_lex(htb2, hbest2, tb, best);  // partner2 = lane without a second helper: a no-op
    }
    tr.tb = has ? tb : tr.tb;
    tr.best = has ? best : tr.best;
    bvh_leaf_done_sel(cont, tr, has);
}

// Whole scan of one ray (parity probe kernel): walk, testing each parked leaf
// at once.
template <bool kCount, bool kExact>
__device__ __forceinline__ int scene_scan_bvh(const KArgs &A, f3 o, f3 d, float &tbest, ScanCount &cnt)
{
    BvhTrav tr;
    bvh_start<kCount, kExact>(A, o, d, tr, cnt);
    const SlabRay sr = slab_ray(A, o, d);
    while (!bvh_done(A, tr)) {
        if (tr.pend >= 0)
            bvh_leaf<kCount, kExact>(A, (gptr<int>)A.bvh_cont, o, d, tr, cnt);
        else
            bvh_node_step<kCount>((gptr<int>)A.bvh_cont, (gptr<u32x4>)A.bvh_qnodes, sr, tr, cnt);
    }
    tbest = tr.tb;
    return tr.best;
}

// Per-lane state machine: one call = one bounce segment of radiance()
// (main.cpp:111-155).  Returns true when the path has ended; E then holds
// its radiance.
// shade(): everything after the scene scan -- sky on a miss, else hit
// record, emission, Russian roulette, BRDF sampling of the next ray.
template <bool kExact>
__device__ __forceinline__ bool shade(const ShadeRec *hit, float t, const float2 *trig, f3 &o, f3 &d, f3 &T, f3 &E,
                                      int &depth, uint32_t &st);

template <bool kBvh, bool kExact, bool kCount = false>
__device__ __forceinline__ bool segment(const KArgs &A, const LinRec *recs, const float2 *trig, f3 &o, f3 &d, f3 &T,
                                        f3 &E, int &depth, uint32_t &st, ScanCount &cnt)
{
    float t;
    const ShadeRec *hit;
    if constexpr (kBvh) {
        const int id = scene_scan_bvh<kCount, kExact>(A, o, d, t, cnt);
        hit = id >= 0 ? A.shade + id : nullptr;
    } else {
        const LinRec *w = scene_scan<kExact, kCount>(A, recs, o, d, t, cnt);
        hit = w != recs + A.n ? &w->s : nullptr;
    }
    return shade<kExact>(hit, t, trig, o, d, T, E, depth, st);
}

template <bool kExact>
__device__ __forceinline__ bool shade(const ShadeRec *hit, float t, const float2 *trig, f3 &o, f3 &d, f3 &T, f3 &E,
                                      int &depth, uint32_t &st)
{
    // the segment count first, for every lane: a sky lane's path ends here
    // (its depth is reset by the refill), so the value is only read below --
    // no per-branch copy of the loop-carried register
    depth += 1;
    if (!hit) {  // main.cpp:115-120: sky
        f3 ud = norm3m<kExact>(d);
        float tt = 0.5f * (ud.y + 1.0f);
        float it = 1.0f - tt;
        E = mk3(__builtin_fmaf(T.x, __builtin_fmaf(tt, 0.5f, it), E.x),
                __builtin_fmaf(T.y, __builtin_fmaf(tt, 0.7f, it), E.y),
                __builtin_fmaf(T.z, __builtin_fmaf(tt, 1.0f, it), E.z));
        return true;
    }
    const ShadeRec &S = *hit;
    float4 s0 = S.s0;
    const float4 s1 = S.s1;
    // hit_record.cpp:3-12
    f3 p = mk3(__builtin_fmaf(d.x, t, o.x), __builtin_fmaf(d.y, t, o.y), __builtin_fmaf(d.z, t, o.z));
    // hit_record.cpp:6 (p - C).norm() as (p - C) * (1/R): p lies on the sphere
    const bool rr = depth > kRRThreshold + 1;  // (the depth before this segment's count)
    const float4 cc = *(rr ? &S.s3 : &S.s2);  // (prepare_scene: 1/R in s2.w and s3.w)
    const float invR = cc.w;
    bool front;
    f3 on, nn;
    [[maybe_unused]] float kn = 0.0f;  // fast mode: nn.d
    if (!kExact) {
        const f3 pc = mk3(p.x - s0.x, p.y - s0.y, p.z - s0.z);
        const float sd = dot3(pc, d);
        front = sd < 0.0f;
        const float ks = front ? invR : -invR;
        nn = mk3(pc.x * ks, pc.y * ks, pc.z * ks);
        kn = sd * ks;
        on = nn;  // (unused: the mirror reflects on nn)
    } else {
        on = mk3((p.x - s0.x) * invR, (p.y - s0.y) * invR, (p.z - s0.z) * invR);
        front = dot3(on, d) < 0.0f;
        nn = front ? on : mk3(-on.x, -on.y, -on.z);
    }
    // main.cpp:126
    E = mk3(__builtin_fmaf(T.x, s1.x, E.x), __builtin_fmaf(T.y, s1.y, E.y), __builtin_fmaf(T.z, s1.z, E.z));
    // main.cpp:128-139: Russian roulette after depth 4 (the colour row read
    // above by address)
    // Russian roulette without an early return: the roulette's draw advances the state of the
    // rr lanes only (a select), and a killed lane runs on with its materials
    // masked -- its next ray and state are discarded (the early return's
    // merge had cost state copies and exec-mask blocks)
    uint32_t st_rr = st;
    const uint32_t m_rr = draw_bits(st_rr);  // u = m_rr 2^-24; s0.w holds ceil(p 2^24) (prepare_scene)
    st = rr ? st_rr : st;
    const bool killed = rr & !(m_rr < __float_as_uint(s0.w));
    T = mk3(T.x * cc.x, T.y * cc.y, T.z * cc.z);
    // BRDF samplers (main.cpp:44-97).  Diffuse and dielectric lanes share the
    // three expensive ops (one rsqrt, two sqrt) through selects, so a wave
    // holding both materials issues them once; every lane's arithmetic is the
    // same as the per-material code (oracle sample_B).
    const int mat = __float_as_int(s1.w);
    const bool isD = !killed & (mat == PTG_DIFFUSE);
    const bool isG = !killed & (mat == PTG_DIELECTRIC);
    bool spec = !killed & (mat == PTG_SPECULAR);
    // every lane's first BRDF draw taken once, here: the diffuse phi, the
    // dielectric's Fresnel draw -- or, where it cannot refract, its
    // reflection's draw -- and the mirror's draw (main.cpp:46, :89, :62).
    // A dielectric lane reflected by its Fresnel draw takes the reflection's
    // draw below (fres).  Each lane's draws keep their order and count;
    // killed lanes advance a state their ended path no longer reads.
    const uint32_t m1 = draw_bits(st);
    [[maybe_unused]] bool fres = false;
    // its value u = m1 2^-24, converted once for the diffuse phi (fast
    // mode: v_sin / v_cos take revolutions) and the Fresnel compare
    const float u1 = (float)m1 * 0x1p-24f;
    f3 nd = d;  // every lane sets it below (mirror lanes in the spec block)
    // a wave with only mirror lanes skips the diffuse/dielectric work
    // (wave-uniform, exact: those lanes' values are all overwritten)
    // (the active lanes less the mirror lanes' mask, which the spec compare
    // above already formed: a ballot of isD | isG was materialised as
    // v_cndmask + v_cmp, one of mat != PTG_SPECULAR as another compare;
    // killed lanes of those materials run the block for nothing, their
    // values unused)
    if ((__ballot(1) & ~__ballot(mat == PTG_SPECULAR)) != 0ull)
    {
        PTG_STAT(4);
#if PTG_BLOCK_STATS == 3  // debug: wave cycles of the diffuse/dielectric block in [14]
        const unsigned long long dg_t0 = clock64();
#endif
        {
        // read only where isD (the ?: operands and the isD branch below):
        // no initial values to set for the other lanes
        float cp, sp, ra;
        if (isD) {  // main.cpp:46-47: phi = 2 pi u, r = u
            const uint32_t m_phi = m1;
            ra = draw(st);
            if constexpr (!kExact) {
                cp = __builtin_amdgcn_cosf(u1);  // Math<false>::sincos2pi of m1
                sp = __builtin_amdgcn_sinf(u1);
            } else
            Math<kExact>::sincos2pi(m_phi, trig, cp, sp);
        }
        // op1: diffuse -> u = norm((|w.x| > 0.1 ? y : x) x w) (main.cpp:52); dielectric -> norm(d) (main.cpp:75)
        f3 uu = __builtin_fabsf(nn.x) > 0.1f ? mk3(nn.z, 0.0f, -nn.x) : mk3(0.0f, -nn.z, nn.y);
        f3 v1 = isD ? uu : d;
        const float r1 = Math<kExact>::rsqrt(dot3(v1, v1));
        v1 = mk3(v1.x * r1, v1.y * r1, v1.z * r1);
        const float x0 = -dot3(v1, nn);
        // fast mode: one v_min_f32 (differs from the select only for NaN)
        const float cthG = kExact ? (1.0f < x0 ? 1.0f : x0) : __builtin_fminf(1.0f, x0);  // main.cpp:77
        // op2: diffuse -> sin theta = sqrt(r); dielectric -> sin theta = sqrt(1 - cos^2)
        // (fast mode: the argument is >= 0 on every lane that reads s2 --
        // ra >= 0, and 0 < x0 <= 1 + rounding on a dielectric lane (nn faces
        // the ray), so cthG <= 1 and 1 - cthG^2 >= 0 -- so sqrt0's clamp of
        // negative inputs is left out)
        const float s2 = kExact ? Math<kExact>::sqrt0(isD ? ra : __builtin_fmaf(-cthG, cthG, 1.0f))
                                : Math<kExact>::sqrt(isD ? ra : __builtin_fmaf(-cthG, cthG, 1.0f));
        const float ratio = front ? 0.5f : 2.0f;  // main.cpp:72
        if (isG) {
            bool reflect = ratio * s2 > 1.0f;  // cannot refract: no Fresnel draw (main.cpp:89)
            if (!reflect) {
                const float r0 = 0x1.c71c74p-4f;  // ((1-ratio)/(1+ratio))^2, equal for ratio 0.5 and 2
                float xm = 1.0f - cthG;
                float x2 = xm * xm;
                float x5 = (x2 * x2) * xm;
                float R = __builtin_fmaf(1.0f - r0, x5, r0);
                reflect = R > u1;
                fres = true;
                {  // the reflection's draw right after the Fresnel draw that chose it
                    uint32_t st2 = st;
                    (void)draw_bits(st2);
                    st = reflect ? st2 : st;
                }
            }
            spec = reflect;
        }
        // op3: diffuse -> cos theta = sqrt(1 - r); dielectric -> |r_out_parallel| (main.cpp:94)
        const f3 perp = mk3(__builtin_fmaf(nn.x, cthG, v1.x) * ratio, __builtin_fmaf(nn.y, cthG, v1.y) * ratio,
                            __builtin_fmaf(nn.z, cthG, v1.z) * ratio);
        const float s3 = Math<kExact>::sqrt(isD ? 1.0f - ra : __builtin_fabsf(1.0f - dot3(perp, perp)));  // both >= 0
        if (isD) {  // main.cpp:53-55 (unit by construction, not re-normalised)
            f3 vv = cross3(nn, v1);
            float cs = cp * s2, ss = sp * s2;
            nd = mk3(__builtin_fmaf(nn.x, s3, __builtin_fmaf(vv.x, ss, v1.x * cs)),
                     __builtin_fmaf(nn.y, s3, __builtin_fmaf(vv.y, ss, v1.y * cs)),
                     __builtin_fmaf(nn.z, s3, __builtin_fmaf(vv.z, ss, v1.z * cs)));
        } else
        {  // refraction, main.cpp:93-96
            nd = mk3(__builtin_fmaf(nn.x, -s3, perp.x), __builtin_fmaf(nn.y, -s3, perp.y),
                     __builtin_fmaf(nn.z, -s3, perp.z));
        }
        }
#if PTG_BLOCK_STATS == 3
        {
            const unsigned long long dg_t1 = clock64();
            if (__lane_id() == __ffsll((long long)__ballot(1)) - 1)
                atomicAdd(&ptg_dbg_stats[(blockIdx.x & 255) * 16 + 14], dg_t1 - dg_t0);
        }
#endif
    }
    if (spec) {  // main.cpp:60-67 (fuzz draw consumed, multiplied by 0)
        PTG_STAT(5);
        // (fast mode: on the facing normal nn = +-on, its dot kn)
        float k = !kExact ? kn : dot3(on, d);
        k = k + k;
        // (the reflection's draw after a Fresnel draw: taken in the Fresnel block)
        const f3 rn = !kExact ? nn : on;
        nd = mk3(__builtin_fmaf(-k, rn.x, d.x), __builtin_fmaf(-k, rn.y, d.y), __builtin_fmaf(-k, rn.z, d.z));
    }
    o = p;
    d = nd;
    return killed | (depth >= kDepthLimit);
}

// Slab row -> image (output) row for the band shard.
__device__ __forceinline__ int out_row_of(const KArgs &A, int slab_row)
{
    int band = slab_row / A.band_rows;
    return (band * A.shard_count + A.shard_rank) * A.band_rows + (slab_row - band * A.band_rows);
}

// Exact per-path quantisation (include/ptgpu.h "Sample accumulation").
// trunc(c * 2^32) for c in [0, 2^30] without double arithmetic: integer part
// and fraction * 2^32 are both exact in fp32, so this equals the oracle's
// (uint64_t)((double)c * 0x1p32) bit for bit.
// quant() is exact for c in [0, 2^30]; NaN and negative values become 0 and
// larger ones 2^30 -- the counting kernel reports such paths
// (PTG_FLAG_COUNT_NONFINITE), none are expected
__device__ __forceinline__ bool in_quant_range(float c) { return c >= 0.0f && c <= 0x1p30f; }
__device__ __forceinline__ unsigned long long quant(float c)
{
    if (!(c >= 0.0f))
        return 0ull;
    if (c > 0x1p30f)
        c = 0x1p30f;
    float ip = __builtin_truncf(c);
    uint32_t hi = (uint32_t)ip;
    uint32_t lo = (uint32_t)((c - ip) * 0x1p32f);
    return ((unsigned long long)hi << 32) | lo;
}

// One work unit per wave: a pixel group (pixels_per_wave pixels of one slab
// row, all their sub-pixels = up to 64 "slots") x one chunk of samples.
// The unit's nv*cnt paths form a pool: every lane starts one path, and a lane
// whose path ends takes the next unstarted path of the pool (ballot + rank),
// so all lanes stay busy until the pool is empty.  Path radiance is
// accumulated exactly (u64) per slot in LDS and added to the global
// accumulator once per unit.
template <bool kCount, bool kBvh, bool kExact>
__global__ __launch_bounds__(kBlockOf<kBvh>, PTG_MIN_WAVES_PER_EU) void render_kernel(KArgs A)
{
    constexpr int kWaves = kBlockOf<kBvh> / 64;
    __shared__ unsigned long long lds_acc[kWaves][64 * 3];
    __shared__ unsigned long long lds_key[kWaves][64];
    __shared__ uint32_t lds_pix[kWaves][64];  // slot -> x | sx << 20 | sy << 26
    // sphere records staged once per workgroup in LDS (uniform-address
    // ds_read_b128 broadcasts in the scan, by-id gathers at hits); larger
    // scenes read geometry with wave-uniform scalar loads from L2/HBM instead
    constexpr bool kLdsGeo = !kBvh;  // linear scenes (<= kMaxLdsSpheres) live in LDS
    // dynamic LDS: n geometry records then n shading records (96 B/sphere),
    // sized at launch so small scenes keep 8 workgroups per CU
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn_lds[];
    LinRec *lds_lin = reinterpret_cast<LinRec *>(dyn_lds);
    const LinRec *recs = A.lin;
    // linear kernel: the sin/cos table in LDS; the BVH kernel (latency bound
    // on its node loads) reads it from global memory (L1): measured the same
    const float2 *trig = A.trig;
    if constexpr (kLdsGeo) {
        if constexpr (kExact) {  // (the fast mode's v_sin/v_cos need no table)
            __shared__ float2 lds_trig[kTrigEntries];
            for (int i = threadIdx.x; i < kTrigEntries; i += kBlock)
                lds_trig[i] = A.trig[i];
            trig = lds_trig;
        }
        for (int i = threadIdx.x; i <= A.n + 1 + 2; i += kBlock)  // n records + the sentinel + the wall table(s)
            lds_lin[i] = A.lin[i];
        recs = lds_lin;
    }
    __shared__ float4 lds_cam[4];
    __shared__ int lds_coop_done;  // cooperative levels: waves of the workgroup finished
    if (threadIdx.x == 0) {
        lds_coop_done = 0;
        const CamC c = cam_of(A);
        lds_cam[0] = c.p;
        lds_cam[1] = c.b;
        lds_cam[2] = c.X;
        lds_cam[3] = c.Y;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    // wave-uniform by construction; readfirstlane lets the compiler keep all
    // per-unit bookkeeping in SGPRs
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const long long unit = (long long)blockIdx.x * kWaves + wv;
    if (unit >= A.n_units)
        return;  // whole wave
    // unit -> level (wave-uniform: a few scalar compares) -> pixel group and
    // sample chunk; chunk-major within a level (neighbours are different
    // pixel groups)
    int lv = 0;
    while (lv + 1 < A.n_levels && unit >= A.lvl_unit[lv + 1])
        ++lv;
    const long long t = unit - A.lvl_unit[lv];
    const int nlg = A.lvl_group[lv + 1] - A.lvl_group[lv];
    const bool coop = A.lvl_coop[lv] != 0;  // wave wv of the workgroup takes chunk wv of one pixel group
    const int ps = A.lvl_psplit[lv];        // units per pixel group (pixel-split level) or 1
    const long long nlu = (long long)nlg * ps;  // units per sample chunk
    // part-major like chunk-major: neighbouring units are different pixel groups
    const long long tg = coop ? t / kWaves : t % nlu;
    const int group = A.lvl_group[lv] + (int)(coop ? tg : tg % nlg);
    const int part = coop ? 0 : (int)(tg / nlg);
    const int len = A.lvl_chunk[lv];
    const int s0 = A.sample_begin + (int)(coop ? t % kWaves : t / nlu) * len;
    if (s0 >= A.sample_end)
        return;  // whole wave: alignment padding before a cooperative level
#if PTG_UNIT_TRACE
    const unsigned long long trace_t0 = wall_clock64();
#endif
    // the unit holds every sample of its pixels: resolve in the wave
    const bool in_wave = A.lvl_inwave[lv] != 0;
    const int slab_row = group / A.waves_per_row;
    const int xblk = group - slab_row * A.waves_per_row;
    const int r = out_row_of(A, slab_row);
    const int y = A.H - 1 - r;  // main.cpp:181: y = 0 is the bottom row
    // the unit's pixels: x0, x0 + ps, ... (ps = 1: a contiguous group)
    const int x0 = xblk * A.pixels_per_wave + part;
    int npix = (A.pixels_per_wave - part + ps - 1) / ps;
    const int left = A.W - x0 > 0 ? (A.W - x0 + ps - 1) / ps : 0;
    npix = npix < left ? npix : left;
    const int nv = r < A.H ? npix * A.lanes_per_pixel : 0;  // valid slots are a prefix
    int cnt = A.sample_end - s0;
    cnt = cnt < len ? cnt : len;
    const int total = nv * cnt;

    lds_acc[wv][lane] = 0ull;
    lds_acc[wv][lane + 64] = 0ull;
    lds_acc[wv][lane + 128] = 0ull;
    if (lane < nv) {
        int px = x0 + (lane / A.lanes_per_pixel) * ps;
        int sub = lane % A.lanes_per_pixel;
        int sy = sub / A.nsub;
        int sx = sub - sy * A.nsub;
        const uint64_t pix_sub = ((uint64_t)y * (uint64_t)A.W + (uint64_t)px) * (uint64_t)A.lanes_per_pixel + (uint64_t)sub;
        lds_key[wv][lane] = key_hash(A.seed, pix_sub);
        lds_pix[wv][lane] = (uint32_t)px | ((uint32_t)sx << 20) | ((uint32_t)sy << 26);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");

    int item = lane < total ? lane : -1;
    int slot = 0;
    f3 o, d, T, E;
    int depth = 0;
    uint32_t st = 0;
    uint32_t segs = 0;  // scene scans executed by this lane
    ScanCount scnt;     // BVH sphere/box tests (counting kernel)
    // Each lane keeps its NEXT path's camera ray prefetched in LDS: a lane
    // whose path ends starts the prefetched one at once (two LDS reads), and
    // the camera code runs only in refills of >= PTG_REFILL_BATCH lanes (or
    // when a lane would otherwise idle).
    __shared__ float4 lds_pre[kWaves][64][2];
    // the lane's own record.  BVH kernel: its address formed at each use
    // (v_mbcnt of an opaque all-ones mask: not hoisted), not held in a VGPR
    // for the unit -- at 64 VGPRs it had been spilled and reloaded in the main
    // loop (C5 -0.3 %; the linear kernel, with VGPRs to spare, is 1.4 % slower
    // that way)
    auto pre_rec = [&]() -> float4 * {
        if constexpr (kBvh) {
            unsigned ones = ~0u;
            asm volatile("" : "+s"(ones));
            const unsigned ln = __builtin_amdgcn_mbcnt_hi(ones, __builtin_amdgcn_mbcnt_lo(ones, 0u));
            return lds_pre[wv][ln];
        } else {
            return lds_pre[wv][lane];
        }
    };
    // it / nv and it % nv (only for a unit of fewer than 64 slots; it <
    // 64 * kMaxChunk = 2^22, so the float quotient is within 1 of it / nv and
    // one correction step is exact) through a float reciprocal formed at
    // each use: the compiler's
    // integer division by the unit's nv kept its constants in VGPRs for the
    // whole unit (spilled to scratch)
    auto divmod_nv = [&](int it, int &q, int &r) {
        int n = nv;
        asm volatile("" : "+s"(n));
        q = (int)((float)it * __builtin_amdgcn_rcpf((float)n));
        r = it - q * n;
        q = r < 0 ? q - 1 : (r >= n ? q + 1 : q);
        r = r < 0 ? r + n : (r >= n ? r - n : r);
    };
    auto ray_of = [&](int it, f3 &ro, f3 &rd, uint32_t &rs) {
        int sl, sample;
        if (nv == 64) {
            sl = it & 63;
            sample = s0 + (it >> 6);
        } else {
            int q;
            divmod_nv(it, q, sl);
            sample = s0 + q;
        }
        Lane L;
        uint32_t pk = lds_pix[wv][sl];
        L.x = (int)(pk & 0xFFFFFu);
        int yy = y;  // opaque: (float)y is converted here, not held in a VGPR for the unit
        asm volatile("" : "+s"(yy));
        L.y = yy;
        L.sx = (int)((pk >> 20) & 63u);
        L.sy = (int)(pk >> 26);
        L.key = lds_key[wv][sl];
        // the index is opaque to the compiler, so the reads stay here
        // instead of being hoisted into registers live for the whole unit
        int ci = 0;
        asm volatile("" : "+v"(ci));
        const CamC C{lds_cam[ci], lds_cam[ci + 1], lds_cam[ci + 2], lds_cam[ci + 3]};
        camera_ray(C, L, (uint32_t)sample, rs, ro, rd);
    };
    // (BVH scenes: a started ray is fresh -- in neither of the main loop's
    // scan-phase masks, which its lane has left by then)
    auto begin = [&](int it, f3 ro, f3 rd, uint32_t rs) {
        item = it;
        if (nv == 64) {
            slot = it & 63;
        } else {
            int q;
            divmod_nv(it, q, slot);
        }
        o = ro;
        d = rd;
        st = rs;
        T = mk3(1.0f, 1.0f, 1.0f);
        E = mk3(0.0f, 0.0f, 0.0f);
        depth = 0;
    };
    auto store_pre = [&](int it, f3 ro, f3 rd, uint32_t rs) {
        float4 *rec = pre_rec();
        rec[0] = make_float4(ro.x, ro.y, rd.x, rd.y);
        // ro.z (= the camera's z, the lens offset has no z) rides in the
        // record's last word: read back with the ray, not as a kernel
        // argument (a scalar load + wait in the path-start block)
        rec[1] = make_float4(rd.z, __uint_as_float(rs), __int_as_float(it), ro.z);
    };
    // the lanes' loop state as wave masks (SGPRs, updated by the scalar unit
    // at wave level; a lane's bit read with inverse_ballot): kept per lane,
    // the bools lived in VGPRs and every iteration re-formed their lane masks
    // with compares.  hmask: a prefetched ray in LDS; wmask: path ended, no
    // prefetched ray yet (E kept until the batch); pmask: a finished path's
    // radiance parked in the lane's LDS record
    unsigned long long hmask = 0ull, wmask = 0ull, pmask = 0ull;
    auto lane_in = [](unsigned long long m) { return __builtin_amdgcn_inverse_ballot_w64(m); };
    if (item >= 0) {
        f3 ro, rd;
        uint32_t rs;
        ray_of(item, ro, rd, rs);
        begin(item, ro, rd, rs);
    }
    if (64 + lane < total) {
        f3 ro, rd;
        uint32_t rs;
        ray_of(64 + lane, ro, rd, rs);
        store_pre(64 + lane, ro, rd, rs);
    }
    hmask = __ballot(64 + lane < total);
    int next = total < 128 ? total : 128;  // wave-uniform pool cursor
    uint32_t bad = 0;  // counting kernel: paths with a NaN / negative / > 2^30 radiance component
    auto flush = [&](float ex, float ey, float ez, int sl) {
        if constexpr (kCount)
            bad += (in_quant_range(ex) && in_quant_range(ey) && in_quant_range(ez)) ? 0u : 1u;
        atomicAdd(&lds_acc[wv][sl], quant(ex));
        atomicAdd(&lds_acc[wv][sl + 64], quant(ey));
        atomicAdd(&lds_acc[wv][sl + 128], quant(ez));
    };
    // A finished path parks its radiance (E, slot) in the lane's LDS record
    // lds_pre[wv][lane], which just gave up its prefetched ray; the quantise +
    // LDS adds run for all parked lanes at the next refill batch (before the
    // refill writes new prefetched rays there).  A lane that finishes again
    // before the batch has no prefetched ray: it waits (E in registers),
    // which forces a batch; there its E is parked, and it starts a new ray.
    auto park = [&]() { pre_rec()[0] = make_float4(E.x, E.y, E.z, __int_as_float(slot)); };
    auto flush_parked = [&]() {
        const float4 pk = pre_rec()[0];
        flush(pk.x, pk.y, pk.z, __float_as_int(pk.w));
    };
    // path end of the lanes in done (a wave mask): park the radiance and
    // start the prefetched ray, or wait
    auto paths_done = [&](const unsigned long long done) {
        if (done == 0ull)
            return;
        const unsigned long long start = done & hmask;
        if (lane_in(done)) {
            item = -1;
            if (lane_in(start)) {
                const float4 *rec = pre_rec();
                const float4 p0 = rec[0], p1 = rec[1];
                park();
                begin(__float_as_int(p1.z), mk3(p0.x, p0.y, p1.w), mk3(p0.z, p0.w, p1.x), __float_as_uint(p1.y));
            }
        }
        pmask |= start;
        hmask &= ~start;
        wmask |= done & ~start;
    };
    // refill batch: flush parked paths, prefetch camera rays for lanes
    // without one, start idle lanes
    auto refill = [&]() {
        if (next < total) {
            const unsigned long long need = __ballot(1) & ~hmask;
            const int nn = (int)__popcll(need);
            if (nn >= PTG_REFILL_BATCH || wmask != 0ull) {
                PTG_STAT(6);
#if PTG_BLOCK_STATS == 3
                PTG_SUB_T(rf_t0);
#endif
                const unsigned long long idle = wmask | __ballot(item < 0);
                if (lane_in(pmask))
                    flush_parked();
                if (lane_in(wmask))
                    park();
                pmask = wmask;
                wmask = 0ull;
#if PTG_BLOCK_STATS == 3
                PTG_SUB_T(rf_t1);
                unsigned long long rf_ray = 0;
#endif
                // lanes of need below this one (v_mbcnt: no 64-bit lane mask held in VGPRs)
                const int ni = next + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(need >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((unsigned)need, 0u));
                const unsigned long long got = need & __ballot(ni < total);
                if (lane_in(got)) {
                    f3 ro, rd;
                    uint32_t rs;
#if PTG_BLOCK_STATS == 3
                    PTG_SUB_T(rr_t0);
#endif
                    ray_of(ni, ro, rd, rs);
#if PTG_BLOCK_STATS == 3
                    rf_ray = clock64() - rr_t0;
#endif
                    if (lane_in(idle))  // idle lane: start it now (its record may hold a parked path)
                        begin(ni, ro, rd, rs);
                    else
                        store_pre(ni, ro, rd, rs);
                }
                hmask |= got & ~idle;
                next += nn;
#if PTG_BLOCK_STATS == 3
                {
                    const unsigned long long rf_t2 = clock64();
                    unsigned long long ray_max = rf_ray;  // the wave's camera-ray time: its slowest lane's span
                    for (int off = 32; off > 0; off >>= 1)
                        ray_max = max(ray_max, (unsigned long long)__shfl_xor(ray_max, off, 64));
                    PTG_SUB_ADD(0, 1ull);
                    PTG_SUB_ADD(1, rf_t1 - rf_t0);
                    PTG_SUB_ADD(2, ray_max);
                    PTG_SUB_ADD(3, (rf_t2 - rf_t1) - ray_max);
                }
#endif
            }
        } else if (wmask != 0ull) {  // pool exhausted: nothing left for this lane
            if (lane_in(wmask))
                flush(E.x, E.y, E.z, slot);
            wmask = 0ull;
        }
    };
    if constexpr (!kBvh) {
#if PTG_BLOCK_STATS == 3  // debug: wave cycles of the linear kernel's scan / shade / refill / loop control
        unsigned long long ph_cyc[6] = {0, 0, 0, 0, 0, 0}, ph_t = clock64();
        auto lin_phase = [&](int i) {
            const unsigned long long t_ = clock64();
            ph_cyc[i] += t_ - ph_t;
            ph_t = t_;
        };
#endif
        for (;;) {
            if ((__ballot(item >= 0) | wmask) == 0ull)
                break;
            PTG_STAT(0);
#if PTG_BLOCK_STATS == 3
            lin_phase(5);
            float t3 = 0.0f;
            const LinRec *w3 = nullptr;
            if (item >= 0) {
                if constexpr (kCount)
                    segs += 1;
                w3 = scene_scan<kExact, kCount>(A, recs, o, d, t3, scnt);
            }
            lin_phase(0);
            paths_done(__ballot(item >= 0 && shade<kExact>(w3 != recs + A.n ? &w3->s : nullptr, t3, trig, o, d, T, E, depth, st)));
            lin_phase(3);
            refill();
            lin_phase(4);
#else
            bool done = false;
            if (item >= 0) {
                PTG_STAT(1);
                if constexpr (kCount)
                    segs += 1;
                done = segment<kBvh, kExact, kCount>(A, recs, trig, o, d, T, E, depth, st, scnt);
            }
            paths_done(__ballot(done));
            refill();
#endif
        }
#if PTG_BLOCK_STATS == 3
        if (lane == 0)
            for (int k = 0; k < 6; ++k)
                atomicAdd(&ptg_dbg_stats[(blockIdx.x & 255) * 16 + 8 + k], ph_cyc[k]);
#endif
    } else {
        // BVH scenes: each lane is fresh (ray set, scan not started), walking
        // or ready (scan done, to be shaded); an iteration starts the fresh
        // lanes' scans, walks until enough lanes are ready (PTG_READY_FRAC/8
        // of the active lanes) or none walks, shades the ready lanes.
        BvhTrav tr{};  // started per segment by bvh_start
        unsigned long long wk = 0ull, rd = 0ull;  // walking / scan done (see the loop)
#if PTG_LEAF_SPLIT
        __shared__ uint8_t lds_pair[kWaves][2][64];  // leaf phase: owner / helper lane of each rank
#endif
        // kernel-argument pointers used in the loops, pinned in SGPRs once:
        // left to the compiler they were re-loaded (s_load + wait) in every
        // node step and every shade
        gptr<u32x4> qnodes = (gptr<u32x4>)A.bvh_qnodes;
        asm volatile("" : "+s"(qnodes));
        gptr<int> cont = (gptr<int>)A.bvh_cont;
        asm volatile("" : "+s"(cont));
        if constexpr (kExact)  // (the fast mode's sin/cos read no table)
            asm volatile("" : "+s"(trig));
#if PTG_BLOCK_STATS == 2
        unsigned long long ph_cyc[6] = {0, 0, 0, 0, 0, 0}, ph_t = clock64();
#endif
        for (;;) {
            if ((__ballot(item >= 0) | wmask) == 0ull)
                break;
            PTG_PHASE(5);
            // the lanes' scan phase as wave masks (like hmask / wmask / pmask):
            // wk walking, rd scan done (to be shaded); a fresh lane is active
            // and in neither.  A lane's scan is done when ni == -1 and no leaf
            // is parked: two single-compare ballots (a ballot of the combined
            // predicate is materialised as v_cndmask + v_cmp)
            const unsigned long long act = __ballot(item >= 0);
            {
                const unsigned long long fresh = act & ~(wk | rd);
                if (lane_in(fresh)) {
                    if constexpr (kCount)
                        segs += 1;
                    bvh_start<kCount && !PTG_WAVE_STATS, kExact>(A, o, d, tr, scnt);
                }
                const unsigned long long fin = fresh & __ballot(tr.ni == -1) & __ballot(tr.pend < 0);
                rd |= fin;
                wk |= fresh & ~fin;
            }
            PTG_PHASE(0);
            {
                const SlabRay sr = slab_ray(A, o, d);
                const int na = (int)__popcll(act);
                // Node steps in an inner loop, the leaf phase in the outer one:
                // with both in one loop body, the merge of the two branches'
                // traversal states cost 14+ v_mov per node step (the compiler
                // copied the 7 state registers out and back in; C5 -1.5 %).
                for (;;) {
                    unsigned long long mhas = 0ull;
                    bool walk_done = false;
                    for (;;) {
                        // ballots of single compares: a ballot of a combined
                        // predicate (x && y) is materialised as v_cndmask + v_cmp,
                        // 2 VALU each.  A walking lane has item >= 0 (an item
                        // ends only in shading, after the walk), and na does not
                        // change inside the walk.
                        const unsigned long long mt = wk;
                        const int nt = (int)__popcll(mt);
                        if (mt == 0ull || 8 * (na - nt) >= PTG_READY_FRAC * na) {
                            walk_done = true;
                            break;
                        }
                        mhas = __ballot(tr.pend >= 0) & mt;  // walking lanes holding a leaf
                        if (8 * (int)__popcll(mhas) >= PTG_LEAF_FRAC * nt)
                            break;  // leaf phase
#if PTG_WAVE_STATS == 1  // debug: wave-level node steps (first active lane only)
                        if constexpr (kCount)
                            scnt.boxes += __lane_id() == __ffsll((long long)__ballot(1)) - 1 ? 1 : 0;
#endif
                        PTG_PHASE(5);
                        // (the node step as selects for the whole wave, like the
                        // leaf completion: +2.3 % -- its loads and selects for idle lanes)
                        if (lane_in(mt & ~mhas))
                            bvh_node_step<kCount && !PTG_WAVE_STATS>(cont, qnodes, sr, tr, scnt);
                        PTG_PHASE(1);
                        {
                            const unsigned long long fin = wk & __ballot(tr.ni == -1) & __ballot(tr.pend < 0);
                            rd |= fin;
                            wk &= ~fin;
                        }
                    }
                    if (walk_done)
                        break;
                    // leaf phase (round 1: spreading the parked leaves' spheres over
                    // the whole wave with ds_bpermute + LDS atomicMin measured 1.7 %
                    // slower; pairing idle lanes with the long leaves 1.2-1.5 % faster)
#if PTG_LEAF_SPLIT
                    bvh_leaf_split<kCount && !PTG_WAVE_STATS, kExact>(A, cont, o, d, lane_in(mhas), mhas, tr, scnt,
                                                               lds_pair[wv]);
#else
                    if (lane_in(mhas))
                        bvh_leaf<kCount && !PTG_WAVE_STATS, kExact>(A, cont, o, d, tr, scnt);
#endif
                    PTG_PHASE(2);
                    {
                        const unsigned long long fin = wk & __ballot(tr.ni == -1) & __ballot(tr.pend < 0);
                        rd |= fin;
                        wk &= ~fin;
                    }
                }
            }
#if PTG_WAVE_STATS == 2  // debug: wave-level main-loop iterations / iterations that shade (first active lane)
            if constexpr (kCount) {
                const bool first_lane = __lane_id() == __ffsll((long long)__ballot(1)) - 1;
                scnt.boxes += first_lane ? 1 : 0;
                scnt.spheres += (first_lane && rd != 0ull) ? 1 : 0;
            }
#endif
            PTG_PHASE(5);
            bool done = false;
            const unsigned long long shade_m = rd;
            rd = 0ull;
            if (lane_in(shade_m)) {
                const int sid = tr.best;
                const ShadeRec *hrec = sid >= 0 ? A.shade + sid : nullptr;
                done = shade<kExact>(hrec, tr.tb, trig, o, d, T, E, depth, st);
            }
            paths_done(__ballot(done));
            PTG_PHASE(3);
            refill();
            PTG_PHASE(4);
        }
#if PTG_BLOCK_STATS == 2
        if (lane == 0)
            for (int k = 0; k < 6; ++k)
                atomicAdd(&ptg_dbg_stats[(blockIdx.x & 255) * 16 + 8 + k], ph_cyc[k]);
#endif
    }
    if (lane_in(pmask))
        flush_parked();
    // the lane index re-formed here (v_mbcnt of an opaque all-ones mask):
    // taken from the work-item id it was held, and spilled, through the main
    // loop for the epilogue's uses
    const int lane_e = [] {
        unsigned ones = ~0u;
        asm volatile("" : "+s"(ones));
        return (int)__builtin_amdgcn_mbcnt_hi(ones, __builtin_amdgcn_mbcnt_lo(ones, 0u));
    }();
    if constexpr (kCount) {
        unsigned long long ws = segs, wsph = scnt.spheres, wbox = scnt.boxes, wbad = bad;
        for (int off = 32; off > 0; off >>= 1) {
            ws += __shfl_xor(ws, off, 64);
            wsph += __shfl_xor(wsph, off, 64);
            wbox += __shfl_xor(wbox, off, 64);
            wbad += __shfl_xor(wbad, off, 64);
        }
        if (lane_e == 0 && A.count_nonfinite && wbad)
            atomicAdd(A.segments + 3, wbad);
        if (lane_e == 0 && ws)
            atomicAdd(A.segments, ws);
        if (lane_e == 0 && A.count_tests) {
            atomicAdd(A.segments + 1, wsph);
            atomicAdd(A.segments + 2, wbox);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    bool coop_last = false;
    if (coop) {
        // publish this wave's sums (its LDS adds are complete), count it; the
        // wave that completes the count adds every wave's sums and resolves
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        int prev = 0;
        if (lane_e == 0)
            prev = __hip_atomic_fetch_add(&lds_coop_done, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        prev = __shfl(prev, 0, 64);
        coop_last = prev == kWaves - 1;
        if (!coop_last) {
            PTG_TRACE_END();
            return;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    if (in_wave || coop_last) {
        // the unit (or the workgroup) holds every sample of its pixels:
        // resolve here (main.cpp:195-196, same arithmetic as resolve_kernel)
        // and write 12 B per pixel -- the only HBM traffic of the frame
        if (lane_e < npix && r < A.H) {
            f3 pix = mk3(0.0f, 0.0f, 0.0f);
            for (int j = 0; j < A.lanes_per_pixel; ++j) {
                const int sl = lane_e * A.lanes_per_pixel + j;
                float m[3];
                for (int c = 0; c < 3; ++c) {
                    unsigned long long sum = lds_acc[wv][sl + 64 * c];
                    if (coop_last) {
                        sum = 0ull;
                        for (int w = 0; w < kWaves; ++w)  // exact: integer sums in any order
                            sum += lds_acc[w][sl + 64 * c];
                    }
                    const float mean = A.samps > 0 ? (float)(((double)sum * 0x1p-32) / (double)A.samps) : 0.0f;
                    m[c] = mean < 0.0f ? 0.0f : (1.0f < mean ? 1.0f : mean);
                }
                pix = mk3(__builtin_fmaf(m[0], A.inv_sub2, pix.x), __builtin_fmaf(m[1], A.inv_sub2, pix.y),
                          __builtin_fmaf(m[2], A.inv_sub2, pix.z));
            }
            // opaque lane: the address is formed here, not hoisted to the
            // unit start and held (spilled) in VGPRs through the main loop
            int ln = lane_e;
            asm volatile("" : "+v"(ln));
            float *out = A.out + ((size_t)slab_row * A.W + x0 + ln * ps) * 3;
            out[0] = pix.x;
            out[1] = pix.y;
            out[2] = pix.z;
        }
    } else if (lane_e < nv) {
        // several units share these pixels: exact u64 adds, resolved later
        // opaque: the address is formed here, not held in VGPRs for the unit
        int ln = lane_e, row = slab_row, px0 = x0;
        asm volatile("" : "+v"(ln), "+s"(row), "+s"(px0));
        unsigned long long *g = A.acc + (((size_t)row * A.W + px0) * A.lanes_per_pixel + ln) * 3;
        unsigned long long vx = lds_acc[wv][ln], vy = lds_acc[wv][ln + 64], vz = lds_acc[wv][ln + 128];
        if (vx) atomicAdd(g + 0, vx);
        if (vy) atomicAdd(g + 1, vy);
        if (vz) atomicAdd(g + 2, vz);
    }
    PTG_TRACE_END();
}

// main.cpp:195-196: per pixel, the clamped sub-pixel means added with weight
// 1/nsub^2 in (sy, sx) order; re-zeroes the accumulator for the next frame.
__global__ __launch_bounds__(256) void resolve_kernel(KArgs A)
{
    const long long i = (long long)A.resolve_row0 * A.W + (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long long)A.slab_rows * A.W)
        return;
    const int slab_row = (int)(i / A.W);
    if (out_row_of(A, slab_row) >= A.H)
        return;
    unsigned long long *g = A.acc + (size_t)i * A.lanes_per_pixel * 3;
    f3 pix = mk3(0.0f, 0.0f, 0.0f);
    for (int j = 0; j < A.lanes_per_pixel; ++j) {
        float m[3];
        for (int c = 0; c < 3; ++c) {
            unsigned long long sum = g[3 * j + c];
            if (!A.keep_acc)
                g[3 * j + c] = 0ull;
            float mean = A.samps > 0 ? (float)(((double)sum * 0x1p-32) / (double)A.samps) : 0.0f;
            m[c] = mean < 0.0f ? 0.0f : (1.0f < mean ? 1.0f : mean);
        }
        pix = mk3(__builtin_fmaf(m[0], A.inv_sub2, pix.x), __builtin_fmaf(m[1], A.inv_sub2, pix.y),
                  __builtin_fmaf(m[2], A.inv_sub2, pix.z));
    }
    float *out = A.out + (size_t)i * 3;
    out[0] = pix.x;
    out[1] = pix.y;
    out[2] = pix.z;
}

// Parity probe: one path per record {x, y, sx, sy, sample}.
template <bool kBvh, bool kExact>
__global__ __launch_bounds__(kTraceBlock) void trace_kernel(KArgs A, const int32_t *coords, int n, float *out,
                                                         int32_t *segs_out)
{
    int i = blockIdx.x * kTraceBlock + threadIdx.x;
    if (i >= n)
        return;
    Lane L;
    L.x = coords[5 * i + 0];
    L.y = coords[5 * i + 1];
    L.sx = coords[5 * i + 2];
    L.sy = coords[5 * i + 3];
    uint32_t sample = (uint32_t)coords[5 * i + 4];
    uint64_t pixel_sub = ((uint64_t)L.y * (uint64_t)A.W + (uint64_t)L.x) * (uint64_t)A.lanes_per_pixel +
                         (uint64_t)(L.sy * A.nsub + L.sx);
    L.key = key_hash(A.seed, pixel_sub);
    f3 o, d;
    uint32_t st;
    camera_ray(cam_of(A), L, sample, st, o, d);
    f3 T = mk3(1.0f, 1.0f, 1.0f), E = mk3(0.0f, 0.0f, 0.0f);
    int depth = 0, segs = 0;
    bool done = false;
    while (!done) {
        segs += 1;
        ScanCount scnt;
        done = segment<kBvh, kExact>(A, A.lin, A.trig, o, d, T, E, depth, st, scnt);
    }
    out[3 * i + 0] = E.x;
    out[3 * i + 1] = E.y;
    out[3 * i + 2] = E.z;
    segs_out[i] = segs;
}

// ptg_math_probe_device: the primitives as the render kernels call them
template <bool kExact>
__global__ __launch_bounds__(256) void math_probe_kernel(int op, const float *in, float *out, int n,
                                                         const float2 *trig)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    if (op == PTG_PROBE_SQRT) {
        out[i] = Math<kExact>::sqrt(in[i]);
    } else if (op == PTG_PROBE_RSQRT) {
        out[i] = Math<kExact>::rsqrt(in[i]);
    } else if (op == PTG_PROBE_DIV) {
        out[i] = Math<kExact>::div(in[2 * i], in[2 * i + 1]);
    } else {
        float c, s;
        Math<kExact>::sincos2pi(__float_as_uint(in[i]) & 0xFFFFFFu, trig, c, s);
        out[2 * i] = c;
        out[2 * i + 1] = s;
    }
}

__global__ void unshard_kernel(const float *__restrict__ src, float *__restrict__ dst, int W, int band_rows,
                               int count, int slab_rows)
{
    int r = blockIdx.y;
    int band = r / band_rows;
    int k = band % count;
    int j = band / count;
    size_t srow = (size_t)k * slab_rows + (size_t)j * band_rows + (size_t)(r - band * band_rows);
    const float *s = src + srow * (size_t)W * 3;
    float *t = dst + (size_t)r * (size_t)W * 3;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < W * 3; i += gridDim.x * blockDim.x)
        t[i] = s[i];
}

// utils.cpp:11-16: round(pow(clamp(x), 1/2.2) * 255)
__global__ void tonemap_kernel(const float *__restrict__ in, uint8_t *__restrict__ out, size_t count)
{
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count)
        return;
    double x = (double)in[i];
    x = x < 0.0 ? 0.0 : (1.0 < x ? 1.0 : x);
    out[i] = (uint8_t)(int)round(pow(x, 1.0 / 2.2) * 255.0);
}

}  // namespace

struct ptg_context {
    int device;
    int n;
    int wave_slots;     // CUs x 32 resident waves (split-tail sizing)
    LinRec *d_lin;      // linear scenes
    ShadeRec *d_shade;  // BVH scenes
    void *d_bvh;  // one allocation: nodes | leaf geometry | leaf ids | big geometry | big ids
    float2 *d_trig;  // sin/cos table (trig_table)
    unsigned long long *d_acc;  // exact per-sub-pixel sums; kept zero between frames by resolve
    size_t acc_elems;
    bool acc_dirty;  // progressive sums may be in d_acc (accumulate / keep_acc resolve since the last reset)
    KArgs base;  // camera + scene fields filled
    ptg_sphere *d_sph64;  // the scene as given (PTG_FLAG_REFERENCE_F64)
    ptg_camera cam64;
};

namespace {

bool sphere_ok(const ptg_sphere &s)
{
    if (!(s.radius > 0.0) || !std::isfinite(s.radius))
        return false;
    for (int c = 0; c < 3; ++c)
        if (!std::isfinite(s.position[c]) || !std::isfinite(s.emission[c]) || !std::isfinite(s.color[c]))
            return false;
    return s.material >= PTG_DIFFUSE && s.material <= PTG_DIELECTRIC;
}

// Anchor of a huge sphere (DESIGN.md "Huge spheres"): the point P = C + R n0
// of the sphere and its outward normal n0.  The default n0 is the unit vector
// from C towards the camera.  When the point C + s R e_k of the dominant axis
// direction of that n0 (k = largest |n0_k|, s = its sign) lies near the scene
// -- within max(diagonal, 1) of the box around the camera and the non-huge
// spheres -- that axis point is the anchor instead: any point of the sphere is
// an exact anchor, and one near the scene keeps |o - P| at scene scale (box
// walls: the axis points lie inside that box).  Returns k, or -1 for the
// camera-facing anchor.  The oracle's prep_B makes the same choice
// (oracle/pt_oracle.c: choose_anchor_B).
struct SceneBox {
    double lo[3], hi[3], diag;
};

int choose_anchor(const ptg_sphere &sp, const ptg_camera *cam, const SceneBox &box, double P[3], double N[3])
{
    const double R = sp.radius;
    double v[3], len2 = 0.0;
    for (int c = 0; c < 3; ++c) {
        v[c] = cam->position[c] - sp.position[c];
        len2 += v[c] * v[c];
    }
    const double len = std::sqrt(len2);
    for (int c = 0; c < 3; ++c)
        N[c] = len > 0.0 ? v[c] / len : (c == 1 ? 1.0 : 0.0);
    int k = 0;
    for (int c = 1; c < 3; ++c)
        if (std::fabs(N[c]) > std::fabs(N[k]))
            k = c;
    const double s = N[k] >= 0.0 ? 1.0 : -1.0;
    double out2 = 0.0;  // squared distance of the axis point from the scene box
    for (int c = 0; c < 3; ++c) {
        const double pa = sp.position[c] + (c == k ? s * R : 0.0);
        const double o = pa < box.lo[c] ? box.lo[c] - pa : (pa > box.hi[c] ? pa - box.hi[c] : 0.0);
        out2 += o * o;
    }
    const bool snap = std::sqrt(out2) <= std::max(box.diag, 1.0);
    for (int c = 0; c < 3; ++c) {
        if (snap)
            N[c] = c == k ? s : 0.0;
        P[c] = sp.position[c] + R * N[c];
    }
    return snap ? k : -1;
}

// Box around the camera and every non-huge sphere, and its diagonal.
SceneBox scene_box(const ptg_sphere *s, int n, const ptg_camera *cam)
{
    SceneBox b;
    for (int c = 0; c < 3; ++c)
        b.lo[c] = b.hi[c] = cam->position[c];
    for (int i = 0; i < n; ++i) {
        if (is_huge(s[i], cam))
            continue;
        for (int c = 0; c < 3; ++c) {
            b.lo[c] = std::min(b.lo[c], s[i].position[c] - s[i].radius);
            b.hi[c] = std::max(b.hi[c], s[i].position[c] + s[i].radius);
        }
    }
    double d2 = 0.0;
    for (int c = 0; c < 3; ++c)
        d2 += (b.hi[c] - b.lo[c]) * (b.hi[c] - b.lo[c]);
    b.diag = std::sqrt(d2);
    return b;
}

// Host-side preparation (double -> fp32 records, scene index order), the
// counterpart of the oracle's Mode B prep_B.  axis[i] = anchor axis of a huge
// sphere (-1: camera-facing anchor or not huge).
void prepare_scene(const ptg_sphere *s, int n, const ptg_camera *cam, std::vector<GeoRec> &geo,
                   std::vector<ShadeRec> &shade, std::vector<int> &axis)
{
    geo.resize(n);
    shade.resize(n);
    axis.assign(n, -1);
    const SceneBox box = scene_box(s, n, cam);
    for (int i = 0; i < n; ++i) {
        const ptg_sphere &sp = s[i];
        const double R = sp.radius;
        GeoRec g;
        if (is_huge(sp, cam)) {
            double P[3], N[3];
            axis[i] = choose_anchor(sp, cam, box, P, N);
            g.g0 = make_float4((float)P[0], (float)P[1], (float)P[2], (float)R);
            g.g1 = make_float4((float)N[0], (float)N[1], (float)N[2], (float)(2.0 * R));
        } else {
            g.g0 = make_float4((float)sp.position[0], (float)sp.position[1], (float)sp.position[2],
                               (float)(-(R * R)));
            g.g1 = make_float4(0.0f, 0.0f, 0.0f, (float)(-(R * R)));
        }
        geo[i] = g;
        ShadeRec r;
        float cx = (float)sp.color[0], cy = (float)sp.color[1], cz = (float)sp.color[2];
        float p = cx;
        if (p < cy) p = cy;
        if (p < cz) p = cz;
        float rx = 0.0f, ry = 0.0f, rz = 0.0f;
        if (p > 0.0f) {
            float inv = 1.0f / p;
            rx = cx * inv;
            ry = cy * inv;
            rz = cz * inv;
        }
        int32_t mat = sp.material;
        float matf;
        std::memcpy(&matf, &mat, 4);
        // Russian roulette as an integer compare (main.cpp:130-131, u < p):
        // u = m 2^-24 exactly (m the draw's 24-bit integer), so u < p <=> m <
        // p 2^24 <=> m < ceil(p 2^24) -- the same decisions as the oracle's
        // float compare, without the draw's convert and scale
        uint32_t p24 = !(p > 0.0f) ? 0u : (p >= 1.0f ? (1u << 24) : (uint32_t)std::ceil((double)p * 16777216.0));
        float p24f;
        std::memcpy(&p24f, &p24, 4);
        r.s0 = make_float4((float)sp.position[0], (float)sp.position[1], (float)sp.position[2], p24f);
        r.s1 = make_float4((float)sp.emission[0], (float)sp.emission[1], (float)sp.emission[2], matf);
        r.s2 = make_float4(cx, cy, cz, (float)(1.0 / R));
        r.s3 = make_float4(rx, ry, rz, (float)(1.0 / R));
        shade[i] = r;
    }
}

// Wall pairs (DESIGN.md "wall pairs"): on each axis k, the first (scene
// index order) axis-anchored huge sphere whose centre lies on the + side of
// its anchor (anchor normal -e_k) and the first one on the - side.  Their
// tangent planes at the anchors, x_k = a_plus and x_k = a_minus, bound the
// room: a ray from an origin with a_minus <= o_k <= a_plus can hit the + wall
// only if d_k > 0 and the - wall only if d_k < 0 (each sphere lies entirely
// beyond its tangent plane).  The bounds widen by a margin of 1e-4 max(1, box
// diagonal) so that rays leaving a wall (origin rounded a hair past its
// plane) keep the rule; pair_lo/hi are those bounds rounded to float.  The
// oracle's prep_B forms the same pairs (pt_oracle.c).  plus[k] / minus[k] =
// scene index or -1.
// A wall may take part in wall pairs / box mode only if no ray origin can lie
// genuinely inside it, beyond its tangent plane, where the "test only the
// wall the ray moves toward" rule would drop a hit of the wall from inside:
// the wall is not dielectric (no path is transmitted into it) and the camera
// is on the room side by more than the margin.  Other spheres need no check:
// a sphere sunk into the wall has its sunk part inside the wall, which a ray
// from the room reaches only through the wall's surface -- the wall is hit
// there first (tests/test_scene_file.py: a glass sphere sunk into a wall,
// pairs on vs every sphere tested, same image).  The oracle's wall_clear_B
// makes the same choice.
bool wall_clear(const ptg_sphere *s, int i, int k, bool plus_side, const ptg_camera *cam, const SceneBox &box)
{
    if (s[i].material == PTG_DIELECTRIC)
        return false;
    const double margin = 1e-4 * std::max(1.0, box.diag);
    const double a = plus_side ? s[i].position[k] - s[i].radius : s[i].position[k] + s[i].radius;
    return plus_side ? cam->position[k] < a - margin : cam->position[k] > a + margin;
}

void pair_walls(const ptg_sphere *s, int n, const std::vector<int> &axis, const std::vector<GeoRec> &geo,
                const ptg_camera *cam, const SceneBox &box, int plus[3], int minus[3], float lo[3], float hi[3])
{
    const double margin = 1e-4 * std::max(1.0, box.diag);
    for (int k = 0; k < 3; ++k) {
        plus[k] = minus[k] = -1;
        for (int i = 0; i < n; ++i) {
            if (axis[i] != k)
                continue;
            const float nk = (&geo[i].g1.x)[k];  // anchor normal component: exactly +-1
            if (nk < 0.0f && plus[k] < 0)
                plus[k] = i;
            if (nk > 0.0f && minus[k] < 0)
                minus[k] = i;
        }
        if (plus[k] < 0 || minus[k] < 0 || !wall_clear(s, plus[k], k, true, cam, box) ||
            !wall_clear(s, minus[k], k, false, cam, box)) {
            plus[k] = minus[k] = -1;
            lo[k] = hi[k] = 0.0f;
            continue;
        }
        const double a_plus = s[plus[k]].position[k] - s[plus[k]].radius;
        const double a_minus = s[minus[k]].position[k] + s[minus[k]].radius;
        lo[k] = (float)(a_minus - margin);
        hi[k] = (float)(a_plus + margin);
    }
}

// Box mode (scene_scan; DESIGN.md "box mode"): on when every axis-anchored
// wall is either one of its axis's pair or the only wall of its axis, at
// least one axis has a pair, and there is no other huge sphere.  Fills the
// per-axis records (scan positions in `order`) and tangent planes (the
// records' anchor coordinate), and extends the pair bounds to single walls
// (margin as pair_walls) and open sides (+-kFarPlane).  The oracle's prep_B
// makes the same choice.
// A sphere no ray can start inside (KArgs::box_walls_out).  A camera ray starts
// outside every sphere whose centre is farther from the camera than its
// radius plus the lens offset (< 2 lens radii: camera_ray's rd * (s + t));
// a ray reaches a surface point
// only from outside every opaque sphere it has not hit before, and a diffuse
// or mirror bounce leaves outward -- so, by induction, only dielectric
// spheres are ever entered (up to the fp32 rounding of a hit point next to a
// contact between two spheres, where the outside-only root lets the ray
// leave, as in exact arithmetic).
bool outside_only(const ptg_sphere &s, const ptg_camera *cam)
{
    double d2 = 0.0, p2 = 0.0;
    for (int c = 0; c < 3; ++c) {
        const double t = s.position[c] - cam->position[c];
        d2 += t * t;
        p2 += cam->position[c] * cam->position[c];
    }
    // margins: the lens bound's, the fp32 rounding of a camera origin, the
    // double rounding of d2
    const double reach = s.radius + 2.0001 * cam->lens_radius + 1e-6 * (1.0 + std::sqrt(p2)) + 1e-9 * s.radius;
    return s.material != PTG_DIELECTRIC && d2 > reach * reach;
}

// KArgs::room_nmr.  The kernel's up = fl(plane_plus - o_k) >= -m implies
// plane_plus - o_k >= -m (1 + 2^-23) (a rounding of at most half an ulp of a
// difference near -m; a larger difference passes or fails with its sign), so
// with m = gap (1 - 2^-10) the origin lies below plane_plus + gap =
// pair_hi; the same for um and pair_lo.  Open sides (planes at +-inf, up or
// um = +inf) bound nothing, as their +-kFarPlane bounds (unreachable) did.
float room_neg_margin(const KArgs &A)
{
    double gap = HUGE_VAL;
    for (int k = 0; k < 3; ++k) {
        if (A.plane_plus[k] < HUGE_VALF)
            gap = std::min(gap, (double)A.pair_hi[k] - (double)A.plane_plus[k]);
        if (A.plane_minus[k] > -HUGE_VALF)
            gap = std::min(gap, (double)A.plane_minus[k] - (double)A.pair_lo[k]);
    }
    if (!(gap > 0.0) || gap == HUGE_VAL)
        return HUGE_VALF;  // no lane counts as inside: every wave takes the exact per-axis checks
    const float m = (float)(gap * (1.0 - 0x1p-10));
    return -std::nextafter(m, 0.0f);
}

void box_mode_of(const ptg_sphere *s, int n, const ptg_camera *cam, const std::vector<int> &axis,
                 const std::vector<GeoRec> &geo, const std::vector<int> &order, KArgs &A)
{
    A.box_mode = 0;
    A.box_walls_out = 0;
    int cnt[3] = {0, 0, 0}, general = 0;
    for (int i = 0; i < n; ++i) {
        if (!is_huge(s[i], cam))
            continue;
        if (axis[i] < 0)
            ++general;
        else
            ++cnt[axis[i]];
    }
    bool ok = general == 0 && (A.pairs[0] || A.pairs[1] || A.pairs[2]);
    for (int k = 0; k < 3; ++k)
        ok = ok && (A.pairs[k] ? cnt[k] == 2 : cnt[k] <= 1);
    const SceneBox box = scene_box(s, n, cam);
    for (int i = 0; i < n && ok; ++i)  // single walls too (the pairs' members are clear)
        if (is_huge(s[i], cam) && axis[i] >= 0)
            ok = wall_clear(s, i, axis[i], (&geo[i].g1.x)[axis[i]] < 0.0f, cam, box);
    if (!ok)
        return;
    const double margin = 1e-4 * std::max(1.0, box.diag);
    for (int k = 0; k < 3; ++k) {
        A.rec_plus[k] = A.rec_minus[k] = -1;
        A.plane_plus[k] = HUGE_VALF;  // missing wall: never the nearest plane, never needed
        A.plane_minus[k] = -HUGE_VALF;
        const int begin = k == 0 ? 0 : A.end_ax[k - 1];
        for (int j = begin; j < A.end_ax[k]; ++j) {
            const int i = order[j];
            const float nk = (&geo[i].g1.x)[k];  // anchor normal component: exactly +-1
            const float plane = (&geo[i].g0.x)[k];  // the anchor point's coordinate
            if (nk < 0.0f) {  // centre on the + side
                A.rec_plus[k] = j * (int)sizeof(LinRec);
                A.plane_plus[k] = plane;
                if (!A.pairs[k])
                    A.pair_hi[k] = (float)(s[i].position[k] - s[i].radius + margin);
            } else {
                A.rec_minus[k] = j * (int)sizeof(LinRec);
                A.plane_minus[k] = plane;
                if (!A.pairs[k])
                    A.pair_lo[k] = (float)(s[i].position[k] + s[i].radius - margin);
            }
        }
        if (A.rec_plus[k] < 0)
            A.pair_hi[k] = kFarPlane;
        if (A.rec_minus[k] < 0)
            A.pair_lo[k] = -kFarPlane;
    }
    A.box_mode = 1;
    A.box_walls_out = 1;
    for (int i = 0; i < n; ++i)
        if (is_huge(s[i], cam) && axis[i] >= 0 && !outside_only(s[i], cam))
            A.box_walls_out = 0;
}


// Linear scenes: scan order (scene_scan) -- huge spheres anchored on x, y, z
// (each axis group led by its wall pair, + wall first), then the other huge
// spheres, then the small ones, each group otherwise in scene index order;
// end_ax / end_big / pairs receive the group ends and pair flags.
std::vector<int> scan_order_of(const ptg_sphere *s, int n, const ptg_camera *cam, const std::vector<int> &axis,
                               const std::vector<GeoRec> &geo, KArgs &A)
{
    std::vector<int> order;
    int plus[3], minus[3];
    pair_walls(s, n, axis, geo, cam, scene_box(s, n, cam), plus, minus, A.pair_lo, A.pair_hi);
    for (int k = 0; k < 3; ++k) {
        A.pairs[k] = plus[k] >= 0 ? 1 : 0;
        if (A.pairs[k]) {
            order.push_back(plus[k]);
            order.push_back(minus[k]);
        }
        for (int i = 0; i < n; ++i)
            if (axis[i] == k && i != plus[k] && i != minus[k])
                order.push_back(i);
        A.end_ax[k] = (int)order.size();
    }
    box_mode_of(s, n, cam, axis, geo, order, A);
    for (int i = 0; i < n; ++i)
        if (is_huge(s[i], cam) && axis[i] < 0)
            order.push_back(i);
    A.end_big = (int)order.size();
    for (int i = 0; i < n; ++i)
        if (!is_huge(s[i], cam))
            order.push_back(i);
    return order;
}


// Records in scan order.  Axis-anchored records carry the signs in their
// constants: g0.w = s R, g1.w = s 2R (the kernel reads e_k and d_k).
void prepare_scan_order(const ptg_sphere *s, int n, const ptg_camera *cam, const std::vector<GeoRec> &geo,
                        const std::vector<ShadeRec> &shade, const std::vector<int> &axis,
                        std::vector<GeoRec> &lgeo, std::vector<ShadeRec> &lshade, KArgs &A)
{
    lgeo.clear();
    lshade.clear();
    for (int i : scan_order_of(s, n, cam, axis, geo, A)) {
        GeoRec g = geo[i];
        if (axis[i] >= 0) {
            const float sgn = (&g.g1.x)[axis[i]];  // +-1 exactly
            g.g0.w = sgn * g.g0.w;
            g.g1.w = sgn * g.g1.w;
        }
        lgeo.push_back(g);
        lshade.push_back(shade[i]);
    }
}

int check_params(const ptg_params *p)
{
    if (!p)
        return fail(PTG_ERR_INVALID_ARGUMENT, "params is NULL");
    if (p->width <= 0 || p->height <= 0)
        return fail(PTG_ERR_INVALID_ARGUMENT, "width and height must be positive");
    if (p->samples < 0)
        return fail(PTG_ERR_INVALID_ARGUMENT, "samples must be >= 0");
    if (p->num_subpixels < 1 || p->num_subpixels > 8)
        return fail(PTG_ERR_UNSUPPORTED, "num_subpixels must be in [1, 8]");
    if (p->band_rows < 1 || p->shard_count < 1 || p->shard_rank < 0 || p->shard_rank >= p->shard_count)
        return fail(PTG_ERR_INVALID_ARGUMENT, "invalid shard (band_rows >= 1, 0 <= rank < count)");
    if ((int64_t)p->width * p->height > (int64_t)1 << 28 || p->width >= (1 << 20))
        return fail(PTG_ERR_UNSUPPORTED, "image too large");
    return PTG_OK;
}

// Launch geometry for samples [s_begin, s_end) of every sub-pixel.
int fill_launch(const ptg_context *ctx, const ptg_params *p, KArgs &A, int &grid, int s_begin = 0, int s_end = -1,
                bool accumulate_only = false)
{
    if (s_end < 0)
        s_end = p->samples;
    const int nsamp = s_end - s_begin;
    A = ctx->base;
    A.W = p->width;
    A.H = p->height;
    A.samps = p->samples;
    A.nsub = p->num_subpixels;
    A.lanes_per_pixel = p->num_subpixels * p->num_subpixels;
    A.pixels_per_wave = 64 / A.lanes_per_pixel;
    A.waves_per_row = (p->width + A.pixels_per_wave - 1) / A.pixels_per_wave;
    int bands = (p->height + p->band_rows - 1) / p->band_rows;
    A.slab_rows = ((bands + p->shard_count - 1) / p->shard_count) * p->band_rows;
    A.band_rows = p->band_rows;
    A.shard_rank = p->shard_rank;
    A.shard_count = p->shard_count;
    A.invW = 1.0f / (float)p->width;
    A.invH = 1.0f / (float)p->height;
    A.inv_samps = p->samples > 0 ? 1.0f / (float)p->samples : 0.0f;
    A.sub_len = 1.0f / (float)p->num_subpixels;
    A.inv_sub2 = 1.0f / (float)(p->num_subpixels * p->num_subpixels);
    A.seed = p->seed;
    A.sample_begin = s_begin;
    A.sample_end = s_end;
    A.keep_acc = 0;
    A.count_tests = (p->flags & PTG_FLAG_COUNT_TESTS) != 0;
    A.count_nonfinite = (p->flags & PTG_FLAG_COUNT_NONFINITE) != 0;
    A.exact_math = (p->flags & PTG_FLAG_EXACT_MATH) != 0;
    if (!A.exact_math && !A.box_walls_out)
        A.box_mode = 0;  // the fast mode's box-mode wall test assumes rays outside the walls
    // work unit = pixel group x chunk of samples.  Auto: split the samples
    // only as far as needed for ~96k work units (about 16 waves per SIMD slot
    // on 256 CUs), which keeps the grid-level tail small at any GPU count.
    // Below the split-tail threshold, BVH scenes aim at PTG_BVH_UNIT_MULT
    // times more units: their cost varies strongly over the image (sky rows
    // vs the sphere field).
    const int groups = A.slab_rows * A.waves_per_row;
    // split tail (below) from PTG_TAIL_MIN_HALF_ROUNDS/2 rounds of the
    // device's wave slots on, BVH scenes from PTG_BVH_TAIL_MIN_HALF_ROUNDS/2
    // (then the head runs whole-pixel units even where ~96k units would split
    // samples, e.g. an 8-GPU shard).  The head's units are whole pixels, so
    // the head needs enough rounds to average out the rows' different costs:
    // at 2 rounds (8-way shards of the bench frame) the split tail gains
    // 1.7-2.1 % on the box scenes but loses 28 % on the 10,000-sphere scene
    // (tools/scene_shard_ab.sh); from 4 rounds on it gains on both.
    const long long tail_min = (long long)(ctx->n > kLinearMax ? PTG_BVH_TAIL_MIN_HALF_ROUNDS : PTG_TAIL_MIN_HALF_ROUNDS) *
                               ctx->wave_slots / 2;
    const bool tail_ok = p->chunk_samples <= 0 && !accumulate_only && s_begin == 0 && s_end == p->samples &&
                         PTG_TAIL_CHUNKS > 1 && nsamp >= PTG_TAIL_CHUNKS && nsamp <= kMaxChunk && groups >= tail_min;
    int chunk = p->chunk_samples;
    if (tail_ok) {
        chunk = nsamp;
    } else if (chunk <= 0) {
        // (linear scenes: PTG_UNIT_ROUNDS rounds of the device's wave slots --
        // C1's 7,500 pixel groups in 6-sample units, 22,500 units: 12 %
        // faster than ~96k units of 2 samples, whose per-unit setup weighed)
        const long long target =
            ctx->n > kLinearMax ? PTG_BVH_UNIT_MULT * 98304 : (long long)PTG_UNIT_ROUNDS * ctx->wave_slots;
        long long want = (target + groups - 1) / groups;
        long long nch = want < 1 ? 1 : (want > nsamp ? nsamp : want);
        chunk = nch > 0 ? (int)((nsamp + nch - 1) / nch) : 1;
    }
    if (chunk > nsamp)
        chunk = nsamp > 0 ? nsamp : 1;
    if (chunk > kMaxChunk)  // the kernel's divmod_nv needs 64 * chunk <= 2^22 (the image does not depend on it)
        chunk = kMaxChunk;
    A.chunk = chunk;
    A.n_groups = groups;
    int n_chunks = nsamp > 0 ? (nsamp + chunk - 1) / chunk : 0;
    // in-wave resolve only when one unit holds ALL samples of its pixels
    A.single_chunk = !accumulate_only && n_chunks <= 1 && s_begin == 0 && s_end == p->samples;
    A.n_units = (long long)A.n_groups * n_chunks;
    A.n_levels = 1;
    A.lvl_group[0] = 0;
    A.lvl_group[1] = groups;
    A.lvl_chunk[0] = chunk;
    A.lvl_unit[0] = 0;
    A.lvl_unit[1] = A.n_units;
    for (int l = 0; l < kMaxLevels; ++l) {
        A.lvl_coop[l] = 0;
        A.lvl_psplit[l] = 1;
        A.lvl_inwave[l] = 0;
    }
    A.lvl_inwave[0] = A.single_chunk;
    A.resolve_row0 = 0;
    A.needs_resolve = !A.single_chunk;
    // Split tail: with whole-pixel units, the grid ends when its slowest last
    // units end (a unit is ~1/16 of the frame per wave slot here).  The last
    // rows -- about one round of the device's wave slots -- run instead as
    // shorter units, accumulated and resolved by resolve_kernel; everything
    // before keeps the in-wave resolve.  The tail's rows get shorter units
    // towards the end (PTG_TAIL_LEVELS levels: the first half of the tail
    // rows in PTG_TAIL_CHUNKS... chunks, see tail_level_chunks), so the last
    // units to start are the shortest.
    if (tail_ok && A.single_chunk) {
        const long long tail_slots = (long long)(ctx->n > kLinearMax ? PTG_BVH_TAIL_HALF_ROUNDS : PTG_LIN_TAIL_HALF_ROUNDS) *
                                     ctx->wave_slots / 2;
        int tail_rows = (int)((tail_slots + A.waves_per_row - 1) / A.waves_per_row);
        tail_rows = tail_rows < A.slab_rows ? tail_rows : A.slab_rows;
        const bool many = groups >= 5LL * ctx->wave_slots;
        // level row counts: halves of what is left, the last level takes the rest
        int rows_left = tail_rows, row = A.slab_rows - tail_rows;
        A.resolve_row0 = A.slab_rows;  // no accumulating level yet
        A.lvl_group[1] = row * A.waves_per_row;
        A.lvl_unit[1] = A.lvl_group[1];  // head: one unit per group
        int l = 1;
        constexpr int kLinWaves = kBlock / 64;
        for (; l <= PTG_TAIL_LEVELS && rows_left > 0; ++l) {
            const int rows = l == PTG_TAIL_LEVELS ? rows_left : (rows_left + 1) / 2;
            const int tc = (many ? (ctx->n > kLinearMax ? PTG_BVH_TAIL_CHUNKS_MANY : PTG_TAIL_CHUNKS_MANY)
                                 : PTG_TAIL_CHUNKS) << (l - 1);
            const int ch = (nsamp + tc - 1) / tc;
            const int nch = (nsamp + ch - 1) / ch;
            // one chunk per wave of a (linear-kernel) workgroup: the level's
            // sums stay in LDS; its first unit starts a workgroup
            const bool coop = ctx->n <= kLinearMax && nch == kLinWaves;
            // BVH kernel (one wave per workgroup, no cooperative level): the
            // pixel group split into as many units of interleaved pixels,
            // each with every sample -- the unit length of nch sample chunks,
            // resolved in the wave (C5: no HBM atomics, no resolve pass)
            const bool psplit = !coop && ctx->n > kLinearMax && l == 1 && nch > 1 &&
                                A.pixels_per_wave >= nch;
            if (coop)
                A.lvl_unit[l] = (A.lvl_unit[l] + kLinWaves - 1) / kLinWaves * kLinWaves;
            else if (!psplit && A.resolve_row0 == A.slab_rows)
                A.resolve_row0 = row;
            A.lvl_coop[l] = coop ? 1 : 0;
            A.lvl_psplit[l] = psplit ? nch : 1;
            A.lvl_inwave[l] = psplit ? 1 : 0;
            row += rows;
            rows_left -= rows;
            A.lvl_chunk[l] = psplit ? nsamp : ch;
            A.lvl_group[l + 1] = row * A.waves_per_row;
            A.lvl_unit[l + 1] = A.lvl_unit[l] + (long long)(A.lvl_group[l + 1] - A.lvl_group[l]) * nch;
        }
        A.n_levels = l;
        A.n_units = A.lvl_unit[l];
        A.needs_resolve = A.resolve_row0 < A.slab_rows;
        if (!A.needs_resolve)
            A.resolve_row0 = 0;
    }
#if PTG_BVH_HEAD_CHUNK > 0
    // BVH frames/shards below their split-tail threshold (e.g. 8-way shards
    // of C5): the head rows run in longer sample chunks -- fewer per-unit
    // pool tails -- and about the last round of wave slots' rows in the auto
    // chunk, so the grid still ends on short units.  Every unit accumulates;
    // resolve_kernel finishes all rows.
    else if (ctx->n > kLinearMax && p->chunk_samples <= 0 && !accumulate_only && s_begin == 0 &&
             s_end == p->samples && chunk < PTG_BVH_HEAD_CHUNK && chunk < nsamp) {
        const long long tslots = (long long)PTG_BVH_HEAD_TAIL_HALF_ROUNDS * ctx->wave_slots / 2;
        int tail_rows = (int)((tslots + A.waves_per_row - 1) / A.waves_per_row);
        if (tail_rows < A.slab_rows) {
            const int hc = PTG_BVH_HEAD_CHUNK < nsamp ? PTG_BVH_HEAD_CHUNK : nsamp;
            const int hn = (nsamp + hc - 1) / hc;
            const int row = A.slab_rows - tail_rows;
            A.lvl_chunk[0] = hc;
            A.lvl_group[1] = row * A.waves_per_row;
            A.lvl_unit[1] = (long long)A.lvl_group[1] * hn;
            const int tc = PTG_BVH_TAIL_CHUNK > 0 ? (PTG_BVH_TAIL_CHUNK < nsamp ? PTG_BVH_TAIL_CHUNK : nsamp) : chunk;
            const int tn = (nsamp + tc - 1) / tc;
            A.lvl_chunk[1] = tc;
            A.lvl_group[2] = groups;
            A.lvl_unit[2] = A.lvl_unit[1] + (long long)(groups - A.lvl_group[1]) * tn;
            A.n_levels = 2;
            A.n_units = A.lvl_unit[2];
            A.needs_resolve = 1;
        }
    }
#endif
    const int waves_per_block = (ctx->n > kLinearMax ? PTG_BVH_BLOCK : kBlock) / 64;
    const long long g = (A.n_units + waves_per_block - 1) / waves_per_block;  // 64-bit before any cast
    grid = 0;
    if (g > 0x7FFFFFFFLL)
        return fail(PTG_ERR_UNSUPPORTED, "too many work units (" + std::to_string(A.n_units) +
                                             "): raise chunk_samples or use 0 (auto)");
    grid = (int)g;
    return PTG_OK;
}

int set_device(int device)
{
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return fail(PTG_ERR_NO_DEVICE, "no HIP device visible");
    if (device >= count)
        return fail(PTG_ERR_INVALID_ARGUMENT, "device ordinal out of range");
    if (device >= 0)
        PTG_HIP(hipSetDevice(device));
    return PTG_OK;
}

}  // namespace

extern "C" {

// internal (csrc/ptg_multi.cpp): set the thread-local error of ptg_last_error
int ptg_set_error_(int code, const char *msg) { return fail(code, msg ? msg : ""); }

int ptg_abi_version(void) { return PTG_ABI_VERSION; }

#if PTG_UNIT_TRACE
// debug builds only: the per-unit trace of the launches since the last call
// (3 values per unit, see ptg_unit_trace; then zeroed)
int ptg_unit_trace_(unsigned long long *out, int n_units)
{
    const size_t n = (size_t)std::min(n_units, kTraceUnits) * 3;
    PTG_HIP(hipDeviceSynchronize());
    PTG_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(ptg_unit_trace), n * sizeof(unsigned long long)));
    std::vector<unsigned long long> z(n, 0ull);
    PTG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(ptg_unit_trace), z.data(), n * sizeof(unsigned long long)));
    return PTG_OK;
}
#endif
#if PTG_BLOCK_STATS
// debug builds only: the 16 block counters summed over their 256 slots (then zeroed)
int ptg_debug_stats2_(unsigned long long *out16)
{
    std::vector<unsigned long long> h(256 * 16);
    PTG_HIP(hipDeviceSynchronize());
    PTG_HIP(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(ptg_dbg_stats2), h.size() * sizeof(h[0])));
    for (int i = 0; i < 16; ++i) {
        out16[i] = 0;
        for (int b = 0; b < 256; ++b)
            out16[i] += h[b * 16 + i];
    }
    std::vector<unsigned long long> z(h.size(), 0ull);
    PTG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(ptg_dbg_stats2), z.data(), z.size() * sizeof(z[0])));
    return PTG_OK;
}
int ptg_debug_stats_(unsigned long long *out16)
{
    std::vector<unsigned long long> h(256 * 16);
    PTG_HIP(hipDeviceSynchronize());
    PTG_HIP(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(ptg_dbg_stats), h.size() * sizeof(h[0])));
    for (int i = 0; i < 16; ++i) {
        out16[i] = 0;
        for (int b = 0; b < 256; ++b)
            out16[i] += h[b * 16 + i];
    }
    std::vector<unsigned long long> z(h.size(), 0ull);
    PTG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(ptg_dbg_stats), z.data(), z.size() * sizeof(z[0])));
    return PTG_OK;
}
#endif

const char *ptg_last_error(void) { return g_last_error.c_str(); }

int ptg_device_count(int *count)
{
    if (!count)
        return fail(PTG_ERR_INVALID_ARGUMENT, "count is NULL");
    *count = 0;
    if (hipGetDeviceCount(count) != hipSuccess)
        *count = 0;
    return PTG_OK;
}

int ptg_shard_rows(int32_t height, int32_t band_rows, int32_t shard_count, int32_t *rows)
{
    if (!rows || height <= 0 || band_rows <= 0 || shard_count <= 0)
        return fail(PTG_ERR_INVALID_ARGUMENT, "invalid shard geometry");
    int bands = (height + band_rows - 1) / band_rows;
    *rows = ((bands + shard_count - 1) / shard_count) * band_rows;
    return PTG_OK;
}

int ptg_context_create(const ptg_sphere *spheres, size_t n_spheres, const ptg_camera *cam, int device,
                       ptg_context **out)
{
    if (!out || !cam || (n_spheres && !spheres))
        return fail(PTG_ERR_INVALID_ARGUMENT, "NULL argument");
    *out = nullptr;
    if (n_spheres > (size_t)(1 << 24))
        return fail(PTG_ERR_UNSUPPORTED, "too many spheres");
    for (size_t i = 0; i < n_spheres; ++i)
        if (!sphere_ok(spheres[i]))
            return fail(PTG_ERR_INVALID_ARGUMENT, "sphere " + std::to_string(i) + " is invalid");
    int rc = set_device(device);
    if (rc)
        return rc;
    int dev = 0;
    PTG_HIP(hipGetDevice(&dev));
    std::vector<GeoRec> geo, lgeo;
    std::vector<ShadeRec> shade, lshade;
    std::vector<int> axis;
    prepare_scene(spheres, (int)n_spheres, cam, geo, shade, axis);
    KArgs order{};
    const bool linear = (int)n_spheres <= kLinearMax;
    std::vector<LinRec> lin;
    if (linear) {  // the scan's record order, interleaved, + the no-hit sentinel
        prepare_scan_order(spheres, (int)n_spheres, cam, geo, shade, axis, lgeo, lshade, order);
        lin.resize(n_spheres + 2 + 2);  // + the box-mode wall table(s) (scene_scan)
        std::memset(lin.data(), 0, lin.size() * sizeof(LinRec));
        for (size_t i = 0; i < n_spheres; ++i)
            lin[i] = LinRec{lgeo[i], lshade[i]};
        int32_t walls[6];
        for (int k = 0; k < 3; ++k) {
            walls[2 * k] = order.rec_plus[k];
            walls[2 * k + 1] = order.rec_minus[k];
        }
        std::memcpy(&lin[n_spheres + 1], walls, sizeof(walls));
        // entry 2 k + side: the wall's geometry, g1.x = its record's byte
        // offset; a missing wall: NaN geometry (its test never wins), offset 0
        GeoRec wg[6];
        for (int e = 0; e < 6; ++e) {
            const float qnan = __builtin_nanf("");
            const int off = walls[e];
            if (order.box_mode && off >= 0 && off / (int)sizeof(LinRec) < (int)n_spheres) {
                wg[e] = lgeo[off / (int)sizeof(LinRec)];
                // the record's byte offset from the sentinel (scene_scan's
                // winner bi)
                const int32_t tag = (off / (int)sizeof(LinRec) - (int)n_spheres) * (int)sizeof(LinRec);
                std::memcpy(&wg[e].g1.x, &tag, 4);
            } else {
                wg[e].g0 = make_float4(qnan, qnan, qnan, qnan);
                wg[e].g1 = make_float4(0.0f, qnan, qnan, qnan);
            }
        }
        static_assert(sizeof(wg) <= 2 * sizeof(LinRec), "wall geometry table size");
        std::memcpy(&lin[n_spheres + 2], wg, sizeof(wg));
    }
    ptg_context *ctx = new ptg_context();
    ctx->device = dev;
    {
        hipDeviceProp_t prop;
        ctx->wave_slots = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount * 32 : 8192;
    }
    ctx->n = (int)n_spheres;
    // linear scenes: d_lin; BVH scenes: d_shade (scene index order) + d_bvh
    const size_t bytes = linear ? lin.size() * sizeof(LinRec) : std::max<size_t>(n_spheres, 1) * sizeof(ShadeRec);
    if (hipMalloc(linear ? (void **)&ctx->d_lin : (void **)&ctx->d_shade, bytes) != hipSuccess) {
        delete ctx;
        return fail(PTG_ERR_OUT_OF_MEMORY, "hipMalloc of the scene failed");
    }
    if (linear)
        PTG_HIP_OR_DESTROY(hipMemcpy(ctx->d_lin, lin.data(), bytes, hipMemcpyHostToDevice));
    else if (n_spheres) {
        std::vector<ShadeRec> up(shade.begin(), shade.begin() + n_spheres);
        PTG_HIP_OR_DESTROY(hipMemcpy(ctx->d_shade, up.data(), n_spheres * sizeof(ShadeRec), hipMemcpyHostToDevice));
    }
    {
        float tab[2 * kTrigEntries];
        trig_table(tab);
        if (hipMalloc(&ctx->d_trig, sizeof(tab)) != hipSuccess) {
            ptg_context_destroy(ctx);
            return fail(PTG_ERR_OUT_OF_MEMORY, "hipMalloc of the sin/cos table failed");
        }
        PTG_HIP_OR_DESTROY(hipMemcpy(ctx->d_trig, tab, sizeof(tab), hipMemcpyHostToDevice));
    }
    ctx->cam64 = *cam;
    if (n_spheres) {
        if (hipMalloc(&ctx->d_sph64, n_spheres * sizeof(ptg_sphere)) != hipSuccess) {
            ptg_context_destroy(ctx);
            return fail(PTG_ERR_OUT_OF_MEMORY, "hipMalloc of the scene (f64) failed");
        }
        PTG_HIP_OR_DESTROY(hipMemcpy(ctx->d_sph64, spheres, n_spheres * sizeof(ptg_sphere), hipMemcpyHostToDevice));
    }
    KArgs &A = ctx->base;
    std::memset(&A, 0, sizeof(A));
    A.trig = ctx->d_trig;
    A.lin = ctx->d_lin;
    A.shade = ctx->d_shade;
    A.n = (int)n_spheres;
    for (int k = 0; k < 3; ++k) {
        A.end_ax[k] = order.end_ax[k];
        A.pairs[k] = order.pairs[k];
        A.pair_lo[k] = order.pair_lo[k];
        A.pair_hi[k] = order.pair_hi[k];
        A.rec_plus[k] = order.rec_plus[k];
        A.rec_minus[k] = order.rec_minus[k];
        A.plane_plus[k] = order.plane_plus[k];
        A.plane_minus[k] = order.plane_minus[k];
    }
    A.box_mode = order.box_mode;
    A.end_big = order.end_big;
    A.box_walls_out = order.box_walls_out;
    A.room_nmr = room_neg_margin(A);
    if ((int)n_spheres > kLinearMax) {
        std::vector<char> huge(n_spheres);
        for (size_t i = 0; i < n_spheres; ++i)
            huge[i] = is_huge(spheres[i], cam);
        BvhBuild b = build_bvh(spheres, (int)n_spheres, huge);
        const size_t n_leaf = b.order.size(), n_big = b.big.size();
        // one allocation: leaf records | leaf ids | huge spheres | their ids |
        // the 8 interleaved wide layouts | their continuations
        const size_t off_geo = 0;
        const size_t off_id = off_geo + n_leaf * sizeof(float4);
        const size_t off_bgeo = (off_id + n_leaf * sizeof(int) + 15) & ~size_t(15);
        const size_t off_bid = off_bgeo + n_big * sizeof(GeoRec);
        const size_t off_q = (off_bid + n_big * sizeof(int) + 15) & ~size_t(15);
        const size_t n_recs = wide_bvh(b, 0, 0).size();  // records per layout
        // near-plane-first boxes: one layout per octant
        const size_t n_layouts = 8;
        const size_t stride = n_recs;  // (interleaved: 8 x n_recs records in all, no layout stride)
        const size_t off_cont = off_q + n_layouts * stride * sizeof(BvhNodeQ);
        const size_t total = off_cont + n_layouts * stride / kWide * sizeof(int32_t) + 16;
        std::vector<unsigned char> blob(total, 0);
        // the 8 layouts interleaved node by node: node j of layout k at
        // interleaved node 8 j + k, so the copies of one node share a 512-B
        // block instead of aliasing a power of two of records apart
        {
            auto ilv = [](int32_t local, int k) { return ((local >> 2) * 8 + k) * 4 + (local & 3); };
            for (int k = 0; k < 8; ++k) {
                std::vector<BvhNodeQ> qk = wide_bvh(b, k, 0);
                const std::vector<int32_t> ck = wide_conts(qk, 0);
                for (size_t r = 0; r < qk.size(); ++r) {
                    BvhNodeQ &z = qk[r];
                    if (z.word >= 0)
                        z.word = ilv(z.word, k);
                    std::memcpy(blob.data() + off_q + (size_t)ilv((int32_t)r, k) * sizeof(BvhNodeQ), &z, sizeof(z));
                }
                for (size_t j = 0; j < ck.size(); ++j) {
                    const int32_t c = ck[j] >= 0 ? ilv(ck[j], k) : ck[j];
                    std::memcpy(blob.data() + off_cont + (j * 8 + (size_t)k) * sizeof(int32_t), &c, sizeof(c));
                }
            }
        }
        const WideGrid wg(b.nodes.empty() ? BvhNodeHost{} : b.nodes[0]);
        for (int c = 0; c < 3; ++c) {
            A.q_lo[c] = wg.centre[c];
            A.q_scale[c] = wg.scale[c];
        }
        for (size_t i = 0; i < n_leaf; ++i) {
            const ptg_sphere &sp = spheres[b.order[i]];  // leaf record {C, -R^2}, as the GeoRec of a small sphere
            const float4 rec = make_float4((float)sp.position[0], (float)sp.position[1], (float)sp.position[2],
                                           (float)(-(sp.radius * sp.radius)));
            std::memcpy(blob.data() + off_geo + i * sizeof(float4), &rec, sizeof(float4));
            std::memcpy(blob.data() + off_id + i * sizeof(int), &b.order[i], sizeof(int));
        }
        for (size_t i = 0; i < n_big; ++i) {
            std::memcpy(blob.data() + off_bgeo + i * sizeof(GeoRec), &geo[b.big[i]], sizeof(GeoRec));
            std::memcpy(blob.data() + off_bid + i * sizeof(int), &b.big[i], sizeof(int));
        }
        if (hipMalloc(&ctx->d_bvh, total) != hipSuccess) {
            ptg_context_destroy(ctx);
            return fail(PTG_ERR_OUT_OF_MEMORY, "hipMalloc of the BVH failed");
        }
        PTG_HIP_OR_DESTROY(hipMemcpy(ctx->d_bvh, blob.data(), total, hipMemcpyHostToDevice));
        unsigned char *base = static_cast<unsigned char *>(ctx->d_bvh);
        A.bvh_qnodes = reinterpret_cast<const uint4 *>(base + off_q);
        A.bvh_cont = reinterpret_cast<const int *>(base + off_cont);
        A.bvh_sph = reinterpret_cast<const float4 *>(base + off_geo);
        A.bvh_id = reinterpret_cast<const int *>(base + off_id);
        A.big_geo = reinterpret_cast<const GeoRec *>(base + off_bgeo);
        A.big_id = reinterpret_cast<const int *>(base + off_bid);
        A.n_nodes = (int)n_recs;
        A.n_big = (int)n_big;
    }
    A.pos_x = (float)cam->position[0];
    A.pos_y = (float)cam->position[1];
    A.pos_z = (float)cam->position[2];
    A.base_x = (float)(cam->lower_left_corner[0] - cam->position[0]);
    A.base_y = (float)(cam->lower_left_corner[1] - cam->position[1]);
    A.base_z = (float)(cam->lower_left_corner[2] - cam->position[2]);
    A.X_x = (float)cam->cam_x_axis[0];
    A.X_y = (float)cam->cam_x_axis[1];
    A.X_z = (float)cam->cam_x_axis[2];
    A.Y_x = (float)cam->cam_y_axis[0];
    A.Y_y = (float)cam->cam_y_axis[1];
    A.Y_z = (float)cam->cam_y_axis[2];
    A.lens = (float)cam->lens_radius;
    *out = ctx;
    return PTG_OK;
}

int ptg_scene_layout(const ptg_sphere *spheres, size_t n_spheres, const ptg_camera *cam, int32_t *anchor_axis,
                     int32_t *scan_order)
{
    if (!cam || (n_spheres && (!spheres || !anchor_axis || !scan_order)))
        return fail(PTG_ERR_INVALID_ARGUMENT, "NULL argument");
    if (n_spheres > (size_t)(1 << 24))
        return fail(PTG_ERR_UNSUPPORTED, "too many spheres");
    const int n = (int)n_spheres;
    std::vector<GeoRec> geo;
    std::vector<ShadeRec> shade;
    std::vector<int> axis;
    prepare_scene(spheres, n, cam, geo, shade, axis);
    KArgs ends{};
    std::vector<int> order;
    if (n <= kLinearMax)
        order = scan_order_of(spheres, n, cam, axis, geo, ends);
    for (int i = 0; i < n; ++i)
        anchor_axis[i] = axis[i];
    for (int k = 0; k < 3 && n <= kLinearMax; ++k)
        if (ends.pairs[k])  // the pair leads axis k's group
            anchor_axis[order[k == 0 ? 0 : ends.end_ax[k - 1]]] = anchor_axis[order[(k == 0 ? 0 : ends.end_ax[k - 1]) + 1]] = k + 3;
    for (int i = 0; i < n; ++i)
        scan_order[i] = n <= kLinearMax ? order[i] : i;
    return PTG_OK;
}

int ptg_context_destroy(ptg_context *ctx)
{
    if (!ctx)
        return PTG_OK;
    (void)hipSetDevice(ctx->device);
    if (ctx->d_lin)
        (void)hipFree(ctx->d_lin);
    if (ctx->d_shade)
        (void)hipFree(ctx->d_shade);
    if (ctx->d_trig)
        (void)hipFree(ctx->d_trig);
    if (ctx->d_bvh)
        (void)hipFree(ctx->d_bvh);
    if (ctx->d_acc)
        (void)hipFree(ctx->d_acc);
    if (ctx->d_sph64)
        (void)hipFree(ctx->d_sph64);
    delete ctx;
    return PTG_OK;
}

}  // extern "C"

namespace {

// exact accumulator: allocated (zeroed) on first use at a size; resolve_kernel
// keeps it zero between one-shot frames.  The zeroing is queued on the launch
// stream: a hipMemset on the null stream is not ordered before kernels on a
// non-blocking stream (ptg_render_multi's), whose first frame could then add
// into a buffer being cleared (seen once as a differing box_mirror frame)
int ensure_acc(ptg_context *ctx, size_t need, hipStream_t stream)
{
    if (need <= ctx->acc_elems)
        return PTG_OK;
    if (ctx->d_acc)
        PTG_HIP(hipFree(ctx->d_acc));
    ctx->d_acc = nullptr;
    ctx->acc_elems = 0;
    if (hipMalloc(&ctx->d_acc, need * sizeof(unsigned long long)) != hipSuccess)
        return fail(PTG_ERR_OUT_OF_MEMORY, "hipMalloc of the accumulator failed");
    PTG_HIP(hipMemsetAsync(ctx->d_acc, 0, need * sizeof(unsigned long long), stream));
    ctx->acc_elems = need;
    ctx->acc_dirty = false;  // (a progressive frame in the old buffer is lost: reset before reuse)
    return PTG_OK;
}

size_t acc_elems_for(const KArgs &A) { return (size_t)A.slab_rows * A.W * A.lanes_per_pixel * 3; }

int launch_render(const KArgs &A, int grid, bool count, hipStream_t s)
{
    if (grid <= 0)
        return PTG_OK;
    const bool bvh = A.n > kLinearMax;
    const size_t lds = bvh ? 0 : (size_t)(A.n + 2 + 2) * sizeof(LinRec);
    // the exact mode's sin/cos table has its own LDS (render_kernel)
    const int sel = (count ? 4 : 0) | (bvh ? 2 : 0) | (A.exact_math ? 1 : 0);
    switch (sel) {
    case 0: render_kernel<false, false, false><<<grid, kBlock, lds, s>>>(A); break;
    case 1: render_kernel<false, false, true><<<grid, kBlock, lds, s>>>(A); break;
    case 2: render_kernel<false, true, false><<<grid, PTG_BVH_BLOCK, 0, s>>>(A); break;
    case 3: render_kernel<false, true, true><<<grid, PTG_BVH_BLOCK, 0, s>>>(A); break;
    case 4: render_kernel<true, false, false><<<grid, kBlock, lds, s>>>(A); break;
    case 5: render_kernel<true, false, true><<<grid, kBlock, lds, s>>>(A); break;
    case 6: render_kernel<true, true, false><<<grid, PTG_BVH_BLOCK, 0, s>>>(A); break;
    default: render_kernel<true, true, true><<<grid, PTG_BVH_BLOCK, 0, s>>>(A); break;
    }
    PTG_HIP(hipGetLastError());
    return PTG_OK;
}

// PTG_FLAG_REFERENCE_F64: the reference's double arithmetic (ref64.hpp), one
// lane per sub-pixel; out64 or out32 receives the slab
int launch_ref64(const ptg_context *ctx, const KArgs &A, double *out64, float *out32,
                 unsigned long long *d_segments, hipStream_t s)
{
    ref64::Args R{};
    R.spheres = ctx->d_sph64;
    R.n = ctx->n;
    R.cam = ctx->cam64;
    R.W = A.W;
    R.H = A.H;
    R.samps = A.samps;
    R.nsub = A.nsub;
    R.lanes_per_pixel = A.lanes_per_pixel;
    R.pixels_per_wave = A.pixels_per_wave;
    R.waves_per_row = A.waves_per_row;
    R.slab_rows = A.slab_rows;
    R.band_rows = A.band_rows;
    R.shard_rank = A.shard_rank;
    R.shard_count = A.shard_count;
    R.seed = A.seed;
    R.out64 = out64;
    R.out32 = out32;
    R.segments = d_segments;
    const long long waves = (long long)A.slab_rows * A.waves_per_row;
    const long long blocks = (waves + 3) / 4;
    if (blocks > 0x7FFFFFFFLL)
        return fail(PTG_ERR_UNSUPPORTED, "image too large for the reference-arithmetic mode");
    if (blocks > 0)
        ref64::render_kernel<<<(unsigned)blocks, 256, 0, s>>>(R);
    PTG_HIP(hipGetLastError());
    return PTG_OK;
}

int launch_resolve(const KArgs &A, hipStream_t s)
{
    long long pixels = (long long)(A.slab_rows - A.resolve_row0) * A.W;
    if (pixels <= 0)
        return PTG_OK;
    resolve_kernel<<<(unsigned)((pixels + 255) / 256), 256, 0, s>>>(A);
    PTG_HIP(hipGetLastError());
    return PTG_OK;
}

}  // namespace

extern "C" {

int ptg_render_device(ptg_context *ctx, const ptg_params *params, float *d_slab, unsigned long long *d_segments,
                      void *stream)
{
    if (!ctx || !d_slab)
        return fail(PTG_ERR_INVALID_ARGUMENT, "NULL context or output");
    int rc = check_params(params);
    if (rc)
        return rc;
    PTG_HIP(hipSetDevice(ctx->device));
    KArgs A;
    int grid = 0;
    if ((rc = fill_launch(ctx, params, A, grid)))
        return rc;
    if (params->flags & PTG_FLAG_REFERENCE_F64)
        return launch_ref64(ctx, A, nullptr, d_slab, d_segments, reinterpret_cast<hipStream_t>(stream));
    // several units per pixel, a split tail accumulated in HBM, or no samples at all
    const bool resolve = A.needs_resolve || grid == 0;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if ((rc = ensure_acc(ctx, resolve ? acc_elems_for(A) : 0, s)))
        return rc;
    A.out = d_slab;
    A.acc = ctx->d_acc;
    A.segments = d_segments;
    if (resolve && ctx->acc_dirty) {
        // progressive sums left by accumulate / keep_acc resolve: a one-shot
        // frame starts from zero (its resolve leaves the buffer zero again)
        PTG_HIP(hipMemsetAsync(ctx->d_acc, 0, ctx->acc_elems * sizeof(unsigned long long), s));
        ctx->acc_dirty = false;
    }
    if ((rc = launch_render(A, grid, d_segments != nullptr, s)))
        return rc;
    return resolve ? launch_resolve(A, s) : PTG_OK;
}

int ptg_launch_info(ptg_context *ctx, const ptg_params *params, int64_t *info, int n_info)
{
    if (!ctx || !info || n_info < 1)
        return fail(PTG_ERR_INVALID_ARGUMENT, "launch_info: NULL argument");
    int rc = check_params(params);
    if (rc)
        return rc;
    KArgs A;
    int grid = 0;
    if ((rc = fill_launch(ctx, params, A, grid)))
        return rc;
    const bool bvh = ctx->n > kLinearMax;
    const int64_t v[PTG_LAUNCH_INFO_COUNT] = {
        bvh ? 0 : A.box_mode, bvh ? 0 : A.box_walls_out, bvh ? 1 : 0, A.n_units, grid, A.n_levels,
        A.needs_resolve ? 1 : 0, (int64_t)(A.pairs[0] | (A.pairs[1] << 1) | (A.pairs[2] << 2))};
    for (int i = 0; i < n_info; ++i)
        info[i] = i < PTG_LAUNCH_INFO_COUNT ? v[i] : 0;
    return PTG_OK;
}

int ptg_accumulate_device(ptg_context *ctx, const ptg_params *params, int32_t sample_begin, int32_t sample_end,
                          unsigned long long *d_segments, void *stream)
{
    if (!ctx)
        return fail(PTG_ERR_INVALID_ARGUMENT, "NULL context");
    int rc = check_params(params);
    if (rc)
        return rc;
    if (sample_begin < 0 || sample_end < sample_begin || sample_end > params->samples)
        return fail(PTG_ERR_INVALID_ARGUMENT, "sample range must satisfy 0 <= begin <= end <= samples");
    if (params->flags & PTG_FLAG_REFERENCE_F64)
        return fail(PTG_ERR_UNSUPPORTED, "progressive passes are fp32 only (the reference-arithmetic mode sums "
                                         "its samples sequentially, main.cpp:192)");
    PTG_HIP(hipSetDevice(ctx->device));
    KArgs A;
    int grid = 0;
    if ((rc = fill_launch(ctx, params, A, grid, sample_begin, sample_end, /*accumulate_only=*/true)))
        return rc;
    if ((rc = ensure_acc(ctx, acc_elems_for(A), reinterpret_cast<hipStream_t>(stream))))
        return rc;
    A.acc = ctx->d_acc;
    A.segments = d_segments;
    ctx->acc_dirty = true;
    return launch_render(A, grid, d_segments != nullptr, reinterpret_cast<hipStream_t>(stream));
}

int ptg_resolve_device(ptg_context *ctx, const ptg_params *params, int32_t samples_done, float *d_slab, void *stream)
{
    if (!ctx || !d_slab)
        return fail(PTG_ERR_INVALID_ARGUMENT, "NULL context or output");
    int rc = check_params(params);
    if (rc)
        return rc;
    if (samples_done < 0 || samples_done > params->samples)
        return fail(PTG_ERR_INVALID_ARGUMENT, "samples_done must be in [0, samples]");
    PTG_HIP(hipSetDevice(ctx->device));
    KArgs A;
    int grid = 0;
    if ((rc = fill_launch(ctx, params, A, grid)))
        return rc;
    if ((rc = ensure_acc(ctx, acc_elems_for(A), reinterpret_cast<hipStream_t>(stream))))
        return rc;
    A.samps = samples_done;  // mean over the samples accumulated so far
    A.keep_acc = 1;
    A.resolve_row0 = 0;  // every row (the one-shot split tail does not apply here)
    A.acc = ctx->d_acc;
    A.out = d_slab;
    return launch_resolve(A, reinterpret_cast<hipStream_t>(stream));
}

int ptg_reset_accumulation_device(ptg_context *ctx, const ptg_params *params, void *stream)
{
    if (!ctx)
        return fail(PTG_ERR_INVALID_ARGUMENT, "NULL context");
    int rc = check_params(params);
    if (rc)
        return rc;
    PTG_HIP(hipSetDevice(ctx->device));
    KArgs A;
    int grid = 0;
    if ((rc = fill_launch(ctx, params, A, grid)))
        return rc;
    if ((rc = ensure_acc(ctx, acc_elems_for(A), reinterpret_cast<hipStream_t>(stream))))
        return rc;
    PTG_HIP(hipMemsetAsync(ctx->d_acc, 0, ctx->acc_elems * sizeof(unsigned long long),
                           reinterpret_cast<hipStream_t>(stream)));
    ctx->acc_dirty = false;
    return PTG_OK;
}

int ptg_trace_samples_device(ptg_context *ctx, const ptg_params *params, const int32_t *d_coords, size_t n,
                             float *d_out, int32_t *d_segs, void *stream)
{
    if (!ctx || (n && (!d_coords || !d_out || !d_segs)))
        return fail(PTG_ERR_INVALID_ARGUMENT, "NULL argument");
    int rc = check_params(params);
    if (rc)
        return rc;
    if (n == 0)
        return PTG_OK;
    if (params->flags & PTG_FLAG_REFERENCE_F64)
        return fail(PTG_ERR_UNSUPPORTED, "trace_samples probes the fp32 kernel");
    PTG_HIP(hipSetDevice(ctx->device));
    KArgs A;
    int grid = 0;
    if ((rc = fill_launch(ctx, params, A, grid)))
        return rc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int blocks = (int)((n + kTraceBlock - 1) / kTraceBlock);
    const bool bvh = A.n > kLinearMax;
    if (A.exact_math)
        bvh ? trace_kernel<true, true><<<blocks, kTraceBlock, 0, s>>>(A, d_coords, (int)n, d_out, d_segs)
            : trace_kernel<false, true><<<blocks, kTraceBlock, 0, s>>>(A, d_coords, (int)n, d_out, d_segs);
    else
        bvh ? trace_kernel<true, false><<<blocks, kTraceBlock, 0, s>>>(A, d_coords, (int)n, d_out, d_segs)
            : trace_kernel<false, false><<<blocks, kTraceBlock, 0, s>>>(A, d_coords, (int)n, d_out, d_segs);
    PTG_HIP(hipGetLastError());
    return PTG_OK;
}

int ptg_math_probe_device(ptg_context *ctx, int32_t op, int32_t exact, const float *d_in, float *d_out, size_t n,
                          void *stream)
{
    if (!ctx || (n && (!d_in || !d_out)))
        return fail(PTG_ERR_INVALID_ARGUMENT, "NULL argument");
    if (op < PTG_PROBE_SQRT || op > PTG_PROBE_SINCOS)
        return fail(PTG_ERR_INVALID_ARGUMENT, "unknown probe op");
    if (n > (size_t)INT32_MAX / 2)
        return fail(PTG_ERR_UNSUPPORTED, "too many operands");
    if (n == 0)
        return PTG_OK;
    PTG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const unsigned blocks = (unsigned)((n + 255) / 256);
    if (exact)
        math_probe_kernel<true><<<blocks, 256, 0, s>>>(op, d_in, d_out, (int)n, ctx->d_trig);
    else
        math_probe_kernel<false><<<blocks, 256, 0, s>>>(op, d_in, d_out, (int)n, ctx->d_trig);
    PTG_HIP(hipGetLastError());
    return PTG_OK;
}

int ptg_unshard_device(const float *d_gathered, float *d_image, int32_t width, int32_t height, int32_t band_rows,
                       int32_t shard_count, void *stream)
{
    if (!d_gathered || !d_image || width <= 0 || height <= 0 || band_rows <= 0 || shard_count <= 0)
        return fail(PTG_ERR_INVALID_ARGUMENT, "invalid unshard arguments");
    if (height > 65535)
        return fail(PTG_ERR_UNSUPPORTED, "height > 65535");
    int32_t slab_rows = 0;
    ptg_shard_rows(height, band_rows, shard_count, &slab_rows);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int bx = std::max(1, std::min(64, (width * 3 + 255) / 256));
    unshard_kernel<<<dim3(bx, height), 256, 0, s>>>(d_gathered, d_image, width, band_rows, shard_count, slab_rows);
    PTG_HIP(hipGetLastError());
    return PTG_OK;
}

int ptg_tonemap_device(const float *d_image, uint8_t *d_out, size_t count, void *stream)
{
    if (!d_image || !d_out)
        return fail(PTG_ERR_INVALID_ARGUMENT, "NULL argument");
    if (count == 0)
        return PTG_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    size_t blocks = (count + 255) / 256;
    tonemap_kernel<<<(unsigned)blocks, 256, 0, s>>>(d_image, d_out, count);
    PTG_HIP(hipGetLastError());
    return PTG_OK;
}

int ptg_render(const ptg_sphere *spheres, size_t n_spheres, const ptg_camera *cam, const ptg_params *params,
               int device, double *image_rgb)
{
    if (!image_rgb)
        return fail(PTG_ERR_INVALID_ARGUMENT, "image is NULL");
    int rc = check_params(params);
    if (rc)
        return rc;
    ptg_context *ctx = nullptr;
    rc = ptg_context_create(spheres, n_spheres, cam, device, &ctx);
    if (rc)
        return rc;
    int32_t slab_rows = 0;
    ptg_shard_rows(params->height, params->band_rows, params->shard_count, &slab_rows);
    size_t slab_elems = (size_t)slab_rows * params->width * 3;
    // the reference-arithmetic mode keeps its doubles to the host image
    const bool f64 = (params->flags & PTG_FLAG_REFERENCE_F64) != 0;
    const size_t esz = f64 ? sizeof(double) : sizeof(float);
    void *d_slab = nullptr;
    std::vector<unsigned char> host(slab_elems * esz);
    rc = PTG_OK;
    if (hipMalloc(&d_slab, slab_elems * esz) != hipSuccess) {
        ptg_context_destroy(ctx);
        return fail(PTG_ERR_OUT_OF_MEMORY, "hipMalloc of the image slab failed");
    }
    if (f64) {
        KArgs A;
        int grid = 0;
        rc = fill_launch(ctx, params, A, grid);
        if (rc == PTG_OK)
            rc = launch_ref64(ctx, A, static_cast<double *>(d_slab), nullptr, nullptr, nullptr);
    } else {
        rc = ptg_render_device(ctx, params, static_cast<float *>(d_slab), nullptr, nullptr);
    }
    if (rc == PTG_OK) {
        hipError_t e = hipDeviceSynchronize();
        if (e == hipSuccess)
            e = hipMemcpy(host.data(), d_slab, slab_elems * esz, hipMemcpyDeviceToHost);
        if (e != hipSuccess)
            rc = fail(PTG_ERR_HIP, std::string("render: ") + hipGetErrorString(e));
    }
    (void)hipFree(d_slab);
    ptg_context_destroy(ctx);
    if (rc)
        return rc;
    const int W = params->width, H = params->height, BR = params->band_rows;
    for (int j = 0; j < slab_rows; ++j) {
        int band = j / BR;
        int r = (band * params->shard_count + params->shard_rank) * BR + (j - band * BR);
        if (r >= H)
            continue;
        double *dst = image_rgb + (size_t)r * W * 3;
        const size_t off = (size_t)j * W * 3;
        for (int i = 0; i < W * 3; ++i)  // main.cpp:196: image[row] += ...
            dst[i] = dst[i] + (f64 ? reinterpret_cast<const double *>(host.data())[off + i]
                                   : (double)reinterpret_cast<const float *>(host.data())[off + i]);
    }
    return PTG_OK;
}

}  // extern "C"
