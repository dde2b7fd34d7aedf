// bvh_build.hpp -- host-side BVH over the scene's spheres (SURVEY.md 8(f) f3,
// README.md:8 "Implement a BVH for fast intersection testing").
//
// Huge spheres (R >= 1000, the anchored ones) stay in a small list tested
// linearly first (their boxes would cover everything); every other sphere
// goes into a binary BVH built with binned SAH splits (median split along
// the longest centroid axis where no plane separates the centroids), at most
// kLeafSize spheres per leaf.  Nodes are stored in
// depth-first order with a skip index (the node after the subtree), so the
// device walks it without a stack: hit -> i + 1, miss -> skip.
//
// Boxes are computed in double and widened before rounding to fp32 so that
// the traversal can never skip a sphere whose computed root could win: each
// side moves out by 1e-4 * (extent + |coordinate| + 1), far above the ~1e-6
// relative error of the fp32 root computation.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "../../include/ptgpu.h"

namespace ptg {

struct BvhNodeHost {
    float bmin[3];
    int32_t skip;  // index of the next node after this subtree
    float bmax[3];
    int32_t leaf;  // -1: inner node (children at i+1 ...); else first | count << 24 into the leaf-ordered sphere list
};
static_assert(sizeof(BvhNodeHost) == 32, "BVH node is two float4");

#ifndef PTG_BVH_SAH
#define PTG_BVH_SAH 1  // binned SAH splits (0: median split along the longest centroid axis)
#endif
#ifndef PTG_BVH_LEAF
#define PTG_BVH_LEAF 6  // 10,000-sphere scene, SAH + octant layouts: 6 beats 8 by 1.3 %, 5 and 7 by <1 %, 12 by 3 %
#endif
constexpr int kLeafSize = PTG_BVH_LEAF;

struct BvhBuild {
    std::vector<BvhNodeHost> nodes;
    std::vector<int32_t> order;  // leaf-ordered sphere indices (into the scene)
    std::vector<int32_t> big;    // huge spheres, tested linearly
    std::vector<int8_t> axis;    // per node: split axis of an inner node (its first child is the low side), -1 leaf
};

namespace detail {

inline float widen_down(double v, double pad) { return std::nextafter((float)(v - pad), -INFINITY); }
inline float widen_up(double v, double pad) { return std::nextafter((float)(v + pad), INFINITY); }

inline double half_area(const double mn[3], const double mx[3])
{
    const double x = mx[0] - mn[0], y = mx[1] - mn[1], z = mx[2] - mn[2];
    return x * y + y * z + z * x;
}

// Binned surface-area heuristic: centroids in kSahBins bins per axis, the
// split plane minimising A_left * N_left + A_right * N_right (sphere bounds).
// Partitions idx[lo, hi) (low side first), sets `axis`, returns the split
// index, or -1 when no plane separates the centroids (median split then).
#ifndef PTG_SAH_BINS
#define PTG_SAH_BINS 128  // C5: 27.42 -> 27.12 box tests per segment, 216.9 -> 216.2 ms (16: 27.80, 64: 27.29; A/B r05zt)
#endif
constexpr int kSahBins = PTG_SAH_BINS;
inline int sah_split(const ptg_sphere *s, std::vector<int32_t> &idx, int lo, int hi, const double cmn[3],
                     const double cmx[3], int &axis, double *cost_out = nullptr)
{
    double best = INFINITY;
    int best_axis = -1, best_bin = -1;
    for (int c = 0; c < 3; ++c) {
        const double ext = cmx[c] - cmn[c];
        if (!(ext > 0.0))
            continue;
        const double k = kSahBins / ext;
        int cnt[kSahBins] = {};
        double bmn[kSahBins][3], bmx[kSahBins][3];
        for (int b = 0; b < kSahBins; ++b)
            for (int j = 0; j < 3; ++j) {
                bmn[b][j] = INFINITY;
                bmx[b][j] = -INFINITY;
            }
        for (int i = lo; i < hi; ++i) {
            const ptg_sphere &sp = s[idx[i]];
            const int b = std::min(kSahBins - 1, (int)((sp.position[c] - cmn[c]) * k));
            cnt[b] += 1;
            for (int j = 0; j < 3; ++j) {
                bmn[b][j] = std::min(bmn[b][j], sp.position[j] - sp.radius);
                bmx[b][j] = std::max(bmx[b][j], sp.position[j] + sp.radius);
            }
        }
        // suffix areas/counts, then a prefix sweep over the kSahBins - 1 planes
        double rarea[kSahBins];
        int rcnt[kSahBins];
        double rmn[3] = {INFINITY, INFINITY, INFINITY}, rmx[3] = {-INFINITY, -INFINITY, -INFINITY};
        int rc = 0;
        for (int b = kSahBins - 1; b > 0; --b) {
            for (int j = 0; j < 3; ++j) {
                rmn[j] = std::min(rmn[j], bmn[b][j]);
                rmx[j] = std::max(rmx[j], bmx[b][j]);
            }
            rc += cnt[b];
            rcnt[b] = rc;
            rarea[b] = rc ? half_area(rmn, rmx) : 0.0;
        }
        double lmn[3] = {INFINITY, INFINITY, INFINITY}, lmx[3] = {-INFINITY, -INFINITY, -INFINITY};
        int lc = 0;
        for (int b = 0; b < kSahBins - 1; ++b) {
            for (int j = 0; j < 3; ++j) {
                lmn[j] = std::min(lmn[j], bmn[b][j]);
                lmx[j] = std::max(lmx[j], bmx[b][j]);
            }
            lc += cnt[b];
            if (lc == 0 || rcnt[b + 1] == 0)
                continue;
            const double cost = half_area(lmn, lmx) * lc + rarea[b + 1] * rcnt[b + 1];
            if (cost < best) {
                best = cost;
                best_axis = c;
                best_bin = b;
            }
        }
    }
    if (cost_out)
        *cost_out = best;
    if (best_axis < 0)
        return -1;
    axis = best_axis;
    const double k = kSahBins / (cmx[axis] - cmn[axis]);
    const auto it = std::partition(idx.begin() + lo, idx.begin() + hi, [&](int32_t a) {
        return std::min(kSahBins - 1, (int)((s[a].position[axis] - cmn[axis]) * k)) <= best_bin;
    });
    return (int)(it - idx.begin());
}

inline int build_rec(const ptg_sphere *s, std::vector<int32_t> &idx, int lo, int hi, BvhBuild &b)
{
    double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    double cmn[3] = {INFINITY, INFINITY, INFINITY}, cmx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = lo; i < hi; ++i) {
        const ptg_sphere &sp = s[idx[i]];
        for (int c = 0; c < 3; ++c) {
            mn[c] = std::min(mn[c], sp.position[c] - sp.radius);
            mx[c] = std::max(mx[c], sp.position[c] + sp.radius);
            cmn[c] = std::min(cmn[c], sp.position[c]);
            cmx[c] = std::max(cmx[c], sp.position[c]);
        }
    }
    const int me = (int)b.nodes.size();
    b.nodes.push_back(BvhNodeHost{});
    b.axis.push_back(-1);
    {
        BvhNodeHost &n = b.nodes[me];
        for (int c = 0; c < 3; ++c) {
            double pad = 1e-4 * ((mx[c] - mn[c]) + std::max(std::fabs(mn[c]), std::fabs(mx[c])) + 1.0);
            n.bmin[c] = widen_down(mn[c], pad);
            n.bmax[c] = widen_up(mx[c], pad);
        }
    }
#ifndef PTG_SAH_LEAF_CT
#define PTG_SAH_LEAF_CT 0  // > 0: a group of <= kLeafSize spheres is split too where the SAH says so (box test cost in sphere tests x 10; A/B)
#endif
    int mid = -1, axis = 0;
#if PTG_SAH_LEAF_CT > 0
    if (hi - lo <= kLeafSize && hi - lo >= 2) {
        double cost = INFINITY;
        const int m = sah_split(s, idx, lo, hi, cmn, cmx, axis, &cost);
        // split cost: two box tests more (the children's) + the children's
        // spheres weighted by their area, against every sphere of the leaf
        if (m > lo && m < hi && 0.2 * PTG_SAH_LEAF_CT * half_area(mn, mx) + cost < (hi - lo) * half_area(mn, mx))
            mid = m;
    }
    if (mid < 0 && hi - lo <= kLeafSize) {
#else
    if (hi - lo <= kLeafSize) {
#endif
        const int first = (int)b.order.size();
        for (int i = lo; i < hi; ++i)
            b.order.push_back(idx[i]);
        b.nodes[me].leaf = first | ((hi - lo) << 24);
        b.nodes[me].skip = me + 1;
        return me;
    }
    if (mid < 0) {
        axis = 0;
        for (int c = 1; c < 3; ++c)
            if (cmx[c] - cmn[c] > cmx[axis] - cmn[axis])
                axis = c;
#if PTG_BVH_SAH
        mid = sah_split(s, idx, lo, hi, cmn, cmx, axis);
#endif
    }
    if (mid < 0) {  // median split along the longest centroid axis
        mid = (lo + hi) / 2;
        std::nth_element(idx.begin() + lo, idx.begin() + mid, idx.begin() + hi, [&](int32_t a, int32_t c) {
            return s[a].position[axis] < s[c].position[axis] ||
                   (s[a].position[axis] == s[c].position[axis] && a < c);
        });
    }
    b.nodes[me].leaf = -1;
    b.axis[me] = (int8_t)axis;
    build_rec(s, idx, lo, mid, b);
    build_rec(s, idx, mid, hi, b);
    b.nodes[me].skip = (int)b.nodes.size();
    return me;
}

inline void order_rec(const BvhBuild &b, int i, int octant, std::vector<BvhNodeHost> &out)
{
    const int me = (int)out.size();
    out.push_back(b.nodes[i]);
    if (b.nodes[i].leaf >= 0) {
        out[me].skip = me + 1;
        return;
    }
    const int lo = i + 1, hi = b.nodes[lo].skip;
    const bool flip = (octant >> b.axis[i]) & 1;
    order_rec(b, flip ? hi : lo, octant, out);
    order_rec(b, flip ? lo : hi, octant, out);
    out[me].skip = (int)out.size();
}

}  // namespace detail

// The same tree in depth-first order for rays of one direction octant (bit k
// set: d_k < 0): at every inner node the child on the side the ray comes
// from is walked first, so the nearest hit usually shrinks the culling
// distance before the far child's boxes are tested.  Same nodes and leaves;
// skip indices recomputed.  Octant 0 is build_bvh's own order.
inline std::vector<BvhNodeHost> order_bvh(const BvhBuild &b, int octant)
{
    std::vector<BvhNodeHost> out;
    out.reserve(b.nodes.size());
    if (!b.nodes.empty())
        detail::order_rec(b, 0, octant, out);
    return out;
}

// Direction-sign bits worth a layout of their own (order_bvh): an axis
// whose splits carry under 5 % of the tree's weight (each inner node weighs
// its sphere count, so every level weighs about n) is dropped -- rays that
// differ only in that sign share a layout, which halves the nodes' cache
// footprint per dropped axis (10,000-sphere field, thin in y: 1 % faster).
inline int bvh_octant_mask(const BvhBuild &b)
{
    if (b.nodes.empty())
        return 0;
    std::vector<double> w(b.nodes.size(), 0.0);
    double per_axis[3] = {0.0, 0.0, 0.0}, total = 0.0;
    for (int i = (int)b.nodes.size() - 1; i >= 0; --i) {  // children follow their parent
        const BvhNodeHost &nd = b.nodes[i];
        if (nd.leaf >= 0) {
            w[i] = (double)(nd.leaf >> 24);
            continue;
        }
        const int lo = i + 1, hi = b.nodes[lo].skip;
        w[i] = w[lo] + w[hi];
        per_axis[b.axis[i]] += w[i];
        total += w[i];
    }
    int mask = 0;
    for (int k = 0; k < 3; ++k)
        if (total > 0.0 && per_axis[k] >= 0.05 * total)
            mask |= 1 << k;
    return mask;
}

// huge[i]: sphere i takes the anchored form (ptg_render.hip is_huge) and is
// tested linearly, outside the tree
inline BvhBuild build_bvh(const ptg_sphere *s, int n, const std::vector<char> &huge)
{
    BvhBuild b;
    std::vector<int32_t> idx;
    for (int i = 0; i < n; ++i) {
        if (huge[i])
            b.big.push_back(i);
        else
            idx.push_back(i);
    }
    if (!idx.empty())
        detail::build_rec(s, idx, 0, (int)idx.size(), b);
    return b;
}

// Compact 16-B nodes: the box quantised to 16 bits per coordinate on the
// root box's grid (rounded outward by one more step: conservative), and one
// word: >= 0 inner node's skip index, < 0 leaf (INT_MIN | count << 24 | first;
// a leaf's skip is the next node).  The kernel transforms the ray into grid
// units once per ray (t = q * (scale / d) + (lo - o) / d), so a node costs
// one 16-B load instead of two.
struct BvhNodeQ {
    uint32_t xy_min, z_min_x_max, y_max_z_max;
    int32_t word;
};
static_assert(sizeof(BvhNodeQ) == 16, "compact BVH node is one float4");

struct BvhGrid {
    float lo[3], scale[3];
};

// 16-bit box quantiser on the root box's grid (shared by the binary and the
// 4-wide layouts)
struct BvhQuantiser {
    double lo[3], sc[3];
    BvhGrid grid;
    explicit BvhQuantiser(const BvhNodeHost &root) : grid{}
    {
        for (int c = 0; c < 3; ++c) {
            lo[c] = root.bmin[c];
            const double ext = (double)root.bmax[c] - lo[c];
            sc[c] = ext > 0.0 ? ext / 65533.0 : 1e-30;
            grid.lo[c] = (float)lo[c];
            grid.scale[c] = (float)sc[c];
        }
    }
    uint32_t qlo(double v, int c) const
    {
        return (uint32_t)std::clamp(std::floor((v - lo[c]) / sc[c]) - 1.0, 0.0, 65535.0);
    }
    uint32_t qhi(double v, int c) const
    {
        return (uint32_t)std::clamp(std::ceil((v - lo[c]) / sc[c]) + 1.0, 0.0, 65535.0);
    }
    // flip bit k: axis k's planes swapped (far plane in the "min" field),
    // for rays with d_k < 0 -- the first field is then always the near plane
    BvhNodeQ box(const BvhNodeHost &n, int32_t word, int flip = 0) const
    {
        uint32_t a[3], b[3];
        for (int c = 0; c < 3; ++c) {
            a[c] = qlo(n.bmin[c], c);
            b[c] = qhi(n.bmax[c], c);
            if ((flip >> c) & 1)
                std::swap(a[c], b[c]);
        }
        BvhNodeQ q;
        q.xy_min = a[0] | (a[1] << 16);
        q.z_min_x_max = a[2] | (b[0] << 16);
        q.y_max_z_max = b[1] | (b[2] << 16);
        q.word = word;
        return q;
    }
};

inline BvhGrid quantise_bvh(const std::vector<BvhNodeHost> &nodes, std::vector<BvhNodeQ> &out)
{
    out.resize(nodes.size());
    if (nodes.empty())
        return BvhGrid{};
    const BvhQuantiser z(nodes[0]);
    for (size_t i = 0; i < nodes.size(); ++i) {
        const BvhNodeHost &n = nodes[i];
        out[i] = z.box(n, n.leaf >= 0 ? (int32_t)(0x80000000u | (uint32_t)n.leaf) : n.skip);
    }
    return z.grid;
}

// IEEE binary16 on the host (the wide layout's box planes): value of a bit
// pattern, and the largest / smallest finite half <= / >= a double.
inline double half_value(uint16_t h)
{
    const int e = (h >> 10) & 31, m = h & 1023;
    const double v = e == 0 ? std::ldexp((double)m, -24) : std::ldexp((double)(1024 + m), e - 25);
    return (h & 0x8000u) ? -v : v;
}
inline const std::vector<std::pair<double, uint16_t>> &half_table()
{
    static const std::vector<std::pair<double, uint16_t>> t = [] {
        std::vector<std::pair<double, uint16_t>> v;
        for (uint32_t h = 0; h < 65536; ++h)
            if (((h >> 10) & 31) != 31 && h != 0x8000u)  // finite, one zero
                v.emplace_back(half_value((uint16_t)h), (uint16_t)h);
        std::sort(v.begin(), v.end());
        return v;
    }();
    return t;
}
inline uint16_t half_floor(double x)
{
    const auto &t = half_table();
    auto it = std::upper_bound(t.begin(), t.end(), std::make_pair(x, (uint16_t)0xFFFF));
    return it == t.begin() ? t.front().second : std::prev(it)->second;
}
inline uint16_t half_ceil(double x)
{
    const auto &t = half_table();
    auto it = std::lower_bound(t.begin(), t.end(), std::make_pair(x, (uint16_t)0));
    return it == t.end() ? t.back().second : it->second;
}

// 4-wide tree (ptg_render.hip PTG_BVH_WIDE): each wide node is 4 consecutive
// 16-B records (one 64-B line), one per child -- the child's box and a word:
// >= 0 the child node's first record, < 0 a leaf (INT_MIN | count << 24 |
// first).  Box planes are binary16 values on a grid centred on the root box
// (plane = centre + h * scale, |h| <= 30000, rounded outward), so the kernel
// reads each one with a single v_fma_mix_f32 (no integer convert): words
// {near x, near y}, {near z, far x}, {far y, far z}, low half first.  The
// layout of octant k stores each box near-plane first for rays of that
// octant (axis c swapped when bit c of k is set).  Unused slots hold an empty
// leaf (count 0) whose box the octant's rays always miss (near plane beyond
// the far plane).  A wide node collapses up to three binary levels: starting
// from a binary node's two children it repeatedly opens the inner child with
// the largest surface, in place, so the children keep the binary tree's
// near-first order for the octant (order_bvh).  Nodes are in depth-first
// pre-order (a node's children follow it).
#ifndef PTG_BVH_ONE_LAYOUT
// 1: ONE wide layout for all ray octants (octant 0's child order, planes
// stored min first); the kernel puts each slab's near plane first per lane
// with one v_perm_b32 per axis.  0: one layout per octant (8 copies).
#define PTG_BVH_ONE_LAYOUT 0
#endif
#ifndef PTG_WIDE_N
#define PTG_WIDE_N 4  // children per wide node (the kernel's walk is written for 4; 8: design studies, tools/)
#endif
constexpr int kWide = PTG_WIDE_N;
constexpr int32_t kWideEmpty = (int32_t)0x80000000u;

struct WideGrid {
    float centre[3], scale[3];
    explicit WideGrid(const BvhNodeHost &root)
    {
        for (int c = 0; c < 3; ++c) {
            const double half = 0.5 * ((double)root.bmax[c] - (double)root.bmin[c]);
            centre[c] = (float)(0.5 * ((double)root.bmax[c] + (double)root.bmin[c]));
            scale[c] = half > 0.0 ? (float)(half / 30000.0) : 1e-30f;
        }
    }
    // plane value v in grid units, rounded outward (dir -1: down, +1: up),
    // checked against the decoded plane centre + h * scale
    uint16_t plane(double v, int c, int dir) const
    {
        const double g = (v - (double)centre[c]) / (double)scale[c];
        uint16_t h = dir < 0 ? half_floor(g) : half_ceil(g);
        // one more half step out while the decoded plane is inside (at most a
        // step or two: g's own rounding); child boxes lie in the root box, so
        // |g| stays far from the binary16 range end (65504)
        for (int k = 0; k < 64; ++k) {
            const double back = (double)centre[c] + half_value(h) * (double)scale[c];
            if (dir < 0 ? back <= v : back >= v)
                break;
            h = dir < 0 ? half_floor(std::nextafter(half_value(h), -INFINITY))
                        : half_ceil(std::nextafter(half_value(h), INFINITY));
        }
        return h;
    }
    BvhNodeQ box(const BvhNodeHost &n, int32_t word, int flip) const
    {
        uint32_t a[3], b[3];
        for (int c = 0; c < 3; ++c) {
            a[c] = plane(n.bmin[c], c, -1);
            b[c] = plane(n.bmax[c], c, +1);
            if ((flip >> c) & 1)
                std::swap(a[c], b[c]);
        }
        BvhNodeQ q;
        q.xy_min = a[0] | (a[1] << 16);
        q.z_min_x_max = a[2] | (b[0] << 16);
        q.y_max_z_max = b[1] | (b[2] << 16);
        q.word = word;
        return q;
    }
    BvhNodeQ empty(int flip) const
    {
        uint32_t a[3], b[3];
        for (int c = 0; c < 3; ++c) {
            const bool f = (flip >> c) & 1;
#if PTG_BVH_ONE_LAYOUT
            // one layout for every octant (the kernel orders each slab's planes
            // per lane): an inverted box would read as the whole grid, so the
            // empty slot is a point at grid value +60000 on every axis, outside
            // the root box (|h| <= 30000) -- a ray meets it only by passing
            // exactly through it, and then visits an empty leaf (count 0)
            (void)f;
            a[c] = b[c] = 0x7B53u;
#else
            a[c] = f ? 0xFB53u : 0x7B53u;  // near plane -/+60000 and far plane +/-60000: the
            b[c] = f ? 0x7B53u : 0xFB53u;  // octant's rays enter the slab after leaving it
#endif
        }
        BvhNodeQ q;
        q.xy_min = a[0] | (a[1] << 16);
        q.z_min_x_max = a[2] | (b[0] << 16);
        q.y_max_z_max = b[1] | (b[2] << 16);
        q.word = kWideEmpty;
        return q;
    }
};

// PTG_BVH_Q8 (ptg_render.hip): the same wide node in 48 B -- three 16-B
// loads per node step instead of four (the walk is bound by its load
// instructions: tools/node_width_bench.hip).  Dwords 0-3: the 4 child words;
// 4-5: the node's grid origin per axis as binary16 in units of 256 grid
// steps (x, y | z) and per axis F = E + 16 (5 bits at 16, 21, 26 of dword 5);
// 6-11: the 24 plane bytes q, plane = origin + q 2^E grid units, rounded
// outward from the binary16 planes of the 64-B record.  A child's planes are
// three pairs (near x, near y), (near z, far x), (far y, far z): pair 3 c + m.
// Dword i holds pairs 2 i (bytes 0, 2) and 2 i + 1 (bytes 1, 3), so one
// v_and_b32 / v_perm_b32 turns a pair into the binary16 pair {q_A, q_B}
// 2^-24 (subnormal halves, exact in v_fma_mix_f32): the kernel reads the
// planes as t = h (sx 2^(E + 24)) + (origin sx + bx) with the slab scale
// sx taken 256 times larger (KArgs::q_scale).  An empty slot: near q beyond
// far q for the octant (255 / 0, swapped on a flipped axis).
struct WideQ8 {
    uint32_t w[12];
};
inline WideQ8 wide_q8(const BvhNodeQ *r, int flip)
{
    WideQ8 o{};
    double lo[kWide][3], hi[kWide][3];
    double L[3] = {INFINITY, INFINITY, INFINITY}, H[3] = {-INFINITY, -INFINITY, -INFINITY};
    bool used[kWide];
    for (int c = 0; c < kWide; ++c) {
        used[c] = r[c].word != kWideEmpty;
        const uint32_t a[3] = {r[c].xy_min & 0xFFFFu, r[c].xy_min >> 16, r[c].z_min_x_max & 0xFFFFu};
        const uint32_t b[3] = {r[c].z_min_x_max >> 16, r[c].y_max_z_max & 0xFFFFu, r[c].y_max_z_max >> 16};
        for (int k = 0; k < 3; ++k) {
            const double n = half_value((uint16_t)a[k]), f = half_value((uint16_t)b[k]);
            const bool fl = (flip >> k) & 1;
            lo[c][k] = fl ? f : n;
            hi[c][k] = fl ? n : f;
            if (used[c]) {
                L[k] = std::min(L[k], lo[c][k]);
                H[k] = std::max(H[k], hi[c][k]);
            }
        }
    }
    uint16_t oh[3];
    int fe[3];
    uint8_t q[kWide][6];  // near x, y, z, far x, y, z
    for (int k = 0; k < 3; ++k) {
        if (!(L[k] <= H[k]))
            L[k] = H[k] = 0.0;  // no used child
        oh[k] = half_floor(L[k] / 256.0);
        const double O = 256.0 * half_value(oh[k]);  // <= L
        int E = -16;
        while (E < 15 && O + 255.0 * std::ldexp(1.0, E) < H[k])
            ++E;
        fe[k] = E + 16;
        const double D = std::ldexp(1.0, E);
        const bool fl = (flip >> k) & 1;
        for (int c = 0; c < kWide; ++c) {
            int ql, qh;
            if (used[c]) {
                ql = std::max(0, std::min(255, (int)std::floor((lo[c][k] - O) / D)));
                qh = std::max(0, std::min(255, (int)std::ceil((hi[c][k] - O) / D)));
                while (ql > 0 && O + ql * D > lo[c][k])  // exact in double: O a scaled binary16, D a power of two
                    --ql;
                while (qh < 255 && O + qh * D < hi[c][k])
                    ++qh;
            } else {  // empty: the octant's rays enter the slab after leaving it
                ql = 255;
                qh = 0;
            }
            q[c][k] = (uint8_t)(fl ? qh : ql);
            q[c][3 + k] = (uint8_t)(fl ? ql : qh);
        }
    }
    for (int c = 0; c < kWide; ++c)
        o.w[c] = (uint32_t)r[c].word;
    o.w[4] = (uint32_t)oh[0] | ((uint32_t)oh[1] << 16);
    o.w[5] = (uint32_t)oh[2] | ((uint32_t)fe[0] << 16) | ((uint32_t)fe[1] << 21) | ((uint32_t)fe[2] << 26);
    // pair p = 3 c + m: (near x, near y), (near z, far x), (far y, far z)
    static const int kA[3] = {0, 2, 4}, kB[3] = {1, 3, 5};
    for (int p = 0; p < 12; ++p) {
        const int c = p / 3, m = p % 3, i = p / 2, odd = p & 1;
        o.w[6 + i] |= ((uint32_t)q[c][kA[m]] << (8 * odd)) | ((uint32_t)q[c][kB[m]] << (16 + 8 * odd));
    }
    return o;
}

namespace detail {

inline void wide_children(const BvhBuild &b, int i, int octant, int kids[kWide], int &nk)
{
    auto ordered = [&](int node, int &first, int &second) {
        const int lo = node + 1, hi = b.nodes[lo].skip;
        const bool flip = (octant >> b.axis[node]) & 1;
        first = flip ? hi : lo;
        second = flip ? lo : hi;
    };
    nk = 2;
    ordered(i, kids[0], kids[1]);
    while (nk < kWide) {
        int pick = -1;
        double best = -1.0;
        for (int k = 0; k < nk; ++k) {
            const BvhNodeHost &c = b.nodes[kids[k]];
            if (c.leaf >= 0)
                continue;
            double mn[3], mx[3];
            for (int a = 0; a < 3; ++a) {
                mn[a] = c.bmin[a];
                mx[a] = c.bmax[a];
            }
            const double area = half_area(mn, mx);
            if (area > best) {
                best = area;
                pick = k;
            }
        }
        if (pick < 0)
            break;
        int f, s;
        ordered(kids[pick], f, s);
        for (int k = nk; k > pick + 1; --k)
            kids[k] = kids[k - 1];
        kids[pick] = f;
        kids[pick + 1] = s;
        ++nk;
    }
}

// emits binary node i (inner) as a wide node at out.size(); returns its first record
inline int wide_rec(const BvhBuild &b, int i, int octant, const WideGrid &z, int32_t base,
                    std::vector<BvhNodeQ> &out)
{
    const int me = (int)out.size();
    int kids[kWide], nk = 0;
    if (b.nodes[i].leaf >= 0) {  // a one-leaf tree: the root node holds the leaf
        kids[0] = i;
        nk = 1;
    } else {
        wide_children(b, i, octant, kids, nk);
    }
    out.resize(me + kWide);
    for (int k = nk; k < kWide; ++k)
        out[me + k] = z.empty(octant);
    for (int k = 0; k < nk; ++k) {
        const BvhNodeHost &c = b.nodes[kids[k]];
        int32_t word;
        if (c.leaf >= 0)
            word = (int32_t)(0x80000000u | (uint32_t)c.leaf);
        else
            word = base + wide_rec(b, kids[k], octant, z, base, out);
        out[me + k] = z.box(c, word, octant);
    }
    return me;
}

inline void wide_conts_rec(const std::vector<BvhNodeQ> &w, int32_t base, int node, int32_t cont,
                           std::vector<int32_t> &out)
{
    out[node / kWide] = cont;
    int used = 0;
    while (used < kWide && w[node + used].word != kWideEmpty)
        ++used;
    for (int k = 0; k < used; ++k)
        if (w[node + k].word >= 0)
            wide_conts_rec(w, base, w[node + k].word - base, k + 1 < used ? base + node + k + 1 : cont, out);
}

}  // namespace detail

// The 4-wide layout of the tree for rays of one direction octant; record
// words are offset by `base` (the layout's position in the device array).
// Empty for an empty tree.
inline std::vector<BvhNodeQ> wide_bvh(const BvhBuild &b, int octant, int32_t base)
{
    std::vector<BvhNodeQ> out;
    if (b.nodes.empty())
        return out;
    const WideGrid z(b.nodes[0]);
    detail::wide_rec(b, 0, octant, z, base, out);
    return out;
}

// Continuations of a wide layout, one per node (first record / 4): the
// position after the node's subtree in depth-first order -- the parent's
// first record + the next used slot (the walk resumes the parent from that
// slot), else the parent's continuation; -1 after the root.  The kernel's
// short stack falls back on them when it overflows.
inline std::vector<int32_t> wide_conts(const std::vector<BvhNodeQ> &w, int32_t base)
{
    std::vector<int32_t> out(w.size() / kWide, -1);
    if (!w.empty())
        detail::wide_conts_rec(w, base, 0, -1, out);
    return out;
}

}  // namespace ptg
