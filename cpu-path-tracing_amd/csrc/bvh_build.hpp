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
constexpr int kSahBins = 32;
inline int sah_split(const ptg_sphere *s, std::vector<int32_t> &idx, int lo, int hi, const double cmn[3],
                     const double cmx[3], int &axis)
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
    if (hi - lo <= kLeafSize) {
        const int first = (int)b.order.size();
        for (int i = lo; i < hi; ++i)
            b.order.push_back(idx[i]);
        b.nodes[me].leaf = first | ((hi - lo) << 24);
        b.nodes[me].skip = me + 1;
        return me;
    }
    int axis = 0;
    for (int c = 1; c < 3; ++c)
        if (cmx[c] - cmn[c] > cmx[axis] - cmn[axis])
            axis = c;
    int mid = -1;
#if PTG_BVH_SAH
    mid = sah_split(s, idx, lo, hi, cmn, cmx, axis);
#endif
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

inline BvhGrid quantise_bvh(const std::vector<BvhNodeHost> &nodes, std::vector<BvhNodeQ> &out)
{
    BvhGrid g{};
    out.resize(nodes.size());
    if (nodes.empty())
        return g;
    double lo[3], sc[3];
    for (int c = 0; c < 3; ++c) {
        lo[c] = nodes[0].bmin[c];
        const double ext = (double)nodes[0].bmax[c] - lo[c];
        sc[c] = ext > 0.0 ? ext / 65533.0 : 1e-30;
        g.lo[c] = (float)lo[c];
        g.scale[c] = (float)sc[c];
    }
    auto qlo = [&](double v, int c) { return (uint32_t)std::clamp(std::floor((v - lo[c]) / sc[c]) - 1.0, 0.0, 65535.0); };
    auto qhi = [&](double v, int c) { return (uint32_t)std::clamp(std::ceil((v - lo[c]) / sc[c]) + 1.0, 0.0, 65535.0); };
    for (size_t i = 0; i < nodes.size(); ++i) {
        const BvhNodeHost &n = nodes[i];
        BvhNodeQ &q = out[i];
        q.xy_min = qlo(n.bmin[0], 0) | (qlo(n.bmin[1], 1) << 16);
        q.z_min_x_max = qlo(n.bmin[2], 2) | (qhi(n.bmax[0], 0) << 16);
        q.y_max_z_max = qhi(n.bmax[1], 1) | (qhi(n.bmax[2], 2) << 16);
        q.word = n.leaf >= 0 ? (int32_t)(0x80000000u | (uint32_t)n.leaf) : n.skip;
    }
    return g;
}

}  // namespace ptg
