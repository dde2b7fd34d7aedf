// bvh_build.hpp -- host-side BVH over the scene's spheres (SURVEY.md 8(f) f3,
// README.md:8 "Implement a BVH for fast intersection testing").
//
// Huge spheres (R >= 1000, the anchored ones) stay in a small list tested
// linearly first (their boxes would cover everything); every other sphere
// goes into a binary BVH built by median split along the longest axis of the
// centroid bounds, at most kLeafSize spheres per leaf.  Nodes are stored in
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

#ifndef PTG_BVH_LEAF
#define PTG_BVH_LEAF 8  // measured on the 10,000-sphere scene: 8 beats 4 (-3.6 %) and 16 (+8.8 %)
#endif
constexpr int kLeafSize = PTG_BVH_LEAF;

struct BvhBuild {
    std::vector<BvhNodeHost> nodes;
    std::vector<int32_t> order;  // leaf-ordered sphere indices (into the scene)
    std::vector<int32_t> big;    // huge spheres, tested linearly
};

namespace detail {

inline float widen_down(double v, double pad) { return std::nextafter((float)(v - pad), -INFINITY); }
inline float widen_up(double v, double pad) { return std::nextafter((float)(v + pad), INFINITY); }

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
    const int mid = (lo + hi) / 2;
    std::nth_element(idx.begin() + lo, idx.begin() + mid, idx.begin() + hi, [&](int32_t a, int32_t c) {
        return s[a].position[axis] < s[c].position[axis] || (s[a].position[axis] == s[c].position[axis] && a < c);
    });
    b.nodes[me].leaf = -1;
    build_rec(s, idx, lo, mid, b);
    build_rec(s, idx, mid, hi, b);
    b.nodes[me].skip = (int)b.nodes.size();
    return me;
}

}  // namespace detail

inline BvhBuild build_bvh(const ptg_sphere *s, int n, double big_radius)
{
    BvhBuild b;
    std::vector<int32_t> idx;
    for (int i = 0; i < n; ++i) {
        if (s[i].radius >= big_radius)
            b.big.push_back(i);
        else
            idx.push_back(i);
    }
    if (!idx.empty())
        detail::build_rec(s, idx, 0, (int)idx.size(), b);
    return b;
}

}  // namespace ptg
