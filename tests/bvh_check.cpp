// Host-side check of the BVH builder (cpu-path-tracing_amd/csrc/bvh_build.hpp),
// built and run by tests/test_bvh_builder.py with AddressSanitizer/UBSan.
// For random scenes it verifies the invariants the GPU traversal relies on
// (see ptg_render.hip: bvh_node_step):
//   * every non-huge sphere sits in exactly one leaf, huge spheres in `big`;
//   * depth-first layout: a node's subtree is the index range [i, skip);
//     leaves have skip = i + 1; inner nodes' children are i + 1 and the
//     node after the first child's subtree;
//   * every box contains its subtree's spheres (centre +- radius) and its
//     children's boxes (culling can never drop a candidate);
//   * the 16-bit quantised boxes, decoded on the grid, contain the float boxes;
//   * the 4-wide layouts (wide_bvh, PTG_BVH_WIDE): 4 records per node in
//     pre-order, every leaf reached exactly once from the root, each record's
//     decoded box contains its subtree's spheres, empty slots are count-0
//     leaves, and the children keep the binary tree's near-first order.
// Prints "ok <nodes>" per scene; exits non-zero on the first violation.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../cpu-path-tracing_amd/csrc/bvh_build.hpp"

using namespace ptg;

static int fails = 0;
#define CHECK(c, ...)                                                                              \
    do {                                                                                           \
        if (!(c)) {                                                                                \
            std::fprintf(stderr, __VA_ARGS__);                                                     \
            std::fprintf(stderr, "\n");                                                            \
            ++fails;                                                                               \
            return;                                                                                \
        }                                                                                          \
    } while (0)

// depth-first skip layout, leaf coverage and box containment of one layout
static void check_layout(const std::vector<ptg_sphere> &s, const BvhBuild &b, const std::vector<BvhNodeHost> &nodes,
                         int octant)
{
    const int nn = (int)nodes.size();
    CHECK(nn == (int)b.nodes.size(), "octant %d: %d nodes", octant, nn);
    std::vector<int> leaf_cover(b.order.size(), 0);
    for (int i = 0; i < nn; ++i) {
        const BvhNodeHost &nd = nodes[i];
        CHECK(nd.skip > i && nd.skip <= nn, "octant %d node %d skip %d", octant, i, nd.skip);
        if (nd.leaf >= 0) {
            CHECK(nd.skip == i + 1, "octant %d leaf %d skip %d", octant, i, nd.skip);
            const int first = nd.leaf & 0xFFFFFF, cnt = nd.leaf >> 24;
            CHECK(cnt >= 1 && cnt <= kLeafSize && first + cnt <= (int)b.order.size(), "leaf %d range", i);
            for (int k = first; k < first + cnt; ++k) {
                leaf_cover[k] += 1;
                const ptg_sphere &sp = s[b.order[k]];
                for (int c = 0; c < 3; ++c)
                    CHECK(nd.bmin[c] <= sp.position[c] - sp.radius && nd.bmax[c] >= sp.position[c] + sp.radius,
                          "octant %d leaf %d does not contain sphere %d (axis %d)", octant, i, b.order[k], c);
            }
        } else {
            CHECK(i + 1 < nd.skip, "octant %d inner node %d has no children", octant, i);
            const int l = i + 1, r = nodes[l].skip;
            CHECK(r < nd.skip && nodes[r].skip == nd.skip, "octant %d inner node %d children %d %d", octant, i, l, r);
            for (int ch : {l, r})
                for (int c = 0; c < 3; ++c)
                    CHECK(nd.bmin[c] <= nodes[ch].bmin[c] && nd.bmax[c] >= nodes[ch].bmax[c],
                          "octant %d node %d does not contain child %d", octant, i, ch);
        }
    }
    for (size_t k = 0; k < leaf_cover.size(); ++k)
        CHECK(leaf_cover[k] == 1, "octant %d leaf slot %zu covered %d times", octant, k, leaf_cover[k]);
}

// decoded box of a wide record (binary16 planes on the wide grid), in scene units
static void decode(const WideGrid &g, const BvhNodeQ &z, double lo[3], double hi[3])
{
    const uint16_t qv[6] = {(uint16_t)(z.xy_min & 0xFFFFu), (uint16_t)(z.xy_min >> 16),
                            (uint16_t)(z.z_min_x_max & 0xFFFFu), (uint16_t)(z.z_min_x_max >> 16),
                            (uint16_t)(z.y_max_z_max & 0xFFFFu), (uint16_t)(z.y_max_z_max >> 16)};
    for (int c = 0; c < 3; ++c) {  // stored near-first: swapped for d_c < 0
        const double a = g.centre[c] + half_value(qv[c]) * (double)g.scale[c];
        const double b = g.centre[c] + half_value(qv[3 + c]) * (double)g.scale[c];
        lo[c] = std::min(a, b);
        hi[c] = std::max(a, b);
    }
}

// walks wide node `node` (first record index, layout-relative): marks the
// leaves it reaches, checks boxes; returns the spheres' slots of its subtree
static void wide_walk(const std::vector<ptg_sphere> &s, const BvhBuild &b, const WideGrid &g,
                      const std::vector<BvhNodeQ> &w, int32_t base, int node, std::vector<int> &cover,
                      std::vector<int> &slots, int octant)
{
    CHECK(node >= 0 && node % kWide == 0 && node + kWide <= (int)w.size(), "octant %d wide node %d", octant, node);
    int used = 0;
    for (int k = 0; k < kWide; ++k) {
        const BvhNodeQ &r = w[node + k];
        std::vector<int> sub;
        if (r.word == kWideEmpty) {
            const BvhNodeQ e = g.empty(octant);
            CHECK(r.xy_min == e.xy_min && r.z_min_x_max == e.z_min_x_max && r.y_max_z_max == e.y_max_z_max,
                  "octant %d empty slot box", octant);
            continue;
        }
        CHECK(used == k, "octant %d node %d: empty slot before child %d", octant, node, k);
        ++used;
        if (r.word < 0) {
            const int leaf = r.word & 0x7FFFFFFF, first = leaf & 0xFFFFFF, cnt = leaf >> 24;
            CHECK(cnt >= 1 && cnt <= kLeafSize && first + cnt <= (int)b.order.size(), "octant %d wide leaf", octant);
            for (int j = first; j < first + cnt; ++j) {
                cover[j] += 1;
                sub.push_back(j);
            }
        } else {
            const int child = r.word - base;
            CHECK(child > node, "octant %d node %d child %d not after it (pre-order)", octant, node, child);
            wide_walk(s, b, g, w, base, child, cover, sub, octant);
            if (fails)
                return;
        }
        double lo[3], hi[3];
        decode(g, r, lo, hi);
        const double near_x = half_value((uint16_t)(r.xy_min & 0xFFFFu)), far_x = half_value((uint16_t)(r.z_min_x_max >> 16));
        CHECK((octant & 1) ? near_x >= far_x : near_x <= far_x, "octant %d: x planes not near-first", octant);
        for (int j : sub) {
            const ptg_sphere &sp = s[b.order[j]];
            for (int c = 0; c < 3; ++c)
                CHECK(lo[c] <= sp.position[c] - sp.radius && hi[c] >= sp.position[c] + sp.radius,
                      "octant %d node %d slot %d does not contain sphere %d", octant, node, k, b.order[j]);
        }
        slots.insert(slots.end(), sub.begin(), sub.end());
    }
    CHECK(used >= 1, "octant %d node %d has no children", octant, node);
}

static void check_wide(const std::vector<ptg_sphere> &s, const BvhBuild &b)
{
    if (b.nodes.empty()) {  // every sphere huge: no tree, no wide layout
        CHECK(wide_bvh(b, 0, 0).empty() && wide_conts(wide_bvh(b, 0, 0), 0).empty(), "empty tree: wide layout");
        return;
    }
    const WideGrid g(b.nodes[0]);
    for (int oct = 0; oct < 8 && !fails; ++oct) {
        const int32_t base = 1000 * oct;
        const std::vector<BvhNodeQ> w = wide_bvh(b, oct, base);
        CHECK(w.size() % kWide == 0 && !w.empty(), "octant %d: %zu wide records", oct, w.size());
        std::vector<int> cover(b.order.size(), 0), slots;
        wide_walk(s, b, g, w, base, 0, cover, slots, oct);
        for (size_t k = 0; k < cover.size() && !fails; ++k)
            CHECK(cover[k] == 1, "octant %d wide: leaf slot %zu reached %d times", oct, k, cover[k]);
        // continuations: a walk that enters every child and moves on only by
        // next-slot / continuation (the kernel's overflow fallback) reaches
        // every leaf once, in depth-first order
        if (!fails) {
            const std::vector<int32_t> cont = wide_conts(w, base);
            CHECK(cont.size() == w.size() / kWide && cont[0] == -1, "octant %d: continuation array", oct);
            std::vector<int> order;
            int32_t p = base, guard = 0;
            while (p != -1 && !fails && ++guard < 10 * (int)w.size()) {
                const int rel = p - base, node = rel & ~3, slot = rel & 3;
                CHECK(rel >= 0 && rel < (int)w.size() && w[rel].word != kWideEmpty, "octant %d: position %d", oct, p);
                const int32_t word = w[rel].word;
                if (word >= 0) {
                    p = word;
                    continue;
                }
                const int leaf = word & 0x7FFFFFFF;
                for (int j = 0; j < (leaf >> 24); ++j)
                    order.push_back((leaf & 0xFFFFFF) + j);
                p = slot + 1 < kWide && w[node + slot + 1].word != kWideEmpty ? p + 1 : cont[node / kWide];
            }
            CHECK(order == slots, "octant %d: continuation walk order", oct);
        }
        // near-first order: the binary layout of this octant visits the leaves
        // in the same order as the wide walk's depth-first child order
        if (!fails) {
            std::vector<int> bin;
            for (const BvhNodeHost &nd : order_bvh(b, oct))
                if (nd.leaf >= 0)
                    for (int j = 0; j < (nd.leaf >> 24); ++j)
                        bin.push_back((nd.leaf & 0xFFFFFF) + j);
            CHECK(bin == slots, "octant %d: wide child order differs from the binary near-first order", oct);
        }
    }
}

static void check_scene(const std::vector<ptg_sphere> &s)
{
    const int n = (int)s.size();
    std::vector<char> huge_flags(n);
    for (int i = 0; i < n; ++i)
        huge_flags[i] = s[i].radius >= 1000.0;
    BvhBuild b = build_bvh(s.data(), n, huge_flags);
    std::vector<int> seen(n, 0);
    for (int i : b.big)
        seen[i] += 1;
    for (int i : b.order)
        seen[i] += 10;
    for (int i = 0; i < n; ++i) {
        const bool huge = s[i].radius >= 1000.0;
        CHECK(seen[i] == (huge ? 1 : 10), "sphere %d placed %d (huge %d)", i, seen[i], (int)huge);
    }
    const int nn = (int)b.nodes.size();
    CHECK((int)b.axis.size() == nn, "axis per node");
    if (nn == 0) {
        check_wide(s, b);
        if (!fails)
            std::printf("ok %d spheres, all huge: empty tree\n", n);
        return;
    }
    check_layout(s, b, b.nodes, 0);
    // the 8 octant layouts (ptg_render.hip: one per ray-direction octant):
    // octant 0 is the build order; in octant k every inner node whose split
    // axis has bit k set lists its high-side child first
    for (int oct = 0; oct < 8 && !fails; ++oct) {
        const std::vector<BvhNodeHost> lay = order_bvh(b, oct);
        check_layout(s, b, lay, oct);
        if (oct == 0)
            for (int i = 0; i < nn; ++i)
                CHECK(lay[i].skip == b.nodes[i].skip && lay[i].leaf == b.nodes[i].leaf, "octant 0 node %d", i);
        if (!fails && nn > 1 && lay[0].leaf < 0) {
            const int first_child = b.axis[0] >= 0 && ((oct >> b.axis[0]) & 1) ? b.nodes[1].skip : 1;
            CHECK(lay[1].leaf == b.nodes[first_child].leaf && lay[1].bmin[0] == b.nodes[first_child].bmin[0],
                  "octant %d: root's first child", oct);
        }
    }
    if (fails)
        return;
    // quantised boxes contain the float boxes
    std::vector<BvhNodeQ> q;
    const BvhGrid g = quantise_bvh(b.nodes, q);
    CHECK(q.size() == b.nodes.size(), "quantised node count");
    for (int i = 0; i < nn; ++i) {
        const BvhNodeQ &z = q[i];
        const unsigned qv[6] = {z.xy_min & 0xFFFFu, z.xy_min >> 16, z.z_min_x_max & 0xFFFFu,
                                z.z_min_x_max >> 16, z.y_max_z_max & 0xFFFFu, z.y_max_z_max >> 16};
        const double lo[3] = {g.lo[0] + qv[0] * (double)g.scale[0], g.lo[1] + qv[1] * (double)g.scale[1],
                              g.lo[2] + qv[2] * (double)g.scale[2]};
        const double hi[3] = {g.lo[0] + qv[3] * (double)g.scale[0], g.lo[1] + qv[4] * (double)g.scale[1],
                              g.lo[2] + qv[5] * (double)g.scale[2]};
        for (int c = 0; c < 3; ++c)
            CHECK(lo[c] <= b.nodes[i].bmin[c] && hi[c] >= b.nodes[i].bmax[c], "quantised node %d axis %d", i, c);
        const BvhNodeHost &nd = b.nodes[i];
        if (nd.leaf >= 0)
            CHECK(z.word < 0 && (z.word & 0x7FFFFFFF) == nd.leaf, "quantised leaf word %d", i);
        else
            CHECK(z.word == nd.skip, "quantised skip %d", i);
    }
    check_wide(s, b);
    if (fails)
        return;
    const int mask = bvh_octant_mask(b);
    CHECK(nn <= 1 || (mask >= 0 && mask <= 7), "octant mask %d", mask);
    std::printf("ok %d spheres %d nodes %zu huge, 8 octant layouts (binary and 4-wide), octant mask %d\n", n, nn, b.big.size(), mask);
}

int main()
{
    std::mt19937 rng(1234);
    std::uniform_real_distribution<double> u(0.0, 1.0);
    for (int n : {2, 65, 300, 3000, 20000}) {
        std::vector<ptg_sphere> s(n);
        for (int i = 0; i < n; ++i) {
            ptg_sphere &sp = s[i];
            std::memset(&sp, 0, sizeof(sp));
            const bool huge = i % 97 == 0;  // a few huge spheres anywhere in the list
            sp.radius = huge ? 1e6 : 0.01 + 0.3 * u(rng);
            for (int c = 0; c < 3; ++c)
                sp.position[c] = huge ? (c == 1 ? -1e6 : 0.0) : -20.0 + 40.0 * u(rng);
            if (i % 7 == 0 && !huge)  // clusters of identical centres (median ties)
                for (int c = 0; c < 3; ++c)
                    sp.position[c] = 1.0;
            sp.material = i % 3;
        }
        check_scene(s);
        if (fails)
            return 1;
    }
    {  // every sphere huge: the BVH path with an empty tree
        std::vector<ptg_sphere> s(70);
        for (int i = 0; i < 70; ++i) {
            std::memset(&s[i], 0, sizeof(ptg_sphere));
            s[i].radius = 1000.0 + i;
            s[i].position[0] = 3000.0 * std::cos(i * 0.09);
            s[i].position[2] = 3000.0 * std::sin(i * 0.09);
        }
        check_scene(s);
        if (fails)
            return 1;
    }
    return 0;
}
