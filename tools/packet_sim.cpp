// Packet walk of the 4-wide BVH for camera rays (design study for the BVH
// kernel): for the pixel groups of a frame (16 pixels x
// 2x2 sub-pixels = one wave), a wave-uniform walk that visits a node when
// ANY lane's ray hits it (per-lane culling distance), against each lane
// walking alone.  Prints per packet of 64 rays: node steps and leaf visits
// of the packet walk, and the sums of the per-ray walks.
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../cpu-path-tracing_amd/csrc/bvh_build.hpp"

using namespace ptg;

static double hit_sphere(const ptg_sphere &s, const double o[3], const double d[3])
{
    double e[3] = {o[0] - s.position[0], o[1] - s.position[1], o[2] - s.position[2]};
    const double a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    const double b = e[0] * d[0] + e[1] * d[1] + e[2] * d[2];
    const double c = e[0] * e[0] + e[1] * e[1] + e[2] * e[2] - s.radius * s.radius;
    const double disc = b * b - a * c;
    if (disc < 0)
        return INFINITY;
    const double sq = std::sqrt(disc);
    double t = (-b - sq) / a;
    if (t < 1e-4)
        t = (-b + sq) / a;
    return t < 1e-4 ? INFINITY : t;
}

static bool box_hit_d(const WideGrid &g, const BvhNodeQ &q, const double o[3], const double d[3], double tb)
{
    if (q.word == kWideEmpty)
        return false;
    const uint16_t qv[6] = {(uint16_t)(q.xy_min & 0xFFFFu), (uint16_t)(q.xy_min >> 16),
                            (uint16_t)(q.z_min_x_max & 0xFFFFu), (uint16_t)(q.z_min_x_max >> 16),
                            (uint16_t)(q.y_max_z_max & 0xFFFFu), (uint16_t)(q.y_max_z_max >> 16)};
    double tin = 0, tout = tb;
    for (int c = 0; c < 3; ++c) {
        const double a = g.centre[c] + half_value(qv[c]) * (double)g.scale[c];
        const double b = g.centre[c] + half_value(qv[3 + c]) * (double)g.scale[c];
        const double t1 = (a - o[c]) / d[c], t2 = (b - o[c]) / d[c];
        tin = std::max(tin, std::min(t1, t2));
        tout = std::min(tout, std::max(t1, t2));
    }
    return tin <= tout;
}

struct Ray {
    double o[3], d[3], tb;
};

int main(int argc, char **argv)
{
    FILE *f = std::fopen(argv[1], "rb");
    ptg_camera cam;
    int n = 0, W = 0, H = 0;
    if (!f || std::fread(&cam, sizeof(cam), 1, f) != 1 || std::fread(&W, 4, 1, f) != 1 || std::fread(&H, 4, 1, f) != 1 ||
        std::fread(&n, 4, 1, f) != 1)
        return 2;
    std::vector<ptg_sphere> s(n);
    if (std::fread(s.data(), sizeof(ptg_sphere), n, f) != (size_t)n)
        return 2;
    std::fclose(f);
    std::vector<char> huge(n);
    for (int i = 0; i < n; ++i)
        huge[i] = s[i].radius >= 1000.0;
    const BvhBuild b = build_bvh(s.data(), n, huge);
    const WideGrid g(b.nodes[0]);
    std::vector<std::vector<BvhNodeQ>> lay(8);
    for (int k = 0; k < 8; ++k)
        lay[k] = wide_bvh(b, k, 0);
    std::mt19937 rng(11);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    const int npk = argc > 2 ? std::atoi(argv[2]) : 4000;
    long pk_steps = 0, pk_leaves = 0, pk_sph = 0, lane_steps = 0, lane_sph = 0, rays = 0, other_oct = 0,
         pk_lane_active = 0;
    long hist_steps[8] = {0};
    for (int p = 0; p < npk; ++p) {
        const int y = (int)(U(rng) * H), x0 = 16 * (int)(U(rng) * (W / 16));
        Ray R[64];
        for (int l = 0; l < 64; ++l) {
            const int x = x0 + l / 4, sx = l & 1, sy = (l >> 1) & 1;
            const double fs = (x + 0.5 * sx + 0.5 * U(rng)) / W, ft = (y + 0.5 * sy + 0.5 * U(rng)) / H;
            for (int c = 0; c < 3; ++c) {
                R[l].o[c] = cam.position[c];
                R[l].d[c] = cam.lower_left_corner[c] + fs * cam.cam_x_axis[c] + ft * cam.cam_y_axis[c] - cam.position[c];
            }
            R[l].tb = INFINITY;
            for (int i : b.big)
                R[l].tb = std::min(R[l].tb, hit_sphere(s[i], R[l].o, R[l].d));
        }
        auto oct_of = [](const double *d) { return (d[0] < 0) | ((d[1] < 0) << 1) | ((d[2] < 0) << 2); };
        const int oct = oct_of(R[0].d);
        uint64_t lanes = 0;
        for (int l = 0; l < 64; ++l)
            if (oct_of(R[l].d) == oct)
                lanes |= 1ull << l;
            else
                ++other_oct;
        const std::vector<BvhNodeQ> &w = lay[oct];
        // per-lane walks (full stack, the kernel's visiting order)
        for (int l = 0; l < 64; ++l) {
            if (!((lanes >> l) & 1))
                continue;
            Ray r = R[l];
            std::vector<int> st{0};
            while (!st.empty()) {
                const int cur = st.back();
                st.pop_back();
                if (cur < -1) {
                    const int leaf = cur & 0x7FFFFFFF, first = leaf & 0xFFFFFF, cnt = leaf >> 24;
                    for (int j = first; j < first + cnt; ++j)
                        r.tb = std::min(r.tb, hit_sphere(s[b.order[j]], r.o, r.d));
                    lane_sph += cnt;
                    continue;
                }
                ++lane_steps;
                std::vector<int> hits;
                for (int k = 0; k < kWide; ++k)
                    if (box_hit_d(g, w[cur + k], r.o, r.d, r.tb))
                        hits.push_back(w[cur + k].word);
                for (int k = (int)hits.size() - 1; k >= 0; --k)
                    st.push_back(hits[k]);
            }
            ++rays;
        }
        // packet walk: visit a child when any lane hits it; leaves tested by every packet lane
        long steps = 0;
        std::vector<int> st{0};
        while (!st.empty()) {
            const int cur = st.back();
            st.pop_back();
            if (cur < -1) {
                const int leaf = cur & 0x7FFFFFFF, first = leaf & 0xFFFFFF, cnt = leaf >> 24;
                for (int l = 0; l < 64; ++l)
                    if ((lanes >> l) & 1)
                        for (int j = first; j < first + cnt; ++j)
                            R[l].tb = std::min(R[l].tb, hit_sphere(s[b.order[j]], R[l].o, R[l].d));
                ++pk_leaves;
                pk_sph += cnt;
                continue;
            }
            ++steps;
            std::vector<int> hits;
            for (int k = 0; k < kWide; ++k) {
                bool any = false;
                for (int l = 0; l < 64 && !any; ++l)
                    if ((lanes >> l) & 1)
                        any = box_hit_d(g, w[cur + k], R[l].o, R[l].d, R[l].tb);
                if (any)
                    hits.push_back(w[cur + k].word);
            }
            for (int l = 0; l < 64; ++l)  // lanes with at least one hit child (utilisation)
                if ((lanes >> l) & 1) {
                    bool h = false;
                    for (int k = 0; k < kWide && !h; ++k)
                        h = box_hit_d(g, w[cur + k], R[l].o, R[l].d, R[l].tb);
                    pk_lane_active += h;
                }
            for (int k = (int)hits.size() - 1; k >= 0; --k)
                st.push_back(hits[k]);
        }
        pk_steps += steps;
        hist_steps[std::min(7, (int)(steps / 8))] += 1;
    }
    std::printf("packets %d, rays %ld (other octant %ld)\n", npk, rays, other_oct);
    std::printf("per-lane walk: %.2f node steps, %.2f sphere tests per ray -> x64: %.1f, %.1f\n",
                (double)lane_steps / rays, (double)lane_sph / rays, 64.0 * lane_steps / rays, 64.0 * lane_sph / rays);
    std::printf("packet walk per packet: %.2f node steps (lanes with a hit child %.1f %%), %.2f leaves, %.2f sphere "
                "iterations\n",
                (double)pk_steps / npk, 100.0 * pk_lane_active / (64.0 * pk_steps), (double)pk_leaves / npk,
                (double)pk_sph / npk);
    std::printf("packet node steps histogram (bins of 8):");
    for (int k = 0; k < 8; ++k)
        std::printf(" %ld", hist_steps[k]);
    std::printf("\n");
    return 0;
}
