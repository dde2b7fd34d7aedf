// coop_load_bench.hip -- measurement tool (not product code): what the L1
// request count of the BVH kernel's node loads costs on gfx950, and what a
// cooperative load would save (DESIGN.md §6 "C5").
//
// Each lane walks a chain of dependent 64-B "node" loads (4 x dwordx4, the
// render kernel's node step), the next node chosen from the loaded data.
//   mode 0 (per lane): every lane loads its own node's 4 x 16 B -- the
//          render kernel today: each wave-level load touches up to 64 lines.
//   mode 1 (cooperative): the 4 lanes {p, p+16, p+32, p+48} (one per row of
//          16) load the 4 nodes of the group one after another, each
//          instruction one whole 64-B line per group (16 lines per wave-level
//          load), then a 4 x 4 transpose of 16-B chunks across the rows with
//          v_permlane32_swap + v_permlane16_swap (gfx950) gives every lane its
//          own node; the node addresses reach the group the same way.
// Both modes compute the same per-lane chain (checked).  Access pattern:
// `tree`: a 4-ary descent from the root (index 4i + 1 + (h & 3)) restarted
// every 7 steps over a 65,536-node (4 MB) buffer -- hot upper levels as in
// the BVH walk; `uniform`: uniformly random nodes over the buffer.
//
// Build + run (GPU box): hipcc --offload-arch=gfx950 -O3 -o /tmp/clb tools/coop_load_bench.hip && /tmp/clb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                           \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

constexpr int kNodes = 65536;  // 64 B each: 4 MB
constexpr int kDepth = 7;

__device__ __forceinline__ unsigned mixw(unsigned h, u32x4 a, u32x4 b, u32x4 c, u32x4 d)
{
    // every loaded dword feeds the next address (as the node step's tests do)
    unsigned x = h * 0x9E3779B1u;
    x ^= a.x + a.y * 3u + a.z * 5u + a.w * 7u;
    x ^= (b.x + b.y * 11u + b.z * 13u + b.w * 17u) << 1;
    x ^= (c.x + c.y * 19u + c.z * 23u + c.w * 29u) << 2;
    x ^= (d.x + d.y * 31u + d.z * 37u + d.w * 41u) << 3;
    return x ^ (x >> 15);
}

__device__ __forceinline__ unsigned next_node(unsigned cur, unsigned h, int step, int tree)
{
    if (!tree)
        return h & (kNodes - 1);
    if (step % kDepth == kDepth - 1)
        return 0u;  // restart at the root
    return (cur * 4u + 1u + (h & 3u)) & (kNodes - 1);
}

template <int kMode>
__global__ __launch_bounds__(64, 8) void walk(const u32x4 *__restrict__ nodes, unsigned *out, int steps, int tree)
{
    const unsigned lane = threadIdx.x & 63;
    unsigned h = (blockIdx.x * 64u + lane) * 2654435761u;
    unsigned cur = tree ? 0u : (h & (kNodes - 1));
    for (int s = 0; s < steps; ++s) {
        u32x4 a, b, c, d;
        if constexpr (kMode == 0) {
            const u32x4 *q = nodes + (size_t)cur * 4;
            a = q[0];
            b = q[1];
            c = q[2];
            d = q[3];
        } else {
            // the group's 4 node indices on every row: A_k = cur of row k
            unsigned A0 = cur, A1 = cur, A2 = cur, A3 = cur;
            {
                auto r02 = __builtin_amdgcn_permlane32_swap(A0, A2, false, false);
                auto r13 = __builtin_amdgcn_permlane32_swap(A1, A3, false, false);
                auto r01 = __builtin_amdgcn_permlane16_swap(r02[0], r13[0], false, false);
                auto r23 = __builtin_amdgcn_permlane16_swap(r02[1], r13[1], false, false);
                A0 = r01[0];
                A1 = r01[1];
                A2 = r23[0];
                A3 = r23[1];
            }
            const unsigned row = lane >> 4;  // chunk this lane loads
            u32x4 L0 = nodes[(size_t)A0 * 4 + row];
            u32x4 L1 = nodes[(size_t)A1 * 4 + row];
            u32x4 L2 = nodes[(size_t)A2 * 4 + row];
            u32x4 L3 = nodes[(size_t)A3 * 4 + row];
            // transpose: register k, row r -> register r, row k
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                auto x02 = __builtin_amdgcn_permlane32_swap(L0[j], L2[j], false, false);
                auto x13 = __builtin_amdgcn_permlane32_swap(L1[j], L3[j], false, false);
                auto y01 = __builtin_amdgcn_permlane16_swap(x02[0], x13[0], false, false);
                auto y23 = __builtin_amdgcn_permlane16_swap(x02[1], x13[1], false, false);
                L0[j] = y01[0];
                L1[j] = y01[1];
                L2[j] = y23[0];
                L3[j] = y23[1];
            }
            a = L0;
            b = L1;
            c = L2;
            d = L3;
        }
        h = mixw(h, a, b, c, d);
        cur = next_node(cur, h, s, tree);
    }
    out[blockIdx.x * 64 + lane] = h ^ cur;
}

int main(int argc, char **argv)
{
    const int steps = argc > 1 ? std::atoi(argv[1]) : 2000;
    const int blocks = 256 * 32;  // 8 one-wave workgroups per SIMD
    std::vector<unsigned> host((size_t)kNodes * 16);
    unsigned s = 12345u;
    for (auto &v : host) {
        s ^= s << 13;
        s ^= s >> 17;
        s ^= s << 5;
        v = s;
    }
    u32x4 *d_nodes;
    unsigned *d_out[2];
    CHECK(hipMalloc(&d_nodes, host.size() * 4));
    CHECK(hipMemcpy(d_nodes, host.data(), host.size() * 4, hipMemcpyHostToDevice));
    for (auto &p : d_out)
        CHECK(hipMalloc(&p, (size_t)blocks * 64 * 4));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int tree = 1; tree >= 0; --tree) {
        float ms[2] = {0, 0};
        for (int rep = 0; rep < 3; ++rep)
            for (int mode = 0; mode < 2; ++mode) {
                CHECK(hipEventRecord(e0));
                if (mode == 0)
                    hipLaunchKernelGGL(walk<0>, dim3(blocks), dim3(64), 0, 0, d_nodes, d_out[0], steps, tree);
                else
                    hipLaunchKernelGGL(walk<1>, dim3(blocks), dim3(64), 0, 0, d_nodes, d_out[1], steps, tree);
                CHECK(hipGetLastError());
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float t = 0;
                CHECK(hipEventElapsedTime(&t, e0, e1));
                if (rep > 0)
                    ms[mode] += t / 2;
            }
        std::vector<unsigned> o0((size_t)blocks * 64), o1((size_t)blocks * 64);
        CHECK(hipMemcpy(o0.data(), d_out[0], o0.size() * 4, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(o1.data(), d_out[1], o1.size() * 4, hipMemcpyDeviceToHost));
        const bool same = o0 == o1;
        const double n = (double)blocks * 64 * steps;
        std::printf("%-7s per-lane %.3f ms (%.2f G node loads/s)  cooperative %.3f ms (%.2f G/s)  ratio %.3f  %s\n",
                    tree ? "tree" : "uniform", ms[0], n / ms[0] / 1e6, ms[1], n / ms[1] / 1e6, ms[1] / ms[0],
                    same ? "same chains" : "CHAINS DIFFER");
        if (!same)
            return 2;
    }
    return 0;
}
