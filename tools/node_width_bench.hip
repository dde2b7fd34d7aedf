// node_width_bench.hip -- measurement tool (not product code): does the BVH
// walk's node-step time on gfx950 follow the number of 16-B loads per node
// (DESIGN.md §6 "C5")?  A 48-B node (3 x dwordx4) would need 8-bit planes
// or implicit child indices; this measures what it could buy before that is
// built.
//
// Each lane walks a chain of dependent node loads (the next node chosen from
// the loaded data, a 4-ary descent restarted every 7 steps over a 4 MB buffer:
// hot upper levels as in the BVH walk), K x dwordx4 per node (K = 1..4), and
// optionally W FMAs per step (4 independent chains) on the loaded words (the node step's
// box tests are ~85 VALU); also 3 x 16 B plus one 8-B or 4-B load (a node
// with 16-bit child words).  8 one-wave workgroups per SIMD, as the BVH kernel.
//
// Build + run (GPU box): hipcc --offload-arch=gfx950 -O3 -o /tmp/nwb tools/node_width_bench.hip && /tmp/nwb
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

constexpr int kNodes = 65536;  // 64 B slots: 4 MB
constexpr int kDepth = 7;

template <int K, int W>
__global__ __launch_bounds__(64, 8) void walk(const u32x4 *__restrict__ nodes, unsigned *out, int steps)
{
    const unsigned lane = threadIdx.x & 63;
    unsigned h = (blockIdx.x * 64u + lane) * 2654435761u;
    unsigned cur = 0u;
    float acc = (float)(lane & 7);
    for (int s = 0; s < steps; ++s) {
        const u32x4 *q = nodes + (size_t)cur * 4;
        unsigned x = h * 0x9E3779B1u;
#pragma unroll
        for (int k = 0; k < (K > 4 ? 3 : K); ++k) {
            const u32x4 v = q[k];
            x ^= (v.x + v.y * 3u + v.z * 5u + v.w * 7u) << k;
        }
        if constexpr (K == 5) {  // 3 x 16 B + 8 B
            typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 v = *reinterpret_cast<const u32x2 *>(q + 3);
            x ^= (v.x + v.y * 3u) << 3;
        } else if constexpr (K == 6) {  // 3 x 16 B + 4 B
            x ^= *reinterpret_cast<const unsigned *>(q + 3) << 3;
        }
        // W FMAs on the loaded bits (the box tests' arithmetic), in 4
        // independent chains (issue-bound, as the node step's tests)
        float f0 = __uint_as_float((x & 0x007FFFFFu) | 0x3F800000u), f1 = f0 + 1.0f, f2 = f0 + 2.0f, f3 = f0 + 3.0f;
#pragma unroll
        for (int w = 0; w < W / 4; ++w) {
            f0 = __builtin_fmaf(f0, 0.999f, acc);
            f1 = __builtin_fmaf(f1, 0.998f, acc);
            f2 = __builtin_fmaf(f2, 0.997f, acc);
            f3 = __builtin_fmaf(f3, 0.996f, acc);
        }
        acc = (f0 + f1 + f2 + f3) * 1e-3f;
        h = x ^ (x >> 15) ^ (unsigned)(acc > 1e30f);
        cur = (s % kDepth == kDepth - 1) ? 0u : ((cur * 4u + 1u + (h & 3u)) & (kNodes - 1));
    }
    out[blockIdx.x * 64 + lane] = h ^ cur;
}

template <int K, int W>
float run(const u32x4 *d_nodes, unsigned *d_out, int blocks, int steps)
{
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL((walk<K, W>), dim3(blocks), dim3(64), 0, 0, d_nodes, d_out, steps);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float t = 0;
        CHECK(hipEventElapsedTime(&t, e0, e1));
        if (rep > 0 && t < best)
            best = t;
    }
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return best;
}

int main(int argc, char **argv)
{
    const int steps = argc > 1 ? std::atoi(argv[1]) : 2000;
    const int blocks = 256 * 32;
    std::vector<unsigned> host((size_t)kNodes * 16);
    unsigned s = 12345u;
    for (auto &v : host) {
        s ^= s << 13;
        s ^= s >> 17;
        s ^= s << 5;
        v = s;
    }
    u32x4 *d_nodes;
    unsigned *d_out;
    CHECK(hipMalloc(&d_nodes, host.size() * 4));
    CHECK(hipMemcpy(d_nodes, host.data(), host.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&d_out, (size_t)blocks * 64 * 4));
    const double n = (double)blocks * 64 * steps;
    std::printf("node loads per step K x 16 B, W FMAs per step; ms for %d steps of %d lanes (best of 3)\n", steps,
                blocks * 64);
#define ROW2(W)                                                                                    \
    {                                                                                              \
        const float t5 = run<5, W>(d_nodes, d_out, blocks, steps), t6 = run<6, W>(d_nodes, d_out, blocks, steps); \
        const float t3 = run<3, W>(d_nodes, d_out, blocks, steps), t4 = run<4, W>(d_nodes, d_out, blocks, steps); \
        std::printf("W=%3d  3x16+8 B %.3f  3x16+4 B %.3f  3x16 B %.3f  4x16 B %.3f ms\n", W, t5, t6, t3, t4); \
    }
#define ROW(W)                                                                                     \
    {                                                                                              \
        const float t1 = run<1, W>(d_nodes, d_out, blocks, steps), t2 = run<2, W>(d_nodes, d_out, blocks, steps); \
        const float t3 = run<3, W>(d_nodes, d_out, blocks, steps), t4 = run<4, W>(d_nodes, d_out, blocks, steps); \
        std::printf("W=%3d  K=1 %.3f  K=2 %.3f  K=3 %.3f  K=4 %.3f ms   K=3/K=4 %.3f   (K=4: %.1f G steps/s)\n", W, \
                    t1, t2, t3, t4, t3 / t4, n / t4 / 1e6);                                          \
    }
    ROW(0)
    ROW(40)
    ROW(84)
    ROW2(0)
    ROW2(84)
    {  // a 48-B node whose decode costs ~20 VALU more per step vs today's 64-B node
        const float a = run<3, 104>(d_nodes, d_out, blocks, steps), b = run<4, 84>(d_nodes, d_out, blocks, steps);
        const float c = run<3, 124>(d_nodes, d_out, blocks, steps), e = run<4, 120>(d_nodes, d_out, blocks, steps);
        std::printf("3 x 16 B + 104 FMA %.3f ms vs 4 x 16 B + 84 FMA %.3f ms (%.3f); 3 x 16 B + 124 %.3f vs 4 x 16 B + 120 %.3f\n",
                    a, b, a / b, c, e);
    }
    return 0;
}
