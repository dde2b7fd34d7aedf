// ptg_multi.cpp -- single-process multi-GPU frame: the
// drop-in ptg_render over several devices of one node, one RCCL gather.
//
// Replaces the taskflow row loop (src/main.cpp:214-236) for a C++ caller that
// owns several GPUs in one process (host/main.cpp --devices): device k renders
// the interleaved row bands b with b % n == k into a contiguous slab
// (ptg_render_device, shard_rank = k), ONE ncclGather (rccl.h:745, over xGMI
// between MI355X devices) collects the slabs on the first device, and
// ptg_unshard_device restores the row order there.  The RNG is keyed by the
// global pixel, so the image equals the one-device frame bit for bit.  The
// multi-process path (one rank per GPU, torch.distributed on RCCL) is
// ptgpu.render_sharded; both use the same slab layout and un-shard kernel.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/ptgpu.h"

namespace {

// ptg_last_error is thread-local in ptg_render.hip; errors raised here go
// through the same channel
extern "C" int ptg_set_error_(int code, const char *msg);

int fail(int code, const std::string &msg) { return ptg_set_error_(code, msg.c_str()); }

struct Device {
    int id = -1;
    ptg_context *ctx = nullptr;
    hipStream_t stream = nullptr;
    float *slab = nullptr;
    ncclComm_t comm = nullptr;
};

}  // namespace

extern "C" int ptg_render_multi(const ptg_sphere *spheres, size_t n_spheres, const ptg_camera *cam,
                                const ptg_params *params, const int *devices, int n_devices, double *image_rgb)
{
    if (!params || !image_rgb || !devices || n_devices < 1)
        return fail(PTG_ERR_INVALID_ARGUMENT, "render_multi: NULL argument or no device");
    if (params->shard_count != 1 || params->shard_rank != 0)
        return fail(PTG_ERR_INVALID_ARGUMENT, "render_multi shards the whole frame itself: shard_count must be 1");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return fail(PTG_ERR_NO_DEVICE, "no HIP device visible");
    for (int k = 0; k < n_devices; ++k) {
        if (devices[k] < 0 || devices[k] >= count)
            return fail(PTG_ERR_INVALID_ARGUMENT, "render_multi: device ordinal out of range");
        for (int j = 0; j < k; ++j)
            if (devices[j] == devices[k])
                return fail(PTG_ERR_UNSUPPORTED, "render_multi: RCCL needs distinct devices (one rank per GPU)");
    }
    const int W = params->width, H = params->height, BR = params->band_rows, n = n_devices;
    int32_t rows = 0;
    int rc = ptg_shard_rows(H, BR, n, &rows);
    if (rc)
        return rc;
    const size_t slab_elems = (size_t)rows * W * 3, image_elems = (size_t)W * H * 3;
    std::vector<Device> dv(n);
    float *gathered = nullptr, *d_image = nullptr;
    bool comms = false;
    auto cleanup = [&]() {
        for (Device &d : dv) {
            if (d.id < 0)
                continue;
            (void)hipSetDevice(d.id);
            if (d.stream)
                (void)hipStreamSynchronize(d.stream);
            if (comms && d.comm)
                (void)ncclCommDestroy(d.comm);
            if (d.slab)
                (void)hipFree(d.slab);
            if (d.stream)
                (void)hipStreamDestroy(d.stream);
            if (d.ctx)
                (void)ptg_context_destroy(d.ctx);
        }
        if (n > 0 && dv[0].id >= 0) {
            (void)hipSetDevice(dv[0].id);
            if (gathered)
                (void)hipFree(gathered);
            if (d_image)
                (void)hipFree(d_image);
        }
    };
#define PTG_MULTI_HIP(call)                                                                             \
    do {                                                                                                \
        hipError_t e_ = (call);                                                                         \
        if (e_ != hipSuccess) {                                                                         \
            cleanup();                                                                                  \
            return fail(PTG_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));                \
        }                                                                                               \
    } while (0)
#define PTG_MULTI_NCCL(call)                                                                            \
    do {                                                                                                \
        ncclResult_t r_ = (call);                                                                       \
        if (r_ != ncclSuccess) {                                                                        \
            cleanup();                                                                                  \
            return fail(PTG_ERR_HIP, std::string(#call) + ": " + ncclGetErrorString(r_));               \
        }                                                                                               \
    } while (0)
    // per device: the scene in HBM, a stream, the slab; the root also holds
    // the gathered slabs (rank-major) and the image
    for (int k = 0; k < n; ++k) {
        Device &d = dv[k];
        d.id = devices[k];
        if ((rc = ptg_context_create(spheres, n_spheres, cam, d.id, &d.ctx))) {
            cleanup();
            return rc;
        }
        PTG_MULTI_HIP(hipSetDevice(d.id));
        PTG_MULTI_HIP(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
        PTG_MULTI_HIP(hipMalloc(&d.slab, slab_elems * sizeof(float)));
        if (k == 0) {
            PTG_MULTI_HIP(hipMalloc(&gathered, (size_t)n * slab_elems * sizeof(float)));
            PTG_MULTI_HIP(hipMalloc(&d_image, image_elems * sizeof(float)));
        }
    }
    std::vector<ncclComm_t> cm(n);
    PTG_MULTI_NCCL(ncclCommInitAll(cm.data(), n, devices));
    comms = true;
    for (int k = 0; k < n; ++k)
        dv[k].comm = cm[k];
    // the shards render concurrently (asynchronous launches on each device)
    for (int k = 0; k < n; ++k) {
        ptg_params p = *params;
        p.shard_rank = k;
        p.shard_count = n;
        if ((rc = ptg_render_device(dv[k].ctx, &p, dv[k].slab, nullptr, dv[k].stream))) {
            cleanup();
            return rc;
        }
    }
    // ONE gather of equal-size slabs to the first device, fused across the
    // process's ranks in a group
    PTG_MULTI_NCCL(ncclGroupStart());
    for (int k = 0; k < n; ++k) {
        PTG_MULTI_HIP(hipSetDevice(dv[k].id));
        PTG_MULTI_NCCL(ncclGather(dv[k].slab, k == 0 ? gathered : nullptr, slab_elems, ncclFloat, 0, dv[k].comm,
                                  dv[k].stream));
    }
    PTG_MULTI_NCCL(ncclGroupEnd());
    PTG_MULTI_HIP(hipSetDevice(dv[0].id));
    if ((rc = ptg_unshard_device(gathered, d_image, W, H, BR, n, dv[0].stream))) {
        cleanup();
        return rc;
    }
    std::vector<float> host(image_elems);
    PTG_MULTI_HIP(hipMemcpyAsync(host.data(), d_image, image_elems * sizeof(float), hipMemcpyDeviceToHost,
                                 dv[0].stream));
    PTG_MULTI_HIP(hipStreamSynchronize(dv[0].stream));
    for (size_t i = 0; i < image_elems; ++i)
        image_rgb[i] = image_rgb[i] + (double)host[i];  // main.cpp:196: image[row] += ...
    cleanup();
    return PTG_OK;
#undef PTG_MULTI_HIP
#undef PTG_MULTI_NCCL
}
