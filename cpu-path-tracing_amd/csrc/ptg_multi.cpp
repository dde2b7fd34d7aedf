// ptg_multi.cpp -- single-process multi-GPU frames: the
// drop-in ptg_render over several devices of one node, one RCCL gather.
//
// Replaces the taskflow row loop (src/main.cpp:214-236) for a C++ caller that
// owns several GPUs in one process (host/main.cpp --devices): device k renders
// the interleaved row bands b with b % n == k into a contiguous slab
// (ptg_render_device / ptg_resolve_device, shard_rank = k), ONE ncclGather
// (rccl.h:745, over xGMI between MI355X devices) collects the slabs on the
// first device, and ptg_unshard_device restores the row order there.  The RNG
// is keyed by the global pixel, so the image equals the one-device frame bit
// for bit.
//
// A ptg_multi holds, per device, the scene in HBM (a ptg_context), a
// non-blocking stream and the slab, the RCCL communicator of the device set
// (ncclCommInitAll once), and on the root the gathered slabs and the image:
// repeated frames and progressive passes reuse all of it.  ptg_render_multi is
// create + render + destroy.  The multi-process path (one rank per GPU,
// torch.distributed on RCCL) is ptgpu.render_sharded; all three use the same
// slab layout and un-shard kernel.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ptgpu.h"

// ptg_last_error is thread-local in ptg_render.hip; errors raised here go
// through the same channel
extern "C" int ptg_set_error_(int code, const char *msg);

namespace {

int fail(int code, const std::string &msg) { return ptg_set_error_(code, msg.c_str()); }

struct Shard {
    int id = -1;  // HIP device
    ptg_context *ctx = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;  // local transport: the slab is complete
    hipEvent_t t_begin = nullptr, t_rendered = nullptr;  // timing of the last device frame
    float *slab = nullptr;
    size_t slab_cap = 0;  // floats
    unsigned long long *counters = nullptr;  // PTG_FLAG_COUNT_TESTS: 4 per shard
    ncclComm_t comm = nullptr;
    bool stuck = false;  // destroy(): a broken group's stream did not drain
};

// Restores the calling thread's current HIP device on every return path.
struct DeviceGuard {
    int dev = -1;
    DeviceGuard()
    {
        if (hipGetDevice(&dev) != hipSuccess)
            dev = -1;
    }
    ~DeviceGuard()
    {
        if (dev >= 0)
            (void)hipSetDevice(dev);
    }
};

int hip_fail(const char *what, hipError_t e) { return fail(PTG_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e)); }
int nccl_fail(const char *what, ncclResult_t r)
{
    return fail(PTG_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}

#define MULTI_HIP(call)                                                                                 \
    do {                                                                                                \
        hipError_t e_ = (call);                                                                         \
        if (e_ != hipSuccess)                                                                           \
            return hip_fail(#call, e_);                                                                 \
    } while (0)

}  // namespace

struct ptg_multi {
    std::vector<Shard> shards;
    bool rccl = false;  // false: n shards on one device, gathered by device copies (tests)
    float *gathered = nullptr;  // root: n slabs, rank-major
    size_t gathered_cap = 0;
    float *image = nullptr;  // root: the un-sharded frame
    size_t image_cap = 0;
    std::vector<float> host;
    hipEvent_t t_unsharded = nullptr;  // root: the frame is un-sharded
    // the events and the image hold a completed ptg_multi_frame_device of this
    // size; cleared by every other frame call (render, passes, resolve), which
    // write the image or start frames the events do not describe
    bool timed = false;
    int32_t frame_w = 0, frame_h = 0, frame_band_rows = 0;
    // a failure inside the RCCL group: the communicators were aborted and the
    // context refuses further frames (PTG_ERR_HIP) until destroyed
    bool broken = false;
    int inject_gather_fault = -1;  // tests: fail ncclGather at this shard
};

namespace {

int destroy(ptg_multi *m)
{
    if (!m)
        return PTG_OK;
    DeviceGuard g;
    // Every stream is drained before its buffers are freed -- a broken
    // group's too, since a failed frame's render kernels may still be running
    // on the slabs.  A broken group's communicators were aborted when the
    // group failed, which should release every queued gather; its streams are
    // still drained with a bounded wait, so a peer that never returns cannot
    // hang close(): after ~10 s that shard's buffers are leaked, not freed
    // under a running kernel, and the call reports PTG_ERR_HIP.
    int rc = PTG_OK;
    for (Shard &s : m->shards) {
        if (s.id < 0)
            continue;
        (void)hipSetDevice(s.id);
        if (!s.stream)
            continue;
        if (!m->broken) {
            (void)hipStreamSynchronize(s.stream);
            continue;
        }
        const auto t0 = std::chrono::steady_clock::now();
        while (hipStreamQuery(s.stream) == hipErrorNotReady) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
                s.stuck = true;
                rc = PTG_ERR_HIP;
                break;
            }
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
    }
    bool any_stuck = false;
    for (Shard &s : m->shards) {
        if (s.id < 0)
            continue;
        (void)hipSetDevice(s.id);
        if (s.comm)
            (void)(m->broken ? ncclCommAbort(s.comm) : ncclCommDestroy(s.comm));
        if (s.stuck) {  // still running after the abort: leak its buffers
            any_stuck = true;
            continue;
        }
        if (s.slab)
            (void)hipFree(s.slab);
        if (s.counters)
            (void)hipFree(s.counters);
        if (s.done)
            (void)hipEventDestroy(s.done);
        if (s.t_begin)
            (void)hipEventDestroy(s.t_begin);
        if (s.t_rendered)
            (void)hipEventDestroy(s.t_rendered);
        if (s.stream)
            (void)hipStreamDestroy(s.stream);
        if (s.ctx)
            (void)ptg_context_destroy(s.ctx);
    }
    if (!any_stuck && !m->shards.empty() && m->shards[0].id >= 0) {
        (void)hipSetDevice(m->shards[0].id);
        if (m->gathered)
            (void)hipFree(m->gathered);
        if (m->image)
            (void)hipFree(m->image);
        if (m->t_unsharded)
            (void)hipEventDestroy(m->t_unsharded);
    }
    delete m;
    return rc == PTG_OK ? PTG_OK : fail(rc, "multi: a broken group's stream did not drain within 10 s; its buffers were leaked");
}

int create(const ptg_sphere *spheres, size_t n_spheres, const ptg_camera *cam, const int *devices, int n, bool rccl,
           ptg_multi **out)
{
    if (!out)
        return fail(PTG_ERR_INVALID_ARGUMENT, "multi: out is NULL");
    *out = nullptr;
    if (!devices || n < 1)
        return fail(PTG_ERR_INVALID_ARGUMENT, "multi: no device");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return fail(PTG_ERR_NO_DEVICE, "no HIP device visible");
    for (int k = 0; k < n; ++k) {
        if (devices[k] < 0 || devices[k] >= count)
            return fail(PTG_ERR_INVALID_ARGUMENT, "multi: device ordinal out of range");
        for (int j = 0; j < k && rccl; ++j)
            if (devices[j] == devices[k])
                return fail(PTG_ERR_UNSUPPORTED, "render_multi: RCCL needs distinct devices (one rank per GPU)");
    }
    DeviceGuard g;
    ptg_multi *m = new ptg_multi();
    m->rccl = rccl;
    m->shards.resize(n);
    int rc = PTG_OK;
    for (int k = 0; k < n && rc == PTG_OK; ++k) {
        Shard &s = m->shards[k];
        s.id = devices[k];
        if ((rc = ptg_context_create(spheres, n_spheres, cam, s.id, &s.ctx)))
            break;
        hipError_t e = hipSetDevice(s.id);
        if (e == hipSuccess)
            e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
        if (e == hipSuccess)
            e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
        if (e == hipSuccess)
            e = hipEventCreate(&s.t_begin);
        if (e == hipSuccess)
            e = hipEventCreate(&s.t_rendered);
        if (e == hipSuccess && k == 0)
            e = hipEventCreate(&m->t_unsharded);
        if (e != hipSuccess)
            rc = hip_fail("multi: stream/event", e);
    }
    if (rc == PTG_OK && rccl) {
        std::vector<ncclComm_t> cm(n);
        const ncclResult_t r = ncclCommInitAll(cm.data(), n, devices);
        if (r != ncclSuccess)
            rc = nccl_fail("ncclCommInitAll", r);
        else
            for (int k = 0; k < n; ++k)
                m->shards[k].comm = cm[k];
    }
    if (rc != PTG_OK) {
        destroy(m);
        return rc;
    }
    *out = m;
    return PTG_OK;
}

int check_frame(const ptg_multi *m, const ptg_params *p)
{
    if (!m || !p)
        return fail(PTG_ERR_INVALID_ARGUMENT, "multi: NULL context or params");
    if (m->broken)
        return fail(PTG_ERR_HIP, "multi: the context's RCCL group failed earlier and its communicators were "
                                 "aborted; destroy it");
    if (p->width <= 0 || p->height <= 0 || p->band_rows < 1)
        return fail(PTG_ERR_INVALID_ARGUMENT, "multi: width, height and band_rows must be positive");
    if (p->shard_count != 1 || p->shard_rank != 0)
        return fail(PTG_ERR_INVALID_ARGUMENT, "render_multi shards the whole frame itself: shard_count must be 1");
    if (p->flags & PTG_FLAG_REFERENCE_F64)
        return fail(PTG_ERR_UNSUPPORTED, "render_multi renders the fp32 kernel only (the reference-arithmetic "
                                         "mode keeps doubles: use ptg_render)");
    return PTG_OK;
}

// params of shard k
ptg_params shard_params(const ptg_params *p, int k, int n)
{
    ptg_params q = *p;
    q.shard_rank = k;
    q.shard_count = n;
    return q;
}

// buffers for a frame of this size (grown, never shrunk)
int reserve(ptg_multi *m, const ptg_params *p, size_t &slab_elems)
{
    const int n = (int)m->shards.size();
    int32_t rows = 0;
    int rc = ptg_shard_rows(p->height, p->band_rows, n, &rows);
    if (rc)
        return rc;
    slab_elems = (size_t)rows * p->width * 3;
    const size_t image_elems = (size_t)p->width * p->height * 3;
    for (Shard &s : m->shards) {
        if (s.slab_cap >= slab_elems)
            continue;
        MULTI_HIP(hipSetDevice(s.id));
        if (s.slab) {
            MULTI_HIP(hipStreamSynchronize(s.stream));
            MULTI_HIP(hipFree(s.slab));
            s.slab = nullptr;
            s.slab_cap = 0;
        }
        if (hipMalloc(&s.slab, slab_elems * sizeof(float)) != hipSuccess)
            return fail(PTG_ERR_OUT_OF_MEMORY, "multi: hipMalloc of a slab failed");
        s.slab_cap = slab_elems;
    }
    Shard &r = m->shards[0];
    MULTI_HIP(hipSetDevice(r.id));
    if (m->gathered_cap < (size_t)n * slab_elems) {
        MULTI_HIP(hipStreamSynchronize(r.stream));
        if (m->gathered)
            MULTI_HIP(hipFree(m->gathered));
        m->gathered = nullptr;
        m->gathered_cap = 0;
        if (hipMalloc(&m->gathered, (size_t)n * slab_elems * sizeof(float)) != hipSuccess)
            return fail(PTG_ERR_OUT_OF_MEMORY, "multi: hipMalloc of the gather buffer failed");
        m->gathered_cap = (size_t)n * slab_elems;
    }
    if (m->image_cap < image_elems) {
        MULTI_HIP(hipStreamSynchronize(r.stream));
        if (m->image)
            MULTI_HIP(hipFree(m->image));
        m->image = nullptr;
        m->image_cap = 0;
        if (hipMalloc(&m->image, image_elems * sizeof(float)) != hipSuccess)
            return fail(PTG_ERR_OUT_OF_MEMORY, "multi: hipMalloc of the image failed");
        m->image_cap = image_elems;
    }
    m->host.resize(image_elems);
    return PTG_OK;
}

// ONE gather of the equal-size slabs to the root (RCCL: one ncclGather per
// rank inside a group, rank-major on the root -- rccl.h:745; local shards: the
// same layout by device copies after each shard's slab is complete) and the
// un-shard there, queued on the root's stream (asynchronous).
int gather_unshard_device(ptg_multi *m, const ptg_params *p, size_t slab_elems)
{
    const int n = (int)m->shards.size();
    Shard &root = m->shards[0];
    if (m->rccl) {
        // every device is made current once BEFORE the group opens, so that
        // inside it only the ncclGather calls can fail
        for (int k = n - 1; k >= 0; --k)
            MULTI_HIP(hipSetDevice(m->shards[k].id));
        ncclResult_t r = ncclGroupStart();
        if (r != ncclSuccess)
            return nccl_fail("ncclGroupStart", r);
        int rc = PTG_OK;
        for (int k = 0; k < n && rc == PTG_OK; ++k) {
            Shard &s = m->shards[k];
            (void)hipSetDevice(s.id);
            r = k == m->inject_gather_fault
                    ? ncclInvalidArgument
                    : ncclGather(s.slab, k == 0 ? m->gathered : nullptr, slab_elems, ncclFloat, 0, s.comm, s.stream);
            if (r != ncclSuccess)
                rc = nccl_fail("ncclGather", r);
        }
        // the group is closed on every path (an error inside it must not leave
        // this thread's RCCL group open) ...
        const ncclResult_t re = ncclGroupEnd();
        if (rc != PTG_OK || re != ncclSuccess) {
            // ... but a partial group must not run without its peers: the
            // queued collectives are aborted with the communicators, and the
            // context refuses further frames
            m->broken = true;
            for (Shard &s : m->shards)
                if (s.comm) {
                    (void)hipSetDevice(s.id);
                    (void)ncclCommAbort(s.comm);
                    s.comm = nullptr;
                }
            return rc != PTG_OK ? rc : nccl_fail("ncclGroupEnd", re);
        }
        MULTI_HIP(hipSetDevice(root.id));
    } else {
        MULTI_HIP(hipSetDevice(root.id));
        for (int k = 0; k < n; ++k) {
            Shard &s = m->shards[k];
            MULTI_HIP(hipEventRecord(s.done, s.stream));
            MULTI_HIP(hipStreamWaitEvent(root.stream, s.done, 0));
            MULTI_HIP(hipMemcpyAsync(m->gathered + (size_t)k * slab_elems, s.slab, slab_elems * sizeof(float),
                                     hipMemcpyDeviceToDevice, root.stream));
        }
    }
    return ptg_unshard_device(m->gathered, m->image, p->width, p->height, p->band_rows, n, root.stream);
}

// waits for every shard's stream (root last: its part ends with the un-shard)
int sync_all(ptg_multi *m)
{
    for (int k = (int)m->shards.size() - 1; k >= 0; --k) {
        MULTI_HIP(hipSetDevice(m->shards[k].id));
        MULTI_HIP(hipStreamSynchronize(m->shards[k].stream));
    }
    return PTG_OK;
}

// gather + un-shard, then the image to the host (m->host).  Synchronous.
int gather_unshard(ptg_multi *m, const ptg_params *p, size_t slab_elems)
{
    int rc = gather_unshard_device(m, p, slab_elems);
    if (rc)
        return rc;
    Shard &root = m->shards[0];
    const size_t image_elems = (size_t)p->width * p->height * 3;
    MULTI_HIP(hipSetDevice(root.id));
    MULTI_HIP(hipMemcpyAsync(m->host.data(), m->image, image_elems * sizeof(float), hipMemcpyDeviceToHost,
                             root.stream));
    return sync_all(m);
}

}  // namespace

extern "C" {

int ptg_multi_create(const ptg_sphere *spheres, size_t n_spheres, const ptg_camera *cam, const int *devices,
                     int n_devices, ptg_multi **out)
{
    return create(spheres, n_spheres, cam, devices, n_devices, true, out);
}

// internal (tests): n_shards shards on ONE device, gathered by device copies
// into the same rank-major layout an n-rank ncclGather produces -- the
// n > 1 slab layout, un-shard and host add of the multi path on a 1-GPU box
int ptg_multi_create_local_(const ptg_sphere *spheres, size_t n_spheres, const ptg_camera *cam, int device,
                            int n_shards, ptg_multi **out)
{
    if (n_shards < 1 || n_shards > 64)
        return fail(PTG_ERR_INVALID_ARGUMENT, "multi (local): 1 <= n_shards <= 64");
    std::vector<int> d(n_shards, device);
    return create(spheres, n_spheres, cam, d.data(), n_shards, false, out);
}

int ptg_multi_destroy(ptg_multi *m) { return destroy(m); }

int ptg_multi_render(ptg_multi *m, const ptg_params *params, double *image_rgb)
{
    int rc = check_frame(m, params);
    if (rc)
        return rc;
    m->timed = false;  // the image / events no longer describe a frame_device frame
    if (!image_rgb)
        return fail(PTG_ERR_INVALID_ARGUMENT, "render_multi: image is NULL");
    DeviceGuard g;
    size_t slab_elems = 0;
    if ((rc = reserve(m, params, slab_elems)))
        return rc;
    const int n = (int)m->shards.size();
    // the shards render concurrently (asynchronous launches on each device)
    for (int k = 0; k < n; ++k) {
        const ptg_params q = shard_params(params, k, n);
        if ((rc = ptg_render_device(m->shards[k].ctx, &q, m->shards[k].slab, nullptr, m->shards[k].stream)))
            return rc;
    }
    if ((rc = gather_unshard(m, params, slab_elems)))
        return rc;
    const size_t image_elems = (size_t)params->width * params->height * 3;
    for (size_t i = 0; i < image_elems; ++i)
        image_rgb[i] = image_rgb[i] + (double)m->host[i];  // main.cpp:196: image[row] += ...
    return PTG_OK;
}

int ptg_multi_reset_accumulation(ptg_multi *m, const ptg_params *params)
{
    int rc = check_frame(m, params);
    if (rc)
        return rc;
    m->timed = false;  // the image / events no longer describe a frame_device frame
    DeviceGuard g;
    const int n = (int)m->shards.size();
    for (int k = 0; k < n; ++k) {
        const ptg_params q = shard_params(params, k, n);
        if ((rc = ptg_reset_accumulation_device(m->shards[k].ctx, &q, m->shards[k].stream)))
            return rc;
    }
    return PTG_OK;
}

int ptg_multi_accumulate(ptg_multi *m, const ptg_params *params, int32_t sample_begin, int32_t sample_end)
{
    int rc = check_frame(m, params);
    if (rc)
        return rc;
    m->timed = false;  // the image / events no longer describe a frame_device frame
    DeviceGuard g;
    const int n = (int)m->shards.size();
    for (int k = 0; k < n; ++k) {
        const ptg_params q = shard_params(params, k, n);
        if ((rc = ptg_accumulate_device(m->shards[k].ctx, &q, sample_begin, sample_end, nullptr,
                                        m->shards[k].stream)))
            return rc;
    }
    return PTG_OK;
}

int ptg_multi_resolve(ptg_multi *m, const ptg_params *params, int32_t samples_done, float *image_rgb)
{
    int rc = check_frame(m, params);
    if (rc)
        return rc;
    m->timed = false;  // the image / events no longer describe a frame_device frame
    if (!image_rgb)
        return fail(PTG_ERR_INVALID_ARGUMENT, "multi_resolve: image is NULL");
    DeviceGuard g;
    size_t slab_elems = 0;
    if ((rc = reserve(m, params, slab_elems)))
        return rc;
    const int n = (int)m->shards.size();
    for (int k = 0; k < n; ++k) {
        const ptg_params q = shard_params(params, k, n);
        if ((rc = ptg_resolve_device(m->shards[k].ctx, &q, samples_done, m->shards[k].slab, m->shards[k].stream)))
            return rc;
    }
    if ((rc = gather_unshard(m, params, slab_elems)))
        return rc;
    const size_t image_elems = (size_t)params->width * params->height * 3;
    std::copy(m->host.begin(), m->host.begin() + image_elems, image_rgb);
    return PTG_OK;
}

int ptg_multi_frame_device(ptg_multi *m, const ptg_params *params, unsigned long long *counters)
{
    int rc = check_frame(m, params);
    if (rc)
        return rc;
    DeviceGuard g;
    // before reserve(): a failed re-allocation must not leave the previous
    // frame's flag on a freed image
    m->timed = false;
    size_t slab_elems = 0;
    if ((rc = reserve(m, params, slab_elems)))
        return rc;
    const int n = (int)m->shards.size();
    const bool count = (params->flags & (PTG_FLAG_COUNT_TESTS | PTG_FLAG_COUNT_NONFINITE)) != 0;
    for (int k = 0; k < n; ++k) {
        Shard &s = m->shards[k];
        MULTI_HIP(hipSetDevice(s.id));
        if (count && !s.counters && hipMalloc(&s.counters, 4 * sizeof(unsigned long long)) != hipSuccess)
            return fail(PTG_ERR_OUT_OF_MEMORY, "multi: hipMalloc of the counters failed");
        if (count)
            MULTI_HIP(hipMemsetAsync(s.counters, 0, 4 * sizeof(unsigned long long), s.stream));
        MULTI_HIP(hipEventRecord(s.t_begin, s.stream));
        const ptg_params q = shard_params(params, k, n);
        if ((rc = ptg_render_device(s.ctx, &q, s.slab, count ? s.counters : nullptr, s.stream)))
            return rc;
        MULTI_HIP(hipSetDevice(s.id));
        MULTI_HIP(hipEventRecord(s.t_rendered, s.stream));
    }
    if ((rc = gather_unshard_device(m, params, slab_elems)))
        return rc;
    MULTI_HIP(hipSetDevice(m->shards[0].id));
    MULTI_HIP(hipEventRecord(m->t_unsharded, m->shards[0].stream));
    if ((rc = sync_all(m)))
        return rc;
    m->timed = true;
    m->frame_w = params->width;
    m->frame_h = params->height;
    m->frame_band_rows = params->band_rows;
    if (count && counters) {
        for (int i = 0; i < 4; ++i)
            counters[i] = 0;
        for (Shard &s : m->shards) {
            unsigned long long c[4];
            MULTI_HIP(hipSetDevice(s.id));
            MULTI_HIP(hipMemcpy(c, s.counters, sizeof(c), hipMemcpyDeviceToHost));
            for (int i = 0; i < 4; ++i)
                counters[i] += c[i];
        }
    }
    return PTG_OK;
}

int ptg_multi_frame_timing(const ptg_multi *m, float *render_ms, int n, float *frame_ms)
{
    if (!m || !m->timed)
        return fail(PTG_ERR_INVALID_ARGUMENT, "multi_frame_timing: no completed ptg_multi_frame_device");
    if (n != (int)m->shards.size() || !render_ms || !frame_ms)
        return fail(PTG_ERR_INVALID_ARGUMENT, "multi_frame_timing: render_ms needs one entry per device");
    DeviceGuard g;
    for (int k = 0; k < n; ++k) {
        MULTI_HIP(hipSetDevice(m->shards[k].id));
        MULTI_HIP(hipEventElapsedTime(&render_ms[k], m->shards[k].t_begin, m->shards[k].t_rendered));
    }
    MULTI_HIP(hipSetDevice(m->shards[0].id));
    MULTI_HIP(hipEventElapsedTime(frame_ms, m->shards[0].t_begin, m->t_unsharded));
    return PTG_OK;
}

int ptg_multi_image(ptg_multi *m, const ptg_params *params, float *image_rgb)
{
    int rc = check_frame(m, params);
    if (rc)
        return rc;
    if (!image_rgb || !m->timed)
        return fail(PTG_ERR_INVALID_ARGUMENT, "multi_image: NULL image or no completed ptg_multi_frame_device "
                                              "(since the last render / pass / resolve)");
    if (params->width != m->frame_w || params->height != m->frame_h || params->band_rows != m->frame_band_rows)
        return fail(PTG_ERR_INVALID_ARGUMENT, "multi_image: params differ from the last frame's width, height or "
                                              "band_rows");
    const size_t image_elems = (size_t)params->width * params->height * 3;
    DeviceGuard g;
    MULTI_HIP(hipSetDevice(m->shards[0].id));
    MULTI_HIP(hipMemcpy(image_rgb, m->image, image_elems * sizeof(float), hipMemcpyDeviceToHost));
    return PTG_OK;
}

int ptg_multi_comm_info(const ptg_multi *m, int32_t *ranks, int32_t *comm_devices, int32_t *user_ranks, int n)
{
    if (!m || !ranks || !comm_devices || !user_ranks)
        return fail(PTG_ERR_INVALID_ARGUMENT, "multi_comm_info: NULL argument");
    if (n != (int)m->shards.size())
        return fail(PTG_ERR_INVALID_ARGUMENT, "multi_comm_info: one entry per shard");
    for (int k = 0; k < n; ++k) {
        const Shard &s = m->shards[k];
        ranks[k] = 0;
        comm_devices[k] = s.id;
        user_ranks[k] = -1;
        if (!s.comm)
            continue;
        int c = 0, dev = -1, ur = -1;
        ncclResult_t r = ncclCommCount(s.comm, &c);
        if (r == ncclSuccess)
            r = ncclCommCuDevice(s.comm, &dev);
        if (r == ncclSuccess)
            r = ncclCommUserRank(s.comm, &ur);
        if (r != ncclSuccess)
            return nccl_fail("ncclCommCount/CuDevice/UserRank", r);
        ranks[k] = c;
        comm_devices[k] = dev;
        user_ranks[k] = ur;
    }
    return PTG_OK;
}

int ptg_device_pci_bus_id(int device, char *buf, int len)
{
    if (!buf || len < 1)
        return fail(PTG_ERR_INVALID_ARGUMENT, "pci_bus_id: NULL or empty buffer");
    buf[0] = '\0';
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return fail(PTG_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= count)
        return fail(PTG_ERR_INVALID_ARGUMENT, "pci_bus_id: device ordinal out of range");
    MULTI_HIP(hipDeviceGetPCIBusId(buf, len, device));
    return PTG_OK;
}

// internal (tests): make the next RCCL gather fail at shard k (-1: off)
int ptg_multi_inject_gather_fault_(ptg_multi *m, int k)
{
    if (!m)
        return fail(PTG_ERR_INVALID_ARGUMENT, "multi: NULL context");
    m->inject_gather_fault = k;
    return PTG_OK;
}

int ptg_render_multi(const ptg_sphere *spheres, size_t n_spheres, const ptg_camera *cam, const ptg_params *params,
                     const int *devices, int n_devices, double *image_rgb)
{
    if (!params || !image_rgb || !devices || n_devices < 1)
        return fail(PTG_ERR_INVALID_ARGUMENT, "render_multi: NULL argument or no device");
    ptg_multi probe;  // argument checks before any device work
    probe.shards.resize(1);
    int rc = check_frame(&probe, params);
    if (rc)
        return rc;
    ptg_multi *m = nullptr;
    if ((rc = ptg_multi_create(spheres, n_spheres, cam, devices, n_devices, &m)))
        return rc;
    rc = ptg_multi_render(m, params, image_rgb);
    ptg_multi_destroy(m);
    return rc;
}

}  // extern "C"
