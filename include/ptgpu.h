/*
 * ptgpu.h -- C ABI of the MI355X render loop (libptgpu.so).
 *
 * Drop-in for the per-pixel hot path of AlexandruIca/cpu-path-tracing:
 * the taskflow row loop src/main.cpp:214-236 and everything it calls
 * (render_subpixel main.cpp:179-197, radiance main.cpp:104-158, the scene scan
 * main.cpp:30-42, the BRDF samplers main.cpp:44-97, camera::get_ray
 * camera.cpp:32-38, sphere::intersect sphere.cpp:6-30, get_hit_record_at
 * hit_record.cpp:3-12, rand_state random_state.cpp:3-17) runs as one HIP
 * megakernel on gfx950.  Plain C types only: pointers, sizes, PODs.
 *
 * Conventions (reference: everything noexcept, no error codes):
 *   every entry point returns PTG_OK (0) or a negative ptg_status and never
 *   throws; ptg_last_error() returns a thread-local description of the last
 *   failure.  Calls are not re-entrant on one context.
 */
#ifndef PTGPU_H
#define PTGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: flags = 0 now selects the fast arithmetic mode (hardware
 * transcendentals, not reproducible on a CPU); version 1's flags = 0 was the
 * oracle-exact mode, now PTG_FLAG_EXACT_MATH.  Also added since 1:
 * ptg_multi_*, ptg_math_probe_device.  A caller built against 1 that needs
 * the old bit-exact image must pass PTG_FLAG_EXACT_MATH. */
#define PTG_ABI_VERSION 2

typedef enum ptg_status {
    PTG_OK = 0,
    PTG_ERR_INVALID_ARGUMENT = -1,
    PTG_ERR_HIP = -2,
    PTG_ERR_NO_DEVICE = -3,
    PTG_ERR_UNSUPPORTED = -4,
    PTG_ERR_OUT_OF_MEMORY = -5
} ptg_status;

/* reflection.hpp:7-12 */
typedef enum ptg_material { PTG_DIFFUSE = 0, PTG_SPECULAR = 1, PTG_DIELECTRIC = 2 } ptg_material;

/* Field-for-field mirror of pt::sphere (sphere.hpp:10-17): 88 bytes, so a
 * std::vector<pt::sphere>::data() can be passed as-is. */
typedef struct ptg_sphere {
    double radius;
    double position[3];
    double emission[3];
    double color[3];
    int32_t material; /* ptg_material (pt::reflection_type) */
    int32_t reserved_;
} ptg_sphere;

/* Field-for-field mirror of pt::camera (camera.hpp:23-33): 176 bytes, the
 * output of pt::camera::with_config (camera.cpp:3-17). */
typedef struct ptg_camera {
    double position[3];
    double lower_left_corner[3];
    double cam_x_axis[3];
    double cam_y_axis[3];
    double u[3];
    double v[3];
    double w[3];
    double lens_radius;
} ptg_camera;

/* The ints main.cpp:202-206 hands to the loop, plus the counter-RNG seed
 * (replacing std::random_device, random_state.cpp:5), the row-band shard and
 * the work-unit size.
 *
 * Sample accumulation (main.cpp:192 `r = r + c * (1/samps)`, sequential
 * double) is restated order-independently: every path's radiance is
 * quantised to a u64 fixed-point value q(c) = trunc(c * 2^32) (c clamped to
 * [0, 2^30]) and summed exactly; the sub-pixel mean is
 * (float)((double)sum * 2^-32 / samps).  The image therefore does not depend
 * on scheduling, chunking or sharding. */
typedef struct ptg_params {
    int32_t width;          /* main.cpp:204 */
    int32_t height;         /* main.cpp:205 */
    int32_t samples;        /* per sub-pixel (main.cpp:206: spp / num_subpixels^2) */
    int32_t num_subpixels;  /* per axis (main.cpp:202); 1..8 */
    uint64_t seed;          /* counter RNG key; the image does not depend on sharding */
    int32_t band_rows;      /* shard: output rows per band (>= 1) */
    int32_t shard_rank;     /* this shard renders bands b with b % shard_count == shard_rank */
    int32_t shard_count;    /* 1 = whole image */
    int32_t chunk_samples;  /* samples per sub-pixel per work unit (0 = auto); results do not depend on it */
    int32_t flags;          /* PTG_FLAG_* */
} ptg_params;

/* flags: with PTG_FLAG_COUNT_TESTS, d_segments of ptg_render_device /
 * ptg_accumulate_device points to 3 counters: += scene scans, sphere tests
 * executed (ray-sphere quadratics), and BVH box tests (scenes of > 64
 * spheres) or, of the sphere tests, the box-wall tests (linear scenes) --
 * the inputs of the roofline model.  Linear scenes count each lane's own
 * tests (box mode tests about one wall per segment, not every wall); the
 * survey's model count is scans x spheres. */
#define PTG_FLAG_COUNT_TESTS 1
/* with PTG_FLAG_COUNT_NONFINITE (implies the counters above), d_segments points
 * to 4 counters; the 4th += paths whose radiance has a component that is NaN,
 * negative or above 2^30 -- values the exact accumulation would clip (NaN and
 * negative to 0).  None are expected: the -m gpu tests assert 0. */
#define PTG_FLAG_COUNT_NONFINITE 2
/* PTG_FLAG_REFERENCE_F64: render with the reference's own double-precision
 * arithmetic, operation for operation (src/main.cpp:30-197 and the pt
 * library: linear strict-< scan, (-hb -+ sq)/a roots, libm-style
 * sin/cos/pow, sequential r += c/samps) instead of the fp32 megakernel --
 * a parity mode (csrc/ref64.hpp), several times slower.  Only the counter-RNG
 * draws differ from the reference (as in every mode).  ptg_render keeps the
 * doubles; ptg_render_device rounds them into its float slab.  Not for
 * progressive passes or trace_samples (PTG_ERR_UNSUPPORTED). */
#define PTG_FLAG_REFERENCE_F64 4
/* PTG_FLAG_EXACT_MATH (ABI 2; the default of ABI 1): the fp32 kernel with deterministic square root,
 * reciprocal square root, division and sin/cos sequences (~1 ulp) that the
 * oracle (oracle/pt_oracle.c, Mode B) executes too -- the image then equals
 * the CPU restatement bit for bit.  Without it (the default) the kernel uses
 * the GPU's own v_sqrt/v_rsq/v_rcp/v_sin/v_cos instructions, about as
 * accurate but not reproducible on a CPU: the image is within the north
 * star's per-pixel RMSE of the reference arithmetic (DESIGN.md "arithmetic
 * modes").  Either way a frame does not depend on sharding, work-unit sizes,
 * progressive passes or the GPU count. */
#define PTG_FLAG_EXACT_MATH 8

typedef struct ptg_context ptg_context;

/* ---- metadata -------------------------------------------------------- */
int ptg_abi_version(void);
const char *ptg_last_error(void);
int ptg_device_count(int *count);

/* ---- drop-in entry point ---------------------------------------------
 * Replaces main.cpp:214-236.  Synchronous.  image_rgb is the caller-owned
 * std::vector<pt::vec3> viewed as width*height*3 doubles in the reference's
 * row order (row (H-1-y)*W + x, main.cpp:181); like the loop, the call ADDS
 * sum_sub clamp(mean)/num_subpixels^2 (main.cpp:195-196) into it.  With
 * shard_count > 1 only the shard's bands are added.  device = -1: current. */
int ptg_render(const ptg_sphere *spheres, size_t n_spheres, const ptg_camera *cam,
               const ptg_params *params, int device, double *image_rgb);

/* ---- single-process multi-GPU drop-in ---------------
 * The same contract as ptg_render (params->shard_count must be 1: the call
 * shards the frame itself), rendered on n_devices distinct GPUs of this
 * process: device k renders the interleaved row bands b with
 * b % n_devices == k (band_rows from params), ONE ncclGather (RCCL over xGMI,
 * rccl.h:745) collects the slabs on devices[0], which un-shards the frame.
 * The image equals ptg_render's bit for bit (the RNG is keyed by the global
 * pixel).  Replaces main.cpp:214-236 for a caller owning several GPUs.
 * fp32 kernel only: PTG_FLAG_REFERENCE_F64 is refused (PTG_ERR_UNSUPPORTED;
 * ptg_render keeps that mode's doubles).  The caller's current HIP device is
 * restored on return.  ptg_render_multi = ptg_multi_create + ptg_multi_render
 * + ptg_multi_destroy. */
int ptg_render_multi(const ptg_sphere *spheres, size_t n_spheres, const ptg_camera *cam,
                     const ptg_params *params, const int *devices, int n_devices, double *image_rgb);

/* A persistent multi-GPU context: per device the scene in HBM, a stream and
 * the slab, the RCCL communicator of the device set (ncclCommInitAll once),
 * the root's gather buffer and image -- repeated and progressive frames
 * reuse them.  Not re-entrant. */
typedef struct ptg_multi ptg_multi;
int ptg_multi_create(const ptg_sphere *spheres, size_t n_spheres, const ptg_camera *cam, const int *devices,
                     int n_devices, ptg_multi **out);
int ptg_multi_destroy(ptg_multi *m);
/* ptg_render_multi's frame on the context (synchronous; adds into image_rgb
 * like main.cpp:196). */
int ptg_multi_render(ptg_multi *m, const ptg_params *params, double *image_rgb);
/* Progressive passes over all devices (README.md:9): reset, then sample
 * passes [begin, end) queued on every device (asynchronous), then a resolve
 * of the samples so far -- each device resolves its bands, ONE gather, the
 * un-shard -- written (not added) to image_rgb as W*H*3 floats in the
 * reference's row order (synchronous).  After passes covering [0, samples)
 * the resolve equals ptg_render's image bit for bit. */
int ptg_multi_reset_accumulation(ptg_multi *m, const ptg_params *params);
int ptg_multi_accumulate(ptg_multi *m, const ptg_params *params, int32_t sample_begin, int32_t sample_end);
int ptg_multi_resolve(ptg_multi *m, const ptg_params *params, int32_t samples_done, float *image_rgb);
/* The frame kept in HBM (the benchmark step over several GPUs): every device
 * renders its bands, ONE gather, the un-shard into the root's image buffer;
 * returns when all devices are done, with no host copy of the image.  With
 * PTG_FLAG_COUNT_TESTS in params->flags, counters (optional, host, 4 values)
 * receives the counters of ptg_render_device summed over the devices.
 * ptg_multi_frame_timing then gives, from HIP events of that frame, each
 * device's render time (render_ms[n_devices]) and the root's time from the
 * start of its render to the end of the un-shard (frame_ms);
 * ptg_multi_image copies the frame (W*H*3 floats, reference row order) to the
 * host.  After a failure inside the RCCL group the communicators are aborted
 * (no partial collective runs) and every later frame call returns
 * PTG_ERR_HIP; destroy the context. */
int ptg_multi_frame_device(ptg_multi *m, const ptg_params *params, unsigned long long *counters);
int ptg_multi_frame_timing(const ptg_multi *m, float *render_ms, int n_devices, float *frame_ms);
/* The last ptg_multi_frame_device frame only: params must have the frame's
 * width, height and band_rows (PTG_ERR_INVALID_ARGUMENT otherwise, and after
 * any other frame call on the context). */
int ptg_multi_image(ptg_multi *m, const ptg_params *params, float *image_rgb);
/* What the context's RCCL group actually is (the proof behind a multi-GPU
 * measurement): per shard k, ranks[k] = ncclCommCount of its communicator
 * (0: no communicator -- local shards gathered by device copies, or an
 * aborted group), comm_devices[k] = the HIP device its communicator runs on
 * (ncclCommCuDevice; the shard's device for local shards), user_ranks[k] =
 * ncclCommUserRank (-1 without a communicator).  n_devices must equal the
 * context's shard count. */
int ptg_multi_comm_info(const ptg_multi *m, int32_t *ranks, int32_t *comm_devices, int32_t *user_ranks,
                        int n_devices);
/* PCI bus id of a HIP device ("dddd:bb:dd.f", hipDeviceGetPCIBusId) into
 * buf (len >= 16 recommended).  Distinct devices of a node have distinct ids. */
int ptg_device_pci_bus_id(int device, char *buf, int len);

/* ---- device-resident path (bench, multi-GPU) --------------------------
 * A context holds the prepared scene in HBM on one device. */
int ptg_context_create(const ptg_sphere *spheres, size_t n_spheres, const ptg_camera *cam, int device,
                       ptg_context **out);
int ptg_context_destroy(ptg_context *ctx);

/* How ptg_render_device would launch this frame (host-side, nothing is
 * launched): info[0] box mode on (the linear scan's nearest-wall-first rule;
 * the fast mode turns it off when a ray could start inside a wall),
 * [1] box_walls_out (no ray can start inside a box wall: the fast mode's
 * outside-only wall roots apply), [2] BVH scan (> 64 spheres), [3] work units,
 * [4] workgroups, [5] unit levels, [6] an HBM accumulator + resolve pass,
 * [7] wall-pair mask (x 1, y 2, z 4).  n_info <= PTG_LAUNCH_INFO_COUNT values
 * are written (extra entries 0). */
#define PTG_LAUNCH_INFO_COUNT 8
int ptg_launch_info(ptg_context *ctx, const ptg_params *params, int64_t *info, int n_info);

/* Rows in one shard's slab: ceil(bands / shard_count) * band_rows. */
int ptg_shard_rows(int32_t height, int32_t band_rows, int32_t shard_count, int32_t *rows);

/* Asynchronous render on `stream` (hipStream_t; NULL = default stream).
 * d_slab: device buffer of ptg_shard_rows(...) * width * 3 floats; slab row j
 * holds output row ((j / band_rows) * shard_count + shard_rank) * band_rows +
 * j % band_rows (rows >= height are left untouched).  Pixel values are
 * written (not accumulated).  d_segments: optional device uint64 that
 * receives += the number of scene scans (radiance segments) executed. */
int ptg_render_device(ptg_context *ctx, const ptg_params *params, float *d_slab,
                      unsigned long long *d_segments, void *stream);

/* ---- progressive accumulation (README.md:9 "make the rendering process
 * progressive") ----------------------------------------
 * Sample passes add exact per-sub-pixel sums into the context's accumulator;
 * a resolve turns the sums so far into an image (clamped means over
 * samples_done samples) without consuming them.  After passes that together
 * cover samples [0, params->samples), ptg_resolve_device(..., samples, ...)
 * equals ptg_render_device bit for bit.  Reset before a new frame. */
int ptg_reset_accumulation_device(ptg_context *ctx, const ptg_params *params, void *stream);
int ptg_accumulate_device(ptg_context *ctx, const ptg_params *params, int32_t sample_begin, int32_t sample_end,
                          unsigned long long *d_segments, void *stream);
int ptg_resolve_device(ptg_context *ctx, const ptg_params *params, int32_t samples_done, float *d_slab,
                       void *stream);

/* Reassemble shard_count gathered slabs (rank-major, as all-gather lays them
 * out) into the width*height*3 image. */
int ptg_unshard_device(const float *d_gathered, float *d_image, int32_t width, int32_t height,
                       int32_t band_rows, int32_t shard_count, void *stream);

/* Output stage (utils.cpp:11-16 + main.cpp:240-247): 8-bit gamma-1/2.2
 * values round(pow(clamp(x), 1/2.2) * 255) of `count` floats. */
int ptg_tonemap_device(const float *d_image, uint8_t *d_out, size_t count, void *stream);

/* Scene preparation, host only (no device needed): for each sphere the
 * anchor axis chosen for a huge sphere (0..2; -1 = camera-facing anchor, or
 * not huge) and the order of the linear scan (scan_order[j] = scene index of
 * the sphere tested j-th; scenes of <= 64 spheres).  Exact ties between
 * candidate roots go to the sphere tested first. */
int ptg_scene_layout(const ptg_sphere *spheres, size_t n_spheres, const ptg_camera *cam, int32_t *anchor_axis,
                     int32_t *scan_order);

/* Parity probe: trace individual samples.  d_coords holds n records
 * {x, y, sx, sy, sample} (int32 each); d_out n*3 floats (radiance of that
 * one path, main.cpp:191); d_segs n int32 (scene scans of that path). */
int ptg_trace_samples_device(ptg_context *ctx, const ptg_params *params, const int32_t *d_coords, size_t n,
                             float *d_out, int32_t *d_segs, void *stream);

/* Accuracy probe of the kernels' arithmetic primitives in either mode
 * (exact != 0: PTG_FLAG_EXACT_MATH's sequences; 0: the hardware
 * instructions), n operands on the device: op PTG_PROBE_SQRT out[i] =
 * sqrt(in[i]); PTG_PROBE_RSQRT 1/sqrt(in[i]); PTG_PROBE_DIV in[2i] /
 * in[2i+1] (divisor > 0); PTG_PROBE_SINCOS the bits of in[i] are a 24-bit
 * integer m, out[2i], out[2i+1] = cos, sin of 2 pi m 2^-24 (main.cpp:55's
 * phi).  The arithmetic the render kernels execute, not a separate
 * implementation (tests/test_gpu_fast_math.py). */
#define PTG_PROBE_SQRT 0
#define PTG_PROBE_RSQRT 1
#define PTG_PROBE_DIV 2
#define PTG_PROBE_SINCOS 3
int ptg_math_probe_device(ptg_context *ctx, int32_t op, int32_t exact, const float *d_in, float *d_out, size_t n,
                          void *stream);

#ifdef __cplusplus
}
#endif
#endif /* PTGPU_H */
