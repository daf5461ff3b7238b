/*
 * svo_rt.h -- C-ABI of the MI355X sparse-voxel-octree ray caster (libsvo_rt.so).
 *
 * Drop-in native plugin for the reference's GPU host driver
 * `RaytracingMaster` (Assets/Scripts/SVO/GPU/RaytracingMaster.cs) and the
 * compute kernel it dispatches (Assets/Shaders/RaytraceCompute.compute +
 * NVIDIASVO.compute + AttachmentLookup.compute).  Plain C types only: no
 * torch / HIP types cross this boundary (streams are passed as void*).
 *
 * Conventions:
 *  - every function returns SVO_OK (0) or a negative svo_status; the
 *    thread-local svo_last_error() gives the text.  No C++ exception crosses.
 *  - host arrays are owned by the caller and copied before the call returns
 *    (ComputeBuffer.SetData semantics); device memory is owned by the context.
 *  - one context is driven from one host thread at a time.
 */
#ifndef SVO_RT_H
#define SVO_RT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct svo_ctx svo_ctx;

typedef enum svo_status {
    SVO_OK = 0,
    SVO_ERR_ARG = -1,        /* null / out-of-range argument */
    SVO_ERR_CAPACITY = -2,   /* upload exceeds the node-pool capacity */
    SVO_ERR_FORMAT = -3,     /* malformed node pool (pointer out of range, too deep) */
    SVO_ERR_HIP = -4,        /* HIP runtime failure */
    SVO_ERR_STATE = -5       /* call out of order (e.g. render before upload) */
} svo_status;

/* Stack modes: HLSL reproduces the float2 round trip
 * of NVIDIASVO.compute:98; EXACT keeps exact (parent, t_max) entries. */
typedef enum svo_stack_mode { SVO_STACK_HLSL = 0, SVO_STACK_EXACT = 1 } svo_stack_mode;

/* Per-pixel hit record, 24 bytes. */
typedef struct svo_hit {
    uint32_t parent;     /* descriptor holding the hit leaf (NVIDIASVO.compute:177); 0xFFFFFFFF = miss */
    uint8_t  hit_idx;    /* child slot of the hit leaf = idx ^ octant_mask ^ 7 (:176) */
    uint8_t  hit_scale;  /* leaf scale, 23 - depth */
    uint16_t flags;      /* bit0 hit, bit1 iteration cap, bit2 stack overflow, bit3 in shadow */
    float    t;          /* bestHit.distance = 2048 * t_min (:163,171); +inf on miss */
    float    nx, ny, nz; /* normalize(decodeNormal(att[2*parent+1] >> 16)) (:177-182) */
} svo_hit;

/* Row split of one frame across ranks/GPUs: rows are grouped in bands of
 * `band_rows`; band b belongs to rank b % band_count.  A rank's output holds
 * only its own rows, in increasing y.  {1, 0, 1} (or NULL) = whole frame. */
typedef struct svo_band {
    int band_rows;
    int band_rank;
    int band_count;
} svo_band;

/* ~ RaytracingMaster.InitializeSVOBuffer (RaytracingMaster.cs:111-116):
 * allocate a node pool of `capacity_nodes` descriptors (+2 attachment words
 * each) on HIP device `device`. */
int svo_create(int device, size_t capacity_nodes, svo_ctx **out);

/* ~ RaytracingMaster.SetSVOBuffer(RT.SVOData data, int offset)
 * (RaytracingMaster.cs:118-135, CompactSVO.cs:22-35): upload `n_desc` reference
 * descriptors (int32: ptr16 << 16 | valid8 << 8 | nonleaf8, ptr RELATIVE to the
 * descriptor) and `n_att` attachment words at descriptor offset `dst_offset`.
 * Deviation (documented): attachments land at word 2*dst_offset; the
 * reference writes them at word `offset` (RaytracingMaster.cs:134). */
int svo_set_buffer(svo_ctx *ctx, const int32_t *desc, size_t n_desc,
                   const uint32_t *att, size_t n_att, size_t dst_offset);

/* Wide node format for pools whose child pointers exceed 16 bits:
 * node = (uint64)first_nonleaf_child_abs << 32 | valid8 << 8 | nonleaf8. */
int svo_set_buffer_v2(svo_ctx *ctx, const uint64_t *nodes, size_t n_nodes,
                      const uint32_t *att, size_t n_att, size_t dst_offset);

/* ~ RaytracingMaster.UpdateShaderParameters (RaytracingMaster.cs:32-41):
 * Unity Matrix4x4 (column-major) camera-to-world and inverse projection,
 * _PixelOffset and _DirectionalLight (forward.xyz, intensity). */
int svo_set_camera(svo_ctx *ctx, const float c2w[16], const float inv_proj[16],
                   float px_off_x, float px_off_y, const float light[4]);

/* ~ RaytracingMaster.Render / Dispatch (RaytracingMaster.cs:60-74): trace one
 * primary ray per pixel of a width x height frame.  rgba_out (W*H*4 floats,
 * = the Result RWTexture2D<float4>) and hits_out (W*H records) are HOST
 * buffers, either may be NULL.  Blocks until the results are on the host. */
int svo_render(svo_ctx *ctx, int width, int height, int stack_mode,
               float *rgba_out, svo_hit *hits_out);

/* Device-resident variant for hosts that keep the frame in HBM: d_rgba /
 * d_hits are device pointers on this context's device (either may be NULL),
 * `band` selects this rank's rows (NULL = all), `stream` is a hipStream_t
 * (NULL = the context's own stream).  Asynchronous: returns after enqueue. */
int svo_render_device(svo_ctx *ctx, int width, int height, int stack_mode,
                      const svo_band *band, void *d_rgba, void *d_hits, void *stream);

/* Instrumented trace: per-ray descriptor-fetch counts (device uint32 array,
 * NVIDIASVO.compute:60-62 executions), used for the algorithmic-bytes figure
 * of the roofline.  Same arguments as svo_render_device plus d_fetches. */
int svo_count_fetches(svo_ctx *ctx, int width, int height, int stack_mode,
                      const svo_band *band, void *d_fetches, void *stream);

/* Render options (bit set).  SVO_OPT_SHADOW_RAYS: after the primary pass,
 * trace one shadow ray per hit toward -_DirectionalLight (SURVEY.md 8(d) C3;
 * the reference's shadow test is commented out at RaytraceCompute.compute:105-112):
 * origin = world hit point + 0.001 * normal; an occluded pixel gets hit flag
 * bit 3 and a black Result. */
enum { SVO_OPT_SHADOW_RAYS = 1, SVO_OPT_KERNEL_TIMING = 2 };
int svo_set_options(svo_ctx *ctx, uint32_t options);

/* SVO_OPT_KERNEL_TIMING: every render launch brackets its primary-ray kernel
 * (only that kernel: not the shadow pass, not the dispatch-order kernel) with
 * HIP events on the launch stream.  svo_kernel_time waits for the recorded
 * launches and returns their mean kernel duration in ms and their number, then
 * forgets them.  Measurement only (bench.py's roofline); no reference
 * counterpart. */
int svo_kernel_time(svo_ctx *ctx, double *mean_ms, uint64_t *launches);

/* ~ Graphics.Blit(Result, destination, AddMaterial) with _Sample = `sample`
 * (RaytracingMaster.cs:70-73, AddShader.shader:10,44-47): progressive
 * accumulation dst = src * a + dst * (1 - a), a = 1 / (sample + 1), on all four
 * channels (source alpha = a).  d_accum and d_sample are device buffers of
 * n_px RGBA32F pixels (16-byte aligned) on the context's device; `stream` as in
 * svo_render_device.  The caller keeps `sample` (_currentSample): 0 after a
 * camera change (RaytracingMaster.cs:44-47), +1 per frame. */
int svo_accumulate(svo_ctx *ctx, void *d_accum, const void *d_sample, size_t n_px, uint32_t sample,
                   void *stream);

/* Information about the uploaded pool. */
int svo_get_info(svo_ctx *ctx, size_t *n_nodes, int *max_depth, int *device);

/* Block until all work on the context's stream has finished. */
int svo_synchronize(svo_ctx *ctx);

/* Release device memory (the reference never Release()s its buffers). */
int svo_destroy(svo_ctx *ctx);

/* Thread-local text of the last error (empty string if none). */
const char *svo_last_error(void);

/* ABI version, bumped on any layout change. */
int svo_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
