/*
 * svo_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's SVO primary-ray path, used as the parity
 * checker for the HIP product path and as the `cpu_baseline` of bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library; the product path (raytracingtest_amd/) never does.
 *
 * Follows (all paths relative to the reference repo):
 *   Assets/Shaders/RaytraceCompute.compute:129-151   camera ray + uv
 *   Assets/Shaders/NVIDIASVO.compute:12-198          IntersectSVO
 *   Assets/Shaders/AttachmentLookup.compute:1-61     decodeNormal / decodeDXTColor
 *   Assets/Shaders/RaytraceCompute.compute:93-127    Shade (hit branch)
 *
 * Parity pinning: the reference path is HLSL + C# and cannot run here (no
 * dxc/fxc, no mono/dotnet, no Unity), and the reference holds
 * no traversal outputs.  The decode functions are pinned by the 4,977
 * normal-code known answers of the reference's `Text` dump and by its worked
 * attachment example; the traversal by two independent witnesses
 * (tests/test_oracle.py): a restatement of the reference's own C# CPU tracer
 * (NVIDIAIterativeTracer.cs:72-290, tests/cs_tracer.py), bit-identical to the
 * EXACT stack mode on every reachable hit of both full C1 frames, and a
 * double-precision brute-force first-hit search over the same frames.  The
 * HLSL compiler's own FMA / rsqrt choices stay unpinned (strict IEEE here).
 */
#ifndef SVO_ORACLE_H
#define SVO_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Node-pool formats.
 *  V1: the reference layout, int32 per descriptor:
 *      (ptr16 << 16) | (valid8 << 8) | nonleaf8, ptr relative to the node
 *      (NaiveCreator.cs:184-187, NVIDIASVO.compute:101-105).
 *  V2: uint64 per node: low 32 = (valid8 << 8) | nonleaf8, high 32 = absolute
 *      index of the first non-leaf child (the >16-bit pointer format). */
enum { ORC_FMT_V1 = 1, ORC_FMT_V2 = 2 };

/* Stack modes.
 *  HLSL : stack entries round-trip through float2 as in NVIDIASVO.compute:98.
 *  EXACT: exact (parent, t_max) entries (Laine-Karras / C# tracer). */
enum { ORC_STACK_HLSL = 0, ORC_STACK_EXACT = 1 };
/* OR-ed into the render mode: trace one shadow ray per primary hit. */
#define ORC_SHADOW_RAYS 0x100
/* OR into mode: the fetches output receives loop iterations (NVIDIASVO.compute:57) instead */
#define ORC_COUNT_ITERS 0x200
/* diagnostics (with ORC_SHADOW_RAYS): the fetch output counts the shadow ray's loop
 * iterations instead (0 for pixels without a shadow ray) */
#define ORC_COUNT_SHADOW_ITERS 0x400

/* Per-pixel hit record: identical layout to svo_hit in include/svo_rt.h. */
typedef struct orc_hit {
    uint32_t parent;    /* descriptor index holding the hit leaf, 0xFFFFFFFF = miss */
    uint8_t  hit_idx;   /* child slot of the leaf inside `parent` (NVIDIASVO.compute:176) */
    uint8_t  hit_scale; /* leaf scale (23 - depth) */
    uint16_t flags;     /* bit0 hit, bit1 iteration cap, bit2 stack overflow, bit3 in shadow */
    float    t;         /* bestHit.distance = 2048 * t_min (NVIDIASVO.compute:163,171); +inf on miss */
    float    nx, ny, nz;/* normalize(decodeNormal(att[2p+1] >> 16)) (NVIDIASVO.compute:177-182) */
} orc_hit;

typedef struct orc_svo {
    int             format;     /* ORC_FMT_V1 / ORC_FMT_V2 */
    const int32_t  *desc;       /* V1 descriptors */
    const uint64_t *nodes;      /* V2 nodes */
    size_t          n_nodes;
    const uint32_t *att;        /* 2 words per node */
} orc_svo;

typedef struct orc_camera {
    float c2w[16];      /* Unity Matrix4x4, column-major: element (r,c) at [c*4+r] */
    float inv_proj[16]; /* idem */
    float px_off[2];    /* _PixelOffset */
    float light[4];     /* _DirectionalLight: forward xyz, intensity w */
} orc_camera;

/* ---- leaf functions ---- */
void orc_decode_normal(uint32_t value, float out[3]);                     /* AttachmentLookup.compute:37-61 */
void orc_decode_dxt_color(uint32_t head, uint32_t bits, int texel, float out[3]); /* :9-18 */
void orc_camera_ray(const orc_camera *cam, uint32_t px, uint32_t py, int width, int height,
                    float origin[3], float dir[3]);                       /* RaytraceCompute.compute:129-151 */

/* One IntersectSVO call.  rgb (nullable) receives the Shade() colour of a hit
 * (miss colour is the procedural sky, see orc_sky).  fetches (nullable)
 * receives the number of descriptor fetches (NVIDIASVO.compute:60-62). */
int  orc_intersect(const orc_svo *svo, const float origin[3], const float dir[3], int stack_mode,
                   orc_hit *hit, float albedo[3], uint32_t *fetches, uint32_t *iters);

/* orc_intersect plus bestHit.position (NVIDIASVO.compute:165-174: un-mirrored
 * voxel corner, (clamp(o' + 32 t * d, pos + eps, pos + size - eps) - 1.5) * 64;
 * misses 0) and the voxel key x | y << 21 | z << 42 (integer voxel coordinates
 * at the leaf scale = (bits(pos) & 0x7FFFFF) >> scale; misses all ones). */
int  orc_intersect_ex(const orc_svo *svo, const float origin[3], const float dir[3], int stack_mode,
                      orc_hit *hit, float albedo[3], uint32_t *fetches, uint32_t *iters,
                      float pos[3], uint64_t *voxel);

void orc_sky(const float dir[3], float out[3]);

/* Shadow ray toward -L from a primary hit; 1 if occluded (see svo_oracle.c). */
int  orc_shadow_ray_ex(const orc_svo *svo, const orc_camera *cam, const float o[3], const float d[3],
                       const orc_hit *h, int mode, uint32_t *iters_out);
int  orc_shadow_ray(const orc_svo *svo, const orc_camera *cam, const float o[3], const float d[3],
                    const orc_hit *hit, int stack_mode);

/* Render rows [y0, y1) of a width x height frame with `nthreads` threads.
 * hits / rgba / fetches are indexed by (y - y0) * width + x and are nullable. */
void orc_render(const orc_svo *svo, const orc_camera *cam, int width, int height,
                int y0, int y1, int stack_mode, int nthreads,
                orc_hit *hits, float *rgba, uint32_t *fetches);

/* orc_render plus float4 positions (w = 0) and voxel keys per pixel (nullable). */
void orc_render_ex(const orc_svo *svo, const orc_camera *cam, int width, int height,
                   int y0, int y1, int stack_mode, int nthreads,
                   orc_hit *hits, float *rgba, uint32_t *fetches, float *pos4, uint64_t *voxel);

/* Display RGBA8 words of n RGBA32F pixels (svo_frame.rgba8). */
void orc_pack_rgba8(const float *rgba, size_t n_px, uint32_t *out);

/* Render an explicit list of pixel indices (y * width + x). */
void orc_render_pixels(const orc_svo *svo, const orc_camera *cam, int width, int height,
                       const uint32_t *pixels, size_t n, int stack_mode, int nthreads,
                       orc_hit *hits, float *rgba, uint32_t *fetches);

/* Progressive accumulation, RaytracingMaster.cs:70-73 + AddShader.shader:44-47
 * (Blend SrcAlpha OneMinusSrcAlpha, alpha = 1/(_Sample+1)) on n RGBA float4
 * pixels: dst = src * a + dst * (1 - a), every channel, f32. */
void orc_accumulate(float *dst, const float *src, size_t n_px, uint32_t sample);

/* Relative (V1) -> V2 conversion used by the oracle's own V2 path. */
int  orc_v1_to_v2(const int32_t *desc, size_t n, uint64_t *nodes_out);

#ifdef __cplusplus
}
#endif
#endif
