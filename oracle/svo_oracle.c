/*
 * svo_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * Plain-C, strict-IEEE restatement of the reference's per-pixel SVO ray path.
 * Build with -O2 -ffp-contract=off and WITHOUT -ffast-math (oracle/Makefile):
 * every a*b-c below must round twice, exactly as the HIP kernel does.
 *
 * Reference files (relative to the reference repo root):
 *   Assets/Shaders/NVIDIASVO.compute        IntersectSVO (line refs inline)
 *   Assets/Shaders/AttachmentLookup.compute decodeNormal / decodeDXTColor
 *   Assets/Shaders/RaytraceCompute.compute  CreateCameraRay / CSMain / Shade
 * See svo_oracle.h for the pinning status.
 */
#include "svo_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <string.h>
#include <limits.h>

#define S_MAX 23                 /* NVIDIASVO.compute:2 */
#define EPSILON_F 0.00000001f    /* NVIDIASVO.compute:1 (unused by the hit record) */
#define ORC_MAX_ITERS 65536      /* safety net; identical cap in the HIP kernel */

static inline int32_t f2i_bits(float f) { int32_t i; memcpy(&i, &f, 4); return i; }
static inline float i2f_bits(int32_t i) { float f; memcpy(&f, &i, 4); return f; }

/* HLSL float->int conversion (round toward zero, saturating). */
static inline int32_t hlsl_f2i(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return INT_MAX;
    if (f <= -2147483648.0f) return INT_MIN;
    return (int32_t)f;
}

/* AttachmentLookup.compute:37-61 */
void orc_decode_normal(uint32_t value, float out[3]) {
    float t = 32767.0f;
    if ((value & 0x8000u) != 0) t = -32768.0f;
    float u = (float)((int32_t)(value << 19) >> 16);
    float v = (float)((int32_t)(value << 26) >> 16);
    if ((value & 0x2000u) != 0) {
        out[0] = v; out[1] = t; out[2] = u;
    } else if ((value & 0x4000u) != 0) {
        out[0] = u; out[1] = v; out[2] = t;
    } else {
        out[0] = t; out[1] = u; out[2] = v;
    }
}

/* AttachmentLookup.compute:1-18 */
void orc_decode_dxt_color(uint32_t head, uint32_t bits, int texel, float out[3]) {
    static const float coefs[4] = {
        1.0f / 16777216.0f, 0.0f, 2.0f / 50331648.0f, 1.0f / 50331648.0f };
    float c0 = coefs[(bits >> (texel * 2)) & 3u];
    float c1 = 1.0f / 16777216.0f - c0;
    float r = c0 * (float)(uint32_t)(head << 27) + c1 * (float)(uint32_t)(head << 11);
    float g = c0 * (float)(uint32_t)(head << 21) + c1 * (float)(uint32_t)(head << 5);
    float b = c0 * (float)(uint32_t)(head << 16) + c1 * (float)head;
    out[0] = r * (1.0f / 256.0f);
    out[1] = g * (1.0f / 256.0f);
    out[2] = b * (1.0f / 256.0f);
}

/* HLSL mul(M, v): row r = ((M[r][0]*v0 + M[r][1]*v1) + M[r][2]*v2) + M[r][3]*v3,
 * M column-major (Unity Matrix4x4 memory order). */
static inline void mul4(const float *m, const float v[4], float out[3]) {
    for (int r = 0; r < 3; ++r) {
        float a = m[0 * 4 + r] * v[0];
        a = a + m[1 * 4 + r] * v[1];
        a = a + m[2 * 4 + r] * v[2];
        a = a + m[3 * 4 + r] * v[3];
        out[r] = a;
    }
}

static inline void normalize3(float v[3]) {
    float d = v[0] * v[0];
    d = d + v[1] * v[1];
    d = d + v[2] * v[2];
    float inv = 1.0f / sqrtf(d);
    v[0] = v[0] * inv; v[1] = v[1] * inv; v[2] = v[2] * inv;
}

/* RaytraceCompute.compute:151 (uv) + :129-141 (CreateCameraRay) */
void orc_camera_ray(const orc_camera *cam, uint32_t px, uint32_t py, int width, int height,
                    float origin[3], float dir[3]) {
    float u = ((float)px + cam->px_off[0]) / (float)width * 2.0f - 1.0f;
    float v = ((float)py + cam->px_off[1]) / (float)height * 2.0f - 1.0f;
    const float o4[4] = { 0.0f, 0.0f, 0.0f, 1.0f };
    mul4(cam->c2w, o4, origin);
    const float p4[4] = { u, v, 0.0f, 1.0f };
    float d[3];
    mul4(cam->inv_proj, p4, d);
    const float d4[4] = { d[0], d[1], d[2], 0.0f };
    mul4(cam->c2w, d4, dir);
    normalize3(dir);
}

void orc_sky(const float dir[3], float out[3]) {
    /* The reference samples a skybox texture whose assets are missing
     * (.MISSING_LARGE_BLOBS); this procedural gradient stands in for it and
     * miss pixels are excluded from the colour parity set. */
    float k = 0.5f * dir[1] + 0.5f;
    out[0] = 0.25f + 0.5f * k;
    out[1] = 0.35f + 0.55f * k;
    out[2] = 0.6f + 0.4f * k;
}

/* Fetch the node at `parent`.  Returns the low word in *lo (descriptor masks,
 * V1 keeps its whole word so the HLSL `child_descriptor == 0` test holds) and
 * the absolute first-child index in *first. */
static inline int fetch_node(const orc_svo *svo, uint32_t parent, uint32_t *lo, uint32_t *first) {
    if ((size_t)parent >= svo->n_nodes) {
        /* only an HLSL-rounded stack parent of a pool above 2^24 nodes gets here:
         * an out-of-range StructuredBuffer element reads as 0 */
        *lo = 0; *first = 0;
        return 0;
    }
    if (svo->format == ORC_FMT_V1) {
        uint32_t cd = (uint32_t)svo->desc[parent];
        *lo = cd;
        *first = parent + (cd >> 16);           /* NVIDIASVO.compute:101 relative pointer */
        return cd != 0;                         /* :60 `child_descriptor == 0` re-fetches */
    } else {
        uint64_t n = svo->nodes[parent];
        *lo = (uint32_t)n;
        *first = (uint32_t)(n >> 32);
        return n != 0;                          /* V2 node == 0  <=>  V1 word == 0 */
    }
}

/* NVIDIASVO.compute:12-198.  Returns 1 on hit.  pos_out / voxel_out (nullable):
 * bestHit.position (:165-174) and the voxel key of the hit leaf (see svo_oracle.h). */
int orc_intersect_ex(const orc_svo *svo, const float origin[3], const float dir[3], int stack_mode,
                     orc_hit *hit, float albedo[3], uint32_t *fetches_out, uint32_t *iters_out,
                     float pos_out[3], uint64_t *voxel_out) {
    int32_t stack_p[32];   /* parent, as stored (int2.x) */
    int32_t stack_t[32];   /* asint(t_max), as stored (int2.y) */
    memset(stack_p, 0, sizeof stack_p);   /* never-written entries read as zero */
    memset(stack_t, 0, sizeof stack_t);
    uint32_t fetches = 0, iters = 0;

    /* :15-19  world -> SVO cube [1,2]^3 */
    float ox = origin[0] * (1.0f / 32.0f);
    float oy = origin[1] * (1.0f / 32.0f);
    float oz = origin[2] * (1.0f / 32.0f);
    ox = ox + 1.5f; oy = oy + 1.5f; oz = oz + 1.5f;
    const float dx = dir[0], dy = dir[1], dz = dir[2];

    /* :27-38 */
    float tx_coef = 1.0f / -fabsf(dx);
    float ty_coef = 1.0f / -fabsf(dy);
    float tz_coef = 1.0f / -fabsf(dz);
    float tx_bias = tx_coef * ox;
    float ty_bias = ty_coef * oy;
    float tz_bias = tz_coef * oz;
    int octant_mask = 7;
    if (dx > 0.0f) { octant_mask ^= 1; tx_bias = 3.0f * tx_coef - tx_bias; }
    if (dy > 0.0f) { octant_mask ^= 2; ty_bias = 3.0f * ty_coef - ty_bias; }
    if (dz > 0.0f) { octant_mask ^= 4; tz_bias = 3.0f * tz_coef - tz_bias; }

    /* :40-44 (t_max is NOT clamped to 1 in the HLSL) */
    float t_min = fmaxf(fmaxf(2.0f * tx_coef - tx_bias, 2.0f * ty_coef - ty_bias), 2.0f * tz_coef - tz_bias);
    float t_max = fminf(fminf(tx_coef - tx_bias, ty_coef - ty_bias), tz_coef - tz_bias);
    float h = t_max;
    t_min = fmaxf(t_min, 0.0f);

    /* :46-54 */
    uint32_t parent = 0;
    uint32_t cd = 0, first = 0;    /* cached descriptor */
    int cached = 0;
    int idx = 0;
    float px = 1.0f, py = 1.0f, pz = 1.0f;
    int scale = S_MAX - 1;
    float scale_exp2 = 0.5f;
    if (1.5f * tx_coef - tx_bias > t_min) { idx ^= 1; px = 1.5f; }
    if (1.5f * ty_coef - ty_bias > t_min) { idx ^= 2; py = 1.5f; }
    if (1.5f * tz_coef - tz_bias > t_min) { idx ^= 4; pz = 1.5f; }

    uint16_t flags = 0;
    /* :57-156 */
    while (scale < S_MAX) {
        if (++iters > ORC_MAX_ITERS) { flags |= 2; scale = S_MAX; break; }
        if (!cached) { cached = fetch_node(svo, parent, &cd, &first); ++fetches; }   /* :60-62 */

        float tx_corner = px * tx_coef - tx_bias;
        float ty_corner = py * ty_coef - ty_bias;
        float tz_corner = pz * tz_coef - tz_bias;
        float tc_max = fminf(fminf(tx_corner, ty_corner), tz_corner);

        int child_shift = idx ^ octant_mask;
        uint32_t child_masks = cd << child_shift;
        if ((child_masks & 0x8000u) != 0 && t_min <= t_max) {
            float tv_max = fminf(t_max, tc_max);
            float half = scale_exp2 * 0.5f;
            float tx_center = half * tx_coef + tx_corner;
            float ty_center = half * ty_coef + ty_corner;
            float tz_center = half * tz_coef + tz_corner;
            if (t_min <= tv_max) {
                if ((child_masks & 0x0080u) == 0) break;   /* leaf hit :93-94 */
                /* PUSH :97-98 */
                if (tc_max < h) {
                    if (stack_mode == ORC_STACK_HLSL) {
                        /* int2 <- float2((int)parent, asint(t_max)) */
                        stack_p[scale] = hlsl_f2i((float)(int32_t)parent);
                        stack_t[scale] = hlsl_f2i((float)f2i_bits(t_max));
                    } else {
                        stack_p[scale] = (int32_t)parent;
                        stack_t[scale] = f2i_bits(t_max);
                    }
                }
                h = tc_max;
                /* :101-105 */
                parent = first + (uint32_t)__builtin_popcount(child_masks & 0x7Fu);
                idx = 0;
                scale--;
                scale_exp2 = half;
                if (tx_center > t_min) { idx ^= 1; px = px + scale_exp2; }
                if (ty_center > t_min) { idx ^= 2; py = py + scale_exp2; }
                if (tz_center > t_min) { idx ^= 4; pz = pz + scale_exp2; }
                t_max = tv_max;
                cached = 0;
                continue;
            }
        }
        /* ADVANCE :122-128 */
        int step_mask = 0;
        if (tx_corner <= tc_max) { step_mask ^= 1; px = px - scale_exp2; }
        if (ty_corner <= tc_max) { step_mask ^= 2; py = py - scale_exp2; }
        if (tz_corner <= tc_max) { step_mask ^= 4; pz = pz - scale_exp2; }
        t_min = tc_max;
        idx ^= step_mask;
        if ((idx & step_mask) != 0) {
            /* POP :134-154 */
            uint32_t differing_bits = 0;
            if ((step_mask & 1) != 0) differing_bits |= (uint32_t)(f2i_bits(px) ^ f2i_bits(px + scale_exp2));
            if ((step_mask & 2) != 0) differing_bits |= (uint32_t)(f2i_bits(py) ^ f2i_bits(py + scale_exp2));
            if ((step_mask & 4) != 0) differing_bits |= (uint32_t)(f2i_bits(pz) ^ f2i_bits(pz + scale_exp2));
            scale = (f2i_bits((float)differing_bits) >> 23) - 127;
            scale_exp2 = i2f_bits((scale - S_MAX + 127) << 23);
            parent = (uint32_t)stack_p[scale & 31];
            t_max = i2f_bits(stack_t[scale & 31]);
            int32_t shx = f2i_bits(px) >> scale;
            int32_t shy = f2i_bits(py) >> scale;
            int32_t shz = f2i_bits(pz) >> scale;
            px = i2f_bits((int32_t)((uint32_t)shx << scale));
            py = i2f_bits((int32_t)((uint32_t)shy << scale));
            pz = i2f_bits((int32_t)((uint32_t)shz << scale));
            idx = (shx & 1) | ((shy & 1) << 1) | ((shz & 1) << 2);
            h = 0.0f;
            cached = 0;
        }
    }
    if (fetches_out) *fetches_out = fetches;
    if (iters_out) *iters_out = iters;

    /* :158-161 miss: bestHit untouched (distance = +inf) */
    if (scale >= S_MAX) {
        hit->parent = 0xFFFFFFFFu; hit->hit_idx = 0; hit->hit_scale = 0; hit->flags = flags;
        hit->t = INFINITY; hit->nx = 0.0f; hit->ny = 0.0f; hit->nz = 0.0f;
        if (albedo) { albedo[0] = albedo[1] = albedo[2] = 0.0f; }
        if (pos_out) { pos_out[0] = pos_out[1] = pos_out[2] = 0.0f; }   /* CreateRayHit: position 0 */
        if (voxel_out) *voxel_out = ~(uint64_t)0;
        return 0;
    }
    /* :163-186 */
    t_min = t_min * 32.0f;
    {
        /* :165-168 undo the mirroring */
        if ((octant_mask & 1) == 0) px = 3.0f - scale_exp2 - px;
        if ((octant_mask & 2) == 0) py = 3.0f - scale_exp2 - py;
        if ((octant_mask & 4) == 0) pz = 3.0f - scale_exp2 - pz;
        /* :172-174: ray.origin is the SVO-space origin, t_min the x32-scaled one
         * (reference quirk), clamped into the voxel [pos + eps, pos + size - eps] */
        const float o3[3] = { ox, oy, oz }, d3[3] = { dx, dy, dz }, p3[3] = { px, py, pz };
        uint64_t key = 0;
        for (int k = 0; k < 3; ++k) {
            float hp = o3[k] + t_min * d3[k];
            float lo = p3[k] + EPSILON_F;
            float hi = p3[k] + scale_exp2 - EPSILON_F;
            float c = fminf(fmaxf(hp, lo), hi);
            if (pos_out) pos_out[k] = (c - 1.5f) * 64.0f;
            /* integer voxel coordinate at the leaf scale: the mantissa of the
             * un-mirrored corner (pos in [1, 2), dyadic) shifted by scale */
            key |= (uint64_t)(((uint32_t)f2i_bits(p3[k]) & 0x7FFFFFu) >> scale) << (21 * k);
        }
        if (voxel_out) *voxel_out = key;
    }
    int hit_idx = idx ^ octant_mask ^ 7;
    uint32_t blockA = svo->att[(size_t)parent * 2];
    uint32_t blockB = svo->att[(size_t)parent * 2 + 1];
    float n[3];
    orc_decode_normal(blockB >> 16, n);
    normalize3(n);
    hit->parent = parent;
    hit->hit_idx = (uint8_t)hit_idx;
    hit->hit_scale = (uint8_t)scale;
    hit->flags = (uint16_t)(flags | 1);
    hit->t = t_min * 64.0f;
    hit->nx = n[0]; hit->ny = n[1]; hit->nz = n[2];
    if (albedo) orc_decode_dxt_color(blockA, blockB, hit_idx, albedo);
    return 1;
}

int orc_intersect(const orc_svo *svo, const float origin[3], const float dir[3], int stack_mode,
                  orc_hit *hit, float albedo[3], uint32_t *fetches_out, uint32_t *iters_out) {
    return orc_intersect_ex(svo, origin, dir, stack_mode, hit, albedo, fetches_out, iters_out, NULL, NULL);
}

/* RaytraceCompute.compute:93-127 (hit branch :115) + :159-167.  The bounce
 * loop runs once (specular = 0); ray.energy is read before Shade zeroes it. */
static void shade_pixel(const orc_camera *cam, const orc_hit *hit, const float albedo[3],
                        const float dir[3], float out[4]) {
    if (hit->t < INFINITY) {
        float d = hit->nx * cam->light[0];
        d = d + hit->ny * cam->light[1];
        d = d + hit->nz * cam->light[2];
        float s = d * -1.0f;
        s = fminf(fmaxf(s, 0.0f), 1.0f);
        s = s * cam->light[3];
        out[0] = s * albedo[0]; out[1] = s * albedo[1]; out[2] = s * albedo[2];
    } else {
        orc_sky(dir, out);
    }
    out[3] = 1.0f;
}

/* Shadow ray of a primary hit (the reference's commented-out
 * test RaytraceCompute.compute:105-112 with a corrected origin): world hit point
 * P = o + (t / 64) * d (t = 2048 * t_svo, world distance = 32 * t_svo), origin
 * P + 0.001 * n, direction -L.  Returns 1 when the shadow ray hits a voxel. */
int orc_shadow_ray(const orc_svo *svo, const orc_camera *cam, const float o[3], const float d[3],
                   const orc_hit *h, int mode) {
    return orc_shadow_ray_ex(svo, cam, o, d, h, mode, NULL);
}

int orc_shadow_ray_ex(const orc_svo *svo, const orc_camera *cam, const float o[3], const float d[3],
                      const orc_hit *h, int mode, uint32_t *iters_out) {
    const float tw = h->t * (1.0f / 64.0f);
    const float n[3] = { h->nx, h->ny, h->nz };
    float so[3], sd[3];
    for (int k = 0; k < 3; ++k) {
        float pk = o[k] + tw * d[k];
        so[k] = pk + n[k] * 0.001f;
        sd[k] = -cam->light[k];
    }
    orc_hit sh;
    return orc_intersect(svo, so, sd, mode & 0xFF, &sh, NULL, NULL, iters_out);
}

static void trace_pixel(const orc_svo *svo, const orc_camera *cam, int width, int height,
                        uint32_t x, uint32_t y, int mode, orc_hit *hit_out, float *rgba_out,
                        uint32_t *fetch_out, float *pos_out, uint64_t *voxel_out) {
    float o[3], d[3], alb[3], pos[3];
    orc_hit h;
    uint32_t f = 0, it = 0;
    orc_camera_ray(cam, x, y, width, height, o, d);
    orc_intersect_ex(svo, o, d, mode & 0xFF, &h, alb, &f, &it, pos, voxel_out);
    if (pos_out) { pos_out[0] = pos[0]; pos_out[1] = pos[1]; pos_out[2] = pos[2]; pos_out[3] = 0.0f; }
    if (mode & ORC_COUNT_ITERS) f = it;   /* diagnostics: loop iterations instead of fetches */
    int shadowed = 0;
    if ((mode & ORC_SHADOW_RAYS) && (h.flags & 1)) {
        uint32_t sit = 0;
        shadowed = orc_shadow_ray_ex(svo, cam, o, d, &h, mode, &sit);
        if (shadowed) h.flags |= 8;   /* bit3: in shadow */
        if (mode & ORC_COUNT_SHADOW_ITERS) f = sit;
    } else if (mode & ORC_COUNT_SHADOW_ITERS) {
        f = 0;
    }
    if (hit_out) *hit_out = h;
    if (rgba_out) {
        shade_pixel(cam, &h, alb, d, rgba_out);
        if (shadowed) { rgba_out[0] = 0.0f; rgba_out[1] = 0.0f; rgba_out[2] = 0.0f; }   /* :109-111 */
    }
    if (fetch_out) *fetch_out = f;
}

typedef struct {
    const orc_svo *svo; const orc_camera *cam;
    int width, height, y0, y1, mode;
    const uint32_t *pixels; size_t n;
    orc_hit *hits; float *rgba; uint32_t *fetches; float *pos; uint64_t *voxel;
    atomic_long next;
} job_t;

static void *row_worker(void *arg) {
    job_t *j = (job_t *)arg;
    for (;;) {
        long y = atomic_fetch_add(&j->next, 1) + j->y0;
        if (y >= j->y1) break;
        for (int x = 0; x < j->width; ++x) {
            size_t k = (size_t)(y - j->y0) * (size_t)j->width + (size_t)x;
            trace_pixel(j->svo, j->cam, j->width, j->height, (uint32_t)x, (uint32_t)y, j->mode,
                        j->hits ? &j->hits[k] : NULL, j->rgba ? &j->rgba[4 * k] : NULL,
                        j->fetches ? &j->fetches[k] : NULL, j->pos ? &j->pos[4 * k] : NULL,
                        j->voxel ? &j->voxel[k] : NULL);
        }
    }
    return NULL;
}

static void *pixel_worker(void *arg) {
    job_t *j = (job_t *)arg;
    for (;;) {
        long b = atomic_fetch_add(&j->next, 1);
        size_t lo = (size_t)b * 256;
        if (lo >= j->n) break;
        size_t hi = lo + 256 < j->n ? lo + 256 : j->n;
        for (size_t k = lo; k < hi; ++k) {
            uint32_t p = j->pixels[k];
            trace_pixel(j->svo, j->cam, j->width, j->height, p % (uint32_t)j->width,
                        p / (uint32_t)j->width, j->mode, j->hits ? &j->hits[k] : NULL,
                        j->rgba ? &j->rgba[4 * k] : NULL, j->fetches ? &j->fetches[k] : NULL,
                        j->pos ? &j->pos[4 * k] : NULL, j->voxel ? &j->voxel[k] : NULL);
        }
    }
    return NULL;
}

static void run_threads(job_t *job, int nthreads, void *(*fn)(void *)) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    int started = 0;
    for (int i = 1; i < nthreads; ++i)
        if (pthread_create(&th[started], NULL, fn, job) == 0) ++started;
    fn(job);
    for (int i = 0; i < started; ++i) pthread_join(th[i], NULL);
}

void orc_render_ex(const orc_svo *svo, const orc_camera *cam, int width, int height,
                   int y0, int y1, int stack_mode, int nthreads,
                   orc_hit *hits, float *rgba, uint32_t *fetches, float *pos4, uint64_t *voxel) {
    job_t job;
    memset(&job, 0, sizeof job);
    job.svo = svo; job.cam = cam; job.width = width; job.height = height;
    job.y0 = y0; job.y1 = y1; job.mode = stack_mode;
    job.hits = hits; job.rgba = rgba; job.fetches = fetches; job.pos = pos4; job.voxel = voxel;
    atomic_init(&job.next, 0);
    run_threads(&job, nthreads, row_worker);
}

void orc_render(const orc_svo *svo, const orc_camera *cam, int width, int height,
                int y0, int y1, int stack_mode, int nthreads,
                orc_hit *hits, float *rgba, uint32_t *fetches) {
    orc_render_ex(svo, cam, width, height, y0, y1, stack_mode, nthreads, hits, rgba, fetches, NULL, NULL);
}

/* Display RGBA8 of Result colours: each channel (uint)(saturate(c) * 255 + 0.5),
 * alpha 255 (svo_rt.h svo_frame.rgba8; the reference blits RGBA32F to the screen
 * format, RaytracingMaster.cs:72). */
void orc_pack_rgba8(const float *rgba, size_t n_px, uint32_t *out) {
    for (size_t i = 0; i < n_px; ++i) {
        uint32_t w = 255u << 24;
        for (int c = 0; c < 3; ++c) {
            float v = fminf(fmaxf(rgba[4 * i + c], 0.0f), 1.0f);
            v = v * 255.0f;
            w |= (uint32_t)(v + 0.5f) << (8 * c);
        }
        out[i] = w;
    }
}

void orc_render_pixels(const orc_svo *svo, const orc_camera *cam, int width, int height,
                       const uint32_t *pixels, size_t n, int stack_mode, int nthreads,
                       orc_hit *hits, float *rgba, uint32_t *fetches) {
    job_t job;
    memset(&job, 0, sizeof job);
    job.svo = svo; job.cam = cam; job.width = width; job.height = height;
    job.mode = stack_mode; job.pixels = pixels; job.n = n;
    job.hits = hits; job.rgba = rgba; job.fetches = fetches;
    atomic_init(&job.next, 0);
    run_threads(&job, nthreads, pixel_worker);
}

/* AddShader.shader:44-47 returns float4(Result.rgb, 1/(_Sample+1)); the pass
 * blends with SrcAlpha / OneMinusSrcAlpha (:10), applied to all four channels
 * (src alpha channel = a).  _Sample is the uint _currentSample
 * (RaytracingMaster.cs:71-73), converted to float before the add. */
void orc_accumulate(float *dst, const float *src, size_t n_px, uint32_t sample) {
    const float a = 1.0f / ((float)sample + 1.0f);
    const float b = 1.0f - a;
    for (size_t i = 0; i < n_px; ++i) {
        for (int c = 0; c < 4; ++c) {
            const float s = c < 3 ? src[4 * i + c] : a;
            float lhs = s * a;
            float rhs = dst[4 * i + c] * b;
            dst[4 * i + c] = lhs + rhs;
        }
    }
}

int orc_v1_to_v2(const int32_t *desc, size_t n, uint64_t *nodes_out) {
    for (size_t i = 0; i < n; ++i) {
        uint32_t cd = (uint32_t)desc[i];
        uint32_t ptr = cd >> 16;
        uint32_t first = cd ? (uint32_t)i + ptr : 0u;   /* keeps node==0 <=> word==0 */
        nodes_out[i] = ((uint64_t)first << 32) | (uint64_t)(cd & 0xFFFFu);
    }
    return 0;
}
