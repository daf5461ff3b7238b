// svo_kernel.hip -- gfx950 primary-ray SVO traversal kernel (see svo_traverse.h).
//
// Line references are to the reference repo: NVIDIASVO.compute (N:),
// RaytraceCompute.compute (R:), AttachmentLookup.compute (A:).
#include "svo_traverse.h"

namespace svo {
namespace {

__device__ __forceinline__ void mul4(const float *m, float v0, float v1, float v2, float v3, float out[3]) {
    // HLSL mul(M, v), M column-major, summed left to right (unfused: -ffp-contract=off)
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        float a = m[0 * 4 + r] * v0;
        a = a + m[1 * 4 + r] * v1;
        a = a + m[2 * 4 + r] * v2;
        a = a + m[3 * 4 + r] * v3;
        out[r] = a;
    }
}

__device__ __forceinline__ void normalize3(float v[3]) {
    float d = v[0] * v[0];
    d = d + v[1] * v[1];
    d = d + v[2] * v[2];
    float inv = 1.0f / sqrtf(d);    // correctly rounded div + sqrt (no fast-math)
    v[0] = v[0] * inv;
    v[1] = v[1] * inv;
    v[2] = v[2] * inv;
}

// A:37-61
__device__ __forceinline__ void decode_normal(uint32_t value, float out[3]) {
    float t = (value & 0x8000u) ? -32768.0f : 32767.0f;
    float u = (float)((int32_t)(value << 19) >> 16);
    float v = (float)((int32_t)(value << 26) >> 16);
    if (value & 0x2000u) {
        out[0] = v; out[1] = t; out[2] = u;
    } else if (value & 0x4000u) {
        out[0] = u; out[1] = v; out[2] = t;
    } else {
        out[0] = t; out[1] = u; out[2] = v;
    }
}

// A:1-18
__device__ __forceinline__ void decode_dxt(uint32_t head, uint32_t bits, int texel, float out[3]) {
    const uint32_t sel = (bits >> (texel * 2)) & 3u;
    const float c0 = sel == 0 ? (1.0f / 16777216.0f)
                   : sel == 1 ? 0.0f
                   : sel == 2 ? (2.0f / 50331648.0f) : (1.0f / 50331648.0f);
    const float c1 = 1.0f / 16777216.0f - c0;
    float r = c0 * (float)(uint32_t)(head << 27) + c1 * (float)(uint32_t)(head << 11);
    float g = c0 * (float)(uint32_t)(head << 21) + c1 * (float)(uint32_t)(head << 5);
    float b = c0 * (float)(uint32_t)(head << 16) + c1 * (float)head;
    out[0] = r * (1.0f / 256.0f);
    out[1] = g * (1.0f / 256.0f);
    out[2] = b * (1.0f / 256.0f);
}

// HLSL float -> int (truncating, saturating; NaN -> 0) == v_cvt_i32_f32.
__device__ __forceinline__ int32_t hlsl_f2i(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (int32_t)0x80000000u;
    return (int32_t)f;
}

template <int MODE, bool COUNT>
__global__ __launch_bounds__(BLOCK) void render_kernel(LaunchParams p) {
    extern __shared__ uint2 stk[];   // [p.slots][BLOCK]
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int lr = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    if (x >= p.width || lr >= p.local_rows) return;
    const int band = lr / p.band_rows;
    const int y = (band * p.band_count + p.band_rank) * p.band_rows + (lr - band * p.band_rows);

    // ---- R:151 uv, R:129-141 CreateCameraRay ----
    const float u = ((float)x + p.cam.px_off[0]) / (float)p.width * 2.0f - 1.0f;
    const float v = ((float)y + p.cam.px_off[1]) / (float)p.height * 2.0f - 1.0f;
    float org[3], pd[3], dir[3];
    mul4(p.cam.c2w, 0.0f, 0.0f, 0.0f, 1.0f, org);
    mul4(p.cam.inv_proj, u, v, 0.0f, 1.0f, pd);
    mul4(p.cam.c2w, pd[0], pd[1], pd[2], 0.0f, dir);
    normalize3(dir);

    // ---- N:15-54 setup ----
    float ox = org[0] * (1.0f / 32.0f), oy = org[1] * (1.0f / 32.0f), oz = org[2] * (1.0f / 32.0f);
    ox = ox + 1.5f; oy = oy + 1.5f; oz = oz + 1.5f;
    const float tx_coef = 1.0f / -fabsf(dir[0]);
    const float ty_coef = 1.0f / -fabsf(dir[1]);
    const float tz_coef = 1.0f / -fabsf(dir[2]);
    float tx_bias = tx_coef * ox;
    float ty_bias = ty_coef * oy;
    float tz_bias = tz_coef * oz;
    int octant_mask = 7;
    if (dir[0] > 0.0f) { octant_mask ^= 1; tx_bias = 3.0f * tx_coef - tx_bias; }
    if (dir[1] > 0.0f) { octant_mask ^= 2; ty_bias = 3.0f * ty_coef - ty_bias; }
    if (dir[2] > 0.0f) { octant_mask ^= 4; tz_bias = 3.0f * tz_coef - tz_bias; }
    float t_min = fmaxf(fmaxf(2.0f * tx_coef - tx_bias, 2.0f * ty_coef - ty_bias), 2.0f * tz_coef - tz_bias);
    float t_max = fminf(fminf(tx_coef - tx_bias, ty_coef - ty_bias), tz_coef - tz_bias);
    float h = t_max;
    t_min = fmaxf(t_min, 0.0f);

    uint32_t parent = 0, cd = 0, first = 0;
    bool cached = false;
    int idx = 0;
    float px = 1.0f, py = 1.0f, pz = 1.0f;
    int scale = S_MAX - 1;
    float scale_exp2 = 0.5f;
    if (1.5f * tx_coef - tx_bias > t_min) { idx ^= 1; px = 1.5f; }
    if (1.5f * ty_coef - ty_bias > t_min) { idx ^= 2; py = 1.5f; }
    if (1.5f * tz_coef - tz_bias > t_min) { idx ^= 4; pz = 1.5f; }

    const int scale_lo = S_MAX - p.slots;   // lowest pushed scale
    uint32_t written = 0;                    // bit s: slot s written by this ray
    uint32_t fetches = 0;
    int iters = 0;
    uint32_t flags = 0;

    // ---- N:57-156 ----
    while (scale < S_MAX) {
        if (++iters > MAX_ITERS) { flags |= 2u; scale = S_MAX; break; }
        if (!cached) {                                     // N:60-62
            const uint2 nd = p.nodes[parent];
            cd = nd.x;
            first = nd.y;
            cached = (nd.x | nd.y) != 0u;
            if (COUNT) ++fetches;
        }
        const float tx_corner = px * tx_coef - tx_bias;
        const float ty_corner = py * ty_coef - ty_bias;
        const float tz_corner = pz * tz_coef - tz_bias;
        const float tc_max = fminf(fminf(tx_corner, ty_corner), tz_corner);

        const uint32_t child_masks = cd << (idx ^ octant_mask);
        if ((child_masks & 0x8000u) != 0u && t_min <= t_max) {
            const float tv_max = fminf(t_max, tc_max);
            const float half = scale_exp2 * 0.5f;
            const float tx_center = half * tx_coef + tx_corner;
            const float ty_center = half * ty_coef + ty_corner;
            const float tz_center = half * tz_coef + tz_corner;
            if (t_min <= tv_max) {
                if ((child_masks & 0x0080u) == 0u) break;   // leaf hit (N:93-94)
                if (tc_max < h) {                           // PUSH (N:97-98)
                    const int s = scale - scale_lo;
                    if (s < 0) { flags |= 4u; scale = S_MAX; break; }
                    uint2 e;
                    if (MODE == 0) {   // int2 <- float2((int)parent, asint(t_max))
                        e.x = (uint32_t)hlsl_f2i((float)(int32_t)parent);
                        e.y = (uint32_t)hlsl_f2i((float)__float_as_int(t_max));
                    } else {
                        e.x = parent;
                        e.y = (uint32_t)__float_as_int(t_max);
                    }
                    stk[s * BLOCK + tid] = e;
                    written |= 1u << s;
                }
                h = tc_max;
                parent = first + (uint32_t)__builtin_popcount(child_masks & 0x7Fu);   // N:101-105
                idx = 0;
                scale--;
                scale_exp2 = half;
                if (tx_center > t_min) { idx ^= 1; px = px + scale_exp2; }
                if (ty_center > t_min) { idx ^= 2; py = py + scale_exp2; }
                if (tz_center > t_min) { idx ^= 4; pz = pz + scale_exp2; }
                t_max = tv_max;
                cached = false;
                continue;
            }
        }
        // ADVANCE (N:122-128)
        int step_mask = 0;
        if (tx_corner <= tc_max) { step_mask ^= 1; px = px - scale_exp2; }
        if (ty_corner <= tc_max) { step_mask ^= 2; py = py - scale_exp2; }
        if (tz_corner <= tc_max) { step_mask ^= 4; pz = pz - scale_exp2; }
        t_min = tc_max;
        idx ^= step_mask;
        if ((idx & step_mask) != 0) {
            // POP (N:134-154)
            uint32_t differing = 0;
            if (step_mask & 1) differing |= (uint32_t)(__float_as_int(px) ^ __float_as_int(px + scale_exp2));
            if (step_mask & 2) differing |= (uint32_t)(__float_as_int(py) ^ __float_as_int(py + scale_exp2));
            if (step_mask & 4) differing |= (uint32_t)(__float_as_int(pz) ^ __float_as_int(pz + scale_exp2));
            scale = (__float_as_int((float)differing) >> 23) - 127;
            scale_exp2 = __int_as_float((scale - S_MAX + 127) << 23);
            const int s = scale - scale_lo;
            uint2 e = make_uint2(0u, 0u);
            if (s >= 0 && s < 32 && ((written >> s) & 1u)) e = stk[s * BLOCK + tid];
            parent = e.x;
            t_max = __int_as_float((int32_t)e.y);
            const int32_t shx = __float_as_int(px) >> scale;
            const int32_t shy = __float_as_int(py) >> scale;
            const int32_t shz = __float_as_int(pz) >> scale;
            px = __int_as_float((int32_t)((uint32_t)shx << scale));
            py = __int_as_float((int32_t)((uint32_t)shy << scale));
            pz = __int_as_float((int32_t)((uint32_t)shz << scale));
            idx = (shx & 1) | ((shy & 1) << 1) | ((shz & 1) << 2);
            h = 0.0f;
            cached = false;
        }
    }

    const size_t out = (size_t)lr * (size_t)p.width + (size_t)x;
    if (COUNT) {
        p.fetches[out] = fetches;
        return;
    }
    // ---- N:158-186 hit decode; R:93-127 Shade; R:167 store ----
    Hit hr;
    float rgb[3];
    if (scale >= S_MAX) {
        hr.parent = 0xFFFFFFFFu; hr.hit_idx = 0; hr.hit_scale = 0; hr.flags = (uint16_t)flags;
        hr.t = __int_as_float(0x7F800000); hr.nx = 0.0f; hr.ny = 0.0f; hr.nz = 0.0f;
        // procedural sky (the reference's skybox assets are missing), == orc_sky
        const float k = 0.5f * dir[1] + 0.5f;
        rgb[0] = 0.25f + 0.5f * k;
        rgb[1] = 0.35f + 0.55f * k;
        rgb[2] = 0.6f + 0.4f * k;
    } else {
        t_min = t_min * 32.0f;
        const int hit_idx = idx ^ octant_mask ^ 7;
        const uint2 a = p.att[parent];
        float n[3];
        decode_normal(a.y >> 16, n);
        normalize3(n);
        hr.parent = parent; hr.hit_idx = (uint8_t)hit_idx; hr.hit_scale = (uint8_t)scale;
        hr.flags = (uint16_t)(flags | 1u);
        hr.t = t_min * 64.0f;
        hr.nx = n[0]; hr.ny = n[1]; hr.nz = n[2];
        if (p.rgba) {
            float alb[3];
            decode_dxt(a.x, a.y, hit_idx, alb);
            float d = n[0] * p.cam.light[0];
            d = d + n[1] * p.cam.light[1];
            d = d + n[2] * p.cam.light[2];
            float s = d * -1.0f;
            s = fminf(fmaxf(s, 0.0f), 1.0f);
            s = s * p.cam.light[3];
            rgb[0] = s * alb[0]; rgb[1] = s * alb[1]; rgb[2] = s * alb[2];
        }
    }
    if (p.hits) {
        uint2 *dst = reinterpret_cast<uint2 *>(p.hits + out);
        dst[0] = make_uint2(hr.parent, (uint32_t)hr.hit_idx | ((uint32_t)hr.hit_scale << 8) | ((uint32_t)hr.flags << 16));
        dst[1] = make_uint2((uint32_t)__float_as_int(hr.t), (uint32_t)__float_as_int(hr.nx));
        dst[2] = make_uint2((uint32_t)__float_as_int(hr.ny), (uint32_t)__float_as_int(hr.nz));
    }
    if (p.rgba) p.rgba[out] = make_float4(rgb[0], rgb[1], rgb[2], 1.0f);
}

}  // namespace

hipError_t launch_render(const LaunchParams &p, int stack_mode, hipStream_t stream) {
    dim3 grid((unsigned)((p.width + 15) / 16), (unsigned)((p.local_rows + 15) / 16));
    size_t lds = (size_t)p.slots * BLOCK * sizeof(uint2);
    const bool count = p.fetches != nullptr;
    if (stack_mode == 0) {
        if (count) hipLaunchKernelGGL((render_kernel<0, true>), grid, dim3(BLOCK), lds, stream, p);
        else hipLaunchKernelGGL((render_kernel<0, false>), grid, dim3(BLOCK), lds, stream, p);
    } else {
        if (count) hipLaunchKernelGGL((render_kernel<1, true>), grid, dim3(BLOCK), lds, stream, p);
        else hipLaunchKernelGGL((render_kernel<1, false>), grid, dim3(BLOCK), lds, stream, p);
    }
    return hipGetLastError();
}

}  // namespace svo
