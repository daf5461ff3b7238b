// svo_kernel.hip -- gfx950 primary-ray SVO traversal kernels (see svo_traverse.h).
//
// Line references are to the reference repo: NVIDIASVO.compute (N:),
// RaytraceCompute.compute (R:), AttachmentLookup.compute (A:).
//
// One launch shape: one lane per pixel, a wave64 (= a 64-thread workgroup) is
// an 8x8 pixel tile, tiles dispatched heaviest-first from the previous launch's
// recorded trip counts.  The traversal is the "lean" loop below, written for
// the wave: per-lane branch conditions are 64-bit lane masks in SGPRs, so
// divergent lanes share one instruction stream.  Forms measured slower in
// round 1 (branchy and branch-flattened per-lane steps, 128/256-thread blocks,
// a persistent kernel refilling lanes from a global counter, row-band XCD
// placement) were removed (DESIGN.md 5.1 keeps their numbers).
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

// HLSL float -> int: truncating, saturating, NaN -> 0 == v_cvt_i32_f32 itself.
__device__ __forceinline__ int32_t cvt_i32(float f) {
    int32_t r;
    asm volatile("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(f));
    return r;
}

// Display RGBA8 of a Result colour (alpha 1): saturate, * 255, round half up.
// == orc_pack_rgba8.
__device__ __forceinline__ uint32_t pack_rgba8(float r, float g, float b) {
    auto q = [](float c) {
        c = fminf(fmaxf(c, 0.0f), 1.0f);
        c = c * 255.0f;
        return (uint32_t)(c + 0.5f);
    };
    return q(r) | (q(g) << 8) | (q(b) << 16) | (255u << 24);
}

// Procedural sky (the reference's skybox assets are missing), == orc_sky.
__device__ __forceinline__ void sky(float dir_y, float rgb[3]) {
    const float k = 0.5f * dir_y + 0.5f;
    rgb[0] = 0.25f + 0.5f * k;
    rgb[1] = 0.35f + 0.55f * k;
    rgb[2] = 0.6f + 0.4f * k;
}

// R:93-127 hit branch (:115): saturate(-dot(n, L)) * L.w * albedo.  == shade_pixel.
__device__ __forceinline__ void shade_hit(const Camera &cam, const float n[3], const float alb[3], float rgb[3]) {
    float d = n[0] * cam.light[0];
    d = d + n[1] * cam.light[1];
    d = d + n[2] * cam.light[2];
    float s = d * -1.0f;
    s = fminf(fmaxf(s, 0.0f), 1.0f);
    s = s * cam.light[3];
    rgb[0] = s * alb[0]; rgb[1] = s * alb[1]; rgb[2] = s * alb[2];
}

struct Ray {
    float tx_coef, ty_coef, tz_coef, tx_bias, ty_bias, tz_bias;
    float t_min, t_max, h;
    float px, py, pz, scale_exp2;
    float dir_y;               // for the sky colour
    uint32_t parent;
    uint32_t fetches;
    int idx, octant_mask, scale;
    uint32_t flags;
};

// R:151 uv, R:129-141 CreateCameraRay
__device__ __forceinline__ void camera_ray(const Camera &cam, int width, int height, int x, int y, float org[3],
                                           float dir[3]) {
    const float u = ((float)x + cam.px_off[0]) / (float)width * 2.0f - 1.0f;
    const float v = ((float)y + cam.px_off[1]) / (float)height * 2.0f - 1.0f;
    float pd[3];
    mul4(cam.c2w, 0.0f, 0.0f, 0.0f, 1.0f, org);
    mul4(cam.inv_proj, u, v, 0.0f, 1.0f, pd);
    mul4(cam.c2w, pd[0], pd[1], pd[2], 0.0f, dir);
    normalize3(dir);
}

// N:15-19 world -> SVO cube [1, 2]^3
__device__ __forceinline__ float to_svo(float w) {
    const float s = w * (1.0f / 32.0f);
    return s + 1.5f;
}

// N:15-54 setup for a ray (origin, direction) in world space
__device__ __forceinline__ void setup_ray(const float org[3], const float dir[3], Ray &r) {
    r.dir_y = dir[1];
    const float ox = to_svo(org[0]), oy = to_svo(org[1]), oz = to_svo(org[2]);
    r.tx_coef = 1.0f / -fabsf(dir[0]);
    r.ty_coef = 1.0f / -fabsf(dir[1]);
    r.tz_coef = 1.0f / -fabsf(dir[2]);
    r.tx_bias = r.tx_coef * ox;
    r.ty_bias = r.ty_coef * oy;
    r.tz_bias = r.tz_coef * oz;
    r.octant_mask = 7;
    if (dir[0] > 0.0f) { r.octant_mask ^= 1; r.tx_bias = 3.0f * r.tx_coef - r.tx_bias; }
    if (dir[1] > 0.0f) { r.octant_mask ^= 2; r.ty_bias = 3.0f * r.ty_coef - r.ty_bias; }
    if (dir[2] > 0.0f) { r.octant_mask ^= 4; r.tz_bias = 3.0f * r.tz_coef - r.tz_bias; }
    r.t_min = fmaxf(fmaxf(2.0f * r.tx_coef - r.tx_bias, 2.0f * r.ty_coef - r.ty_bias), 2.0f * r.tz_coef - r.tz_bias);
    r.t_max = fminf(fminf(r.tx_coef - r.tx_bias, r.ty_coef - r.ty_bias), r.tz_coef - r.tz_bias);
    r.h = r.t_max;
    r.t_min = fmaxf(r.t_min, 0.0f);
    r.parent = 0;
    r.idx = 0;
    r.px = 1.0f; r.py = 1.0f; r.pz = 1.0f;
    r.scale = S_MAX - 1;
    r.scale_exp2 = 0.5f;
    if (1.5f * r.tx_coef - r.tx_bias > r.t_min) { r.idx ^= 1; r.px = 1.5f; }
    if (1.5f * r.ty_coef - r.ty_bias > r.t_min) { r.idx ^= 2; r.py = 1.5f; }
    if (1.5f * r.tz_coef - r.tz_bias > r.t_min) { r.idx ^= 4; r.pz = 1.5f; }
    r.fetches = 0; r.flags = 0;
}

// ------------------------------------------------------- lean traversal
// The tile-kernel loop: N:57-156 restructured for VALU issue, which is what
// bounds this kernel at 8 waves/SIMD:
//   * per-lane booleans (child index bits, octant mask, PUSH/ADVANCE/POP,
//     node cached) are held explicitly as 64-bit lane masks in SGPRs
//     (ballot / inverse_ballot), so the index algebra of N:83-154 is SALU
//     work that issues in parallel with other waves' VALU; the loop runs
//     while any lane is active (wave-uniform exit: finished lanes stay in
//     exec with every update gated off), so no lane-exit bookkeeping;
//   * scale is implied by scale_exp2 (an exact power of two);
//   * the stack is zeroed once per ray (never-written entries read as zero),
//     so no written-slot mask is kept, and entries are stored raw: the HLSL
//     float2 round trip (N:98) is applied when an entry is popped -- the same
//     function of the same bits, once per POP instead of once per PUSH;
//   * the iteration cap uses the wave-uniform trip count: all lanes of a tile
//     start together, so a lane still tracing after n trips has iterated n
//     times, exactly the per-ray count of the oracle;
//   * "t_min <= t_max" (N:79) is implied by "t_min <= min(t_max, tc_max)":
//     t_max is never NaN (a min over corner values of which at most two are
//     NaN, a popped stack value -- the round trip cannot create a NaN
//     pattern -- or zero).
typedef uint64_t lmask;

// fminf without the sNaN-quieting canonicalize LLVM adds for operands it
// cannot prove non-signalling (LDS-loaded t_max): every value here comes out
// of f32 arithmetic, so it is never a signalling NaN and v_min_f32 alone has
// fminf's semantics (NaN operand -> the other operand).
__device__ __forceinline__ float vmin(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// tx_center = half * tx_coef + tx_corner (N:111-113) as one fma: half is a power of
// two >= 2^-23 and |tx_coef| >= 1, so half * tx_coef is exact (no rounding, no
// underflow) and the fused result equals the two-rounding HLSL form bit for bit
__device__ __forceinline__ float center(float half, float coef, float corner) {
    return __builtin_fmaf(half, coef, corner);
}

// 3-bit per-lane integer b0 | b1 << 1 | b2 << 2 from three lane masks.
__device__ __forceinline__ int lanes_to_idx(uint64_t b0, uint64_t b1, uint64_t b2) {
    // three independent selects + one or: two dependent levels and no SGPR
    // carry hand-off (the add-with-carry form needed s_nop wait states between
    // its links; measured ~0.5 % slower)
    const int r0 = __builtin_amdgcn_inverse_ballot_w64(b0) ? 1 : 0;
    const int r1 = __builtin_amdgcn_inverse_ballot_w64(b1) ? 2 : 0;
    const int r2 = __builtin_amdgcn_inverse_ballot_w64(b2) ? 4 : 0;
    return r0 | r1 | r2;
}
#define LM_OF(c) __builtin_amdgcn_ballot_w64(c)
#define LM_ON(m) __builtin_amdgcn_inverse_ballot_w64(m)

struct FRay {
    float px, py, pz, cx, cy, cz, bx, by, bz;
    float t_min, t_max, h, sexp, dir_y;
    uint32_t parent, cd16, first, flags;
    uint32_t fetches;       // COUNT: descriptor fetches (N:60-62 executions)
    int idx, octant_mask;   // only at entry / exit
    int trips;              // wave-uniform loop trip count
};

__device__ __forceinline__ void to_fray(const Ray &r, FRay &f) {
    f.px = r.px; f.py = r.py; f.pz = r.pz;
    f.cx = r.tx_coef; f.cy = r.ty_coef; f.cz = r.tz_coef;
    f.bx = r.tx_bias; f.by = r.ty_bias; f.bz = r.tz_bias;
    f.t_min = r.t_min; f.t_max = r.t_max; f.h = r.h; f.sexp = r.scale_exp2; f.dir_y = r.dir_y;
    f.parent = 0; f.cd16 = 0; f.first = 0; f.flags = 0; f.fetches = 0;
    f.idx = r.idx; f.octant_mask = r.octant_mask;
}

// Back to the Ray fields the outputs read.
__device__ __forceinline__ void from_fray(const FRay &f, Ray &r) {
    const bool miss = f.sexp >= 1.0f || (f.flags & 6u) != 0u;
    r.scale = miss ? S_MAX : (int)(__float_as_uint(f.sexp) >> 23) - 104;
    r.idx = f.idx;
    r.octant_mask = f.octant_mask;
    r.t_min = f.t_min; r.parent = f.parent; r.flags = f.flags; r.dir_y = f.dir_y;
    r.px = f.px; r.py = f.py; r.pz = f.pz; r.scale_exp2 = f.sexp;
    r.fetches = f.fetches;
}

struct LeanDiag {            // DIAG instantiation only (env SVO_WAVE_LOG)
    uint64_t fetch_cycles = 0, loop_cycles = 0;   // fetch_cycles: push-only trips | adv-only trips << 16
    uint32_t fetch_trips = 0, pop_trips = 0;
};

template <int MODE, bool GUARD, bool DIAG = false, bool FETCH_ALL = false, bool COUNT = false>
__device__ __forceinline__ void trace_lean(const LaunchParams &p, FRay &r, uint2 *__restrict__ stk,
                                           LeanDiag *diag = nullptr) {
    // GUARD = false (host-proven, svo_rt.hip launch / recompute_depth): one tree of
    // known depth, fewer than 2^29 nodes, and (HLSL stack) parent indices below
    // 2^24, so a PUSH never overflows the stack, the HLSL round trip of a parent
    // index is the identity and node byte offsets fit 32 bits.
    constexpr int STRIDE = TILE;
    const int slots = p.slots;
    // a ray that leaves the root pops the top slot (the root's entry: parent 0) -- every lane,
    // finished ones too, fetches nodes[parent] on every trip (!GUARD), so it must hold a node
    for (int s = 0; s < slots; ++s) stk[s * STRIDE] = make_uint2(0u, 0u);
    const int scale_lo = S_MAX - slots;
    const float sexp_lo = __int_as_float((scale_lo - S_MAX + 127) << 23);   // push below scale_lo overflows
    lmask act = LM_OF(true);
    const int oct = r.octant_mask | 16;    // c ^ (oct | 16) == (c ^ oct) + 16
    int sh = r.idx ^ oct;                  // child index bits ^ oct: the descriptor shift (per lane, VGPR)
    lmask cached = 0, capped = 0, ovf = 0;
    const uint32_t stk_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint2 *)stk;
    constexpr uint32_t SLOT = (uint32_t)(STRIDE * sizeof(uint2));
    constexpr int SLOT_SH = 23 - 9;        // (bits >> 23) * SLOT with SLOT = 512
    static_assert(SLOT == (1u << (23 - SLOT_SH)), "stride must be 64 lanes");
    const uint32_t push_base = stk_base - (uint32_t)(104 + scale_lo) * SLOT;
    // POP: slot address from the exponent field e of float(differing), e = scale + 127
    const uint2 *stk_pop = stk - (127 + scale_lo) * STRIDE;   // indexed by e (never below slot 1)
    const uint32_t e_max = (uint32_t)(127 + scale_lo + slots - 1);   // leaving the root: the top slot
    int it = 0;
    uint64_t tl0 = 0;
    if (DIAG) tl0 = __builtin_amdgcn_s_memtime();
    // per-lane values from here on (works round an LLVM uniformity-analysis bug that
    // otherwise rejects the SGPR trip counter below: "illegal VGPR to SGPR copy")
    asm volatile("" : "+v"(r.parent), "+v"(r.cd16), "+v"(r.first));
    // one exit (no per-trip phi copies), the cap part of the test; a do-while with the
    // continue mask built in asm (s_cmp + s_cselect, then s_cmp_lg + branch: 4 SALU instead of
    // the 7 LLVM makes of `act != 0 && it < MAX_ITERS`; kernel -1 to -2 %).  On entry act != 0
    // (every lane of the wave traces) and it == 0.
    lmask go;
    do {
        // wave-uniform trip count kept in an SGPR (LLVM otherwise counts down in a VGPR)
        asm volatile("s_add_u32 %0, %0, 1" : "+s"(it) : : "scc");
        // N:60-62.  FETCH_ALL (!GUARD, pools below 2^24 nodes -- svo_rt.hip):
        // every lane fetches on every trip, unpredicated; re-fetching a cached node
        // reads the same word, and a load outside a divergent branch issues at the
        // top of the trip with nothing to wait for (C3: 5 % faster, 9 % on the
        // sky-heavy overview pose).  On the 25 M / 100 M-node pools of C4 / C5 the
        // extra loads cost 6-12 %, so those fetch only the lanes that need a node.
        // Every lane's parent is a valid index: a pool proven to be one tree, and
        // a ray that left the root popped the top (root) slot, whose parent is 0.
        constexpr bool ALWAYS = !GUARD && FETCH_ALL && !COUNT;
        const lmask need = ALWAYS ? ~(lmask)0 : act & ~cached;
        if (ALWAYS || LM_ON(need)) {
            // GUARD == false: pool below 2^29 nodes (svo_rt.hip), so the byte offset fits
            // 32 bits (global_load saddr + 32-bit voffset, no 64-bit address add).  GUARD: an
            // HLSL-rounded parent index (> 2^24 nodes) may lie outside the pool; it
            // reads as 0 like an out-of-range StructuredBuffer element.
            const uint2 nd = GUARD ? (r.parent < p.n_nodes ? p.nodes[r.parent] : make_uint2(0u, 0u))
                                   : *(const uint2 *)((const char *)p.nodes + (uint32_t)(r.parent << 3));
            r.cd16 = nd.x;
            r.first = nd.y;
            if (COUNT) r.fetches += 1u;
        }
        if (DIAG && need) diag->fetch_trips += 1;
        // COUNT keeps the HLSL re-fetch of a zero descriptor (N:60 `child_descriptor == 0`):
        // re-reading the same word changes no result, only the fetch count
        cached |= COUNT ? (need & LM_OF((r.cd16 | r.first) != 0u)) : need;
        // node-independent work first: it overlaps the fetch (waited for at the first use of cd16)
        const float tx = r.px * r.cx - r.bx;             // N:67-70
        const float ty = r.py * r.cy - r.by;
        const float tz = r.pz * r.cz - r.bz;
        const float tc_max = fminf(fminf(tx, ty), tz);
        const float tv_max = vmin(r.t_max, tc_max);
        const float half = r.sexp * 0.5f;                // N:111-116
        const lmask cx = LM_OF(center(half, r.cx, tx) > r.t_min);
        const lmask cy = LM_OF(center(half, r.cy, ty) > r.t_min);
        const lmask cz = LM_OF(center(half, r.cz, tz) > r.t_min);
        const lmask lx = LM_OF(tx <= tc_max), ly = LM_OF(ty <= tc_max), lz = LM_OF(tz <= tc_max);
        const lmask in_span = LM_OF(r.t_min <= tv_max), below_h = LM_OF(tc_max < r.h);
        const uint32_t cm = r.cd16 << sh;                // valid bit -> bit 31, leaf bit -> bit 23
        const lmask descend = act & LM_OF((int32_t)cm < 0) & in_span;
        const lmask leaf = LM_OF((cm & 0x00800000u) == 0u);
        const lmask hit = descend & leaf;                // N:93-94
        const lmask store = descend & ~leaf & below_h;
        const lmask of = GUARD ? (store & LM_OF(r.sexp < sexp_lo)) : (lmask)0;
        const lmask push = descend & ~leaf & ~of;
        const lmask adv = act & ~descend;
        if (DIAG) {   // wave-uniform trip kinds: PUSH lanes only / ADVANCE lanes only
            if (adv == 0 && push != 0) diag->fetch_cycles += 1;
            if (push == 0 && adv != 0) diag->fetch_cycles += 1u << 16;
        }
        if (LM_ON(store & ~of)) {                        // N:97-98 (t_max rounded here, parent on POP)
            // slot = scale - scale_lo = (bits(scale_exp2) >> 23) - 104 - scale_lo; two dwords by
            // ds_write2_b32: no copy into an aligned register pair.  scale_exp2 is an exact
            // power of two (zero mantissa), so the shift needs no mask
            const uint32_t a = push_base + (__float_as_uint(r.sexp) >> SLOT_SH);
            // HLSL stack (MODE 0): the float2 round trip of asint(t_max) (N:98, :141-143) is applied
            // here, when the entry is written -- a POP only ever reads a written entry or the zeroed
            // init, so the values are the same, and store trips are rarer than POP trips
            // (r02z A/B: Main pose -1.5 %, flyover +-0, profiles/r02z_ab_round_at_push.txt)
            const uint32_t tmw = MODE == 0 ? (uint32_t)cvt_i32((float)(int32_t)__float_as_uint(r.t_max))
                                           : __float_as_uint(r.t_max);
            asm volatile("ds_write2_b32 %0, %1, %2 offset1:1" : : "v"(a), "v"(r.parent), "v"(tmw) : "memory");
        }
        const lmask sx = adv & lx;                       // N:122-125
        const lmask sy = adv & ly;
        const lmask sz = adv & lz;
        const float se = r.sexp;
        const float delta = LM_ON(push) ? half : -se;
        const float ox = r.px, oy = r.py, oz = r.pz;
        // per axis: PUSH lanes move into the child half, ADVANCE lanes step (PUSH and
        // ADVANCE lanes are disjoint, so one mask per axis serves both)
        const lmask mvx = (push & cx) | sx, mvy = (push & cy) | sy, mvz = (push & cz) | sz;
        const float qx = r.px + (LM_ON(mvx) ? delta : 0.0f);
        const float qy = r.py + (LM_ON(mvy) ? delta : 0.0f);
        const float qz = r.pz + (LM_ON(mvz) ? delta : 0.0f);
        // the same three masks as an integer: the child index on PUSH lanes (N:111-116),
        // the step mask on ADVANCE lanes (N:122-128), 0 elsewhere
        const int mv = lanes_to_idx(mvx, mvy, mvz);
        const lmask pop = adv & LM_OF((mv & ~(sh ^ oct)) != 0);   // N:130-131: (idx ^ step) & step
        const uint32_t child = r.first + (uint32_t)__builtin_popcount(cm & 0x007F0000u);
        sh = (LM_ON(push) ? oct : sh) ^ mv;             // PUSH: idx = mv, else idx ^= mv
        if (LM_ON(push)) {   // an exec-masked block: 4 selects instead cost +1 % / +3.5 % (r03j)
            r.parent = child;
            r.h = tc_max;
            r.t_max = tv_max;
            r.sexp = half;
        }
        r.t_min = LM_ON(adv) ? tc_max : r.t_min;
        cached &= ~(push | pop);
        r.px = qx; r.py = qy; r.pz = qz;
        lmask out = 0;
        if (pop != 0) {                                  // N:134-154
            // Evaluated by the whole wave (a divergent region costs exec
            // bookkeeping and copies of values live on both sides); the popping
            // lanes take the results.  Other lanes read an in-range slot.
            if (DIAG) diag->pop_trips += 1;
            // stepped axis: q + scale_exp2 == o exactly (multiples of scale_exp2 in [0.5, 2));
            // unstepped axis: q == o, xor 0 -- N:135-137 without masks or re-adds
            const uint32_t diff = (__float_as_uint(ox) ^ __float_as_uint(qx)) |
                                  (__float_as_uint(oy) ^ __float_as_uint(qy)) |
                                  (__float_as_uint(oz) ^ __float_as_uint(qz));
            const uint32_t fd = __float_as_uint((float)diff);
            const uint32_t ef = __builtin_amdgcn_ubfe(fd, 23, 8);   // scale + 127
            const int scale = (int)ef - 127;
            const uint2 e = stk_pop[min(ef, e_max) * STRIDE];   // e_max: leaving the root
            uint32_t pa = e.x, tm = e.y;
            if (MODE == 0) {                             // int2 <- float2((int)parent, asint(t_max))
                if (GUARD) pa = (uint32_t)cvt_i32((float)(int32_t)pa);
                // tm: rounded when it was written
            }
            const uint32_t keep = 0xFFFFFFFFu << scale;
            const uint32_t bx_ = __builtin_amdgcn_ubfe(__float_as_uint(qx), scale, 1);
            const uint32_t by_ = __builtin_amdgcn_ubfe(__float_as_uint(qy), scale, 1);
            const uint32_t bz_ = __builtin_amdgcn_ubfe(__float_as_uint(qz), scale, 1);
            const bool pl = LM_ON(pop);
            r.sexp = pl ? __uint_as_float((ef << 23) - (23u << 23)) : r.sexp;
            r.parent = pl ? pa : r.parent;
            r.t_max = pl ? __uint_as_float(tm) : r.t_max;
            // one select of the mask, then in-place ands (r.p == q here)
            const uint32_t k = pl ? keep : 0xFFFFFFFFu;
            r.px = __uint_as_float(__float_as_uint(r.px) & k);
            r.py = __uint_as_float(__float_as_uint(r.py) & k);
            r.pz = __uint_as_float(__float_as_uint(r.pz) & k);
            r.h = pl ? 0.0f : r.h;
            sh = pl ? (int)(bx_ | (by_ << 1) | (bz_ << 2)) ^ oct : sh;
            out = pop & LM_OF(scale >= S_MAX);
        }
        ovf |= of;
        act &= ~(hit | of | out);
        asm volatile("s_cmp_lt_u32 %1, %2\n\ts_cselect_b64 %0, %3, 0" : "=s"(go) : "s"(it), "n"(MAX_ITERS), "s"(act) : "scc");
    } while (go != 0);
    capped = act;                          // still tracing after MAX_ITERS trips
    if (DIAG) diag->loop_cycles = __builtin_amdgcn_s_memtime() - tl0;
    r.idx = sh ^ oct;
    r.trips = it;
    if (LM_ON(capped)) r.flags |= 2u;
    if (LM_ON(ovf)) r.flags |= 4u;
}

// ------------------------------------------------------- latency form
// trace_lean for launches that leave wave slots empty (svo_rt.hip launch: a strong split's
// per-GPU band, a lone tile row): there a wave's serial trip chain, not the SIMD's issue
// rate, bounds the launch, and the node fetch at the top of every trip is
// the longest link of that chain (~L1 latency, after a POP also behind the stack read).
// Same decisions, same arithmetic, same results; two changes to where the node comes from:
//   * the stack entry also keeps the parent's node word (a second [slot][lane] uint2 array
//     behind the {parent, t_max} one: 16 B per entry, 10 KB per wave at depth 10), so a
//     POP takes the node from LDS with its parent instead of fetching it afterwards;
//   * the next trip's node is loaded as soon as it is known, mid-trip: nodes[child] for
//     PUSH lanes, the current node again for the others (an L1 hit), so the load's
//     latency overlaps the rest of the trip instead of opening the next one.
// !GUARD pools only (one tree, exact parents): the load offset is 32-bit and no parent
// round trip is needed.  LDS doubles, so occupancy halves -- the reason this form is not
// the full-frame default.
template <int MODE>
__device__ __forceinline__ void trace_lat(const LaunchParams &p, FRay &r, uint2 *__restrict__ stk) {
    constexpr int STRIDE = TILE;
    const int slots = p.slots;
    const int nodes_off = slots * STRIDE;   // the node half of an entry, in uint2 units
    for (int s = 0; s < slots; ++s) {
        stk[s * STRIDE] = make_uint2(0u, 0u);
        stk[nodes_off + s * STRIDE] = make_uint2(0u, 0u);
    }
    const int scale_lo = S_MAX - slots;
    lmask act = LM_OF(true);
    const int oct = r.octant_mask | 16;
    int sh = r.idx ^ oct;
    const uint32_t stk_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint2 *)stk;
    constexpr uint32_t SLOT = (uint32_t)(STRIDE * sizeof(uint2));
    constexpr int SLOT_SH = 23 - 9;
    const uint32_t push_base = stk_base - (uint32_t)(104 + scale_lo) * SLOT;
    const uint32_t node_bytes = (uint32_t)nodes_off * (uint32_t)sizeof(uint2);
    const uint2 *stk_pop = stk - (127 + scale_lo) * STRIDE;
    const uint32_t e_max = (uint32_t)(127 + scale_lo + slots - 1);
    int it = 0;
    asm volatile("" : "+v"(r.parent));
    // the root's node: every ray starts at node 0
    uint2 pf = *(const uint2 *)((const char *)p.nodes + (uint32_t)(r.parent << 3));
    uint2 nd_pop = make_uint2(0u, 0u);
    lmask popped = 0;
    lmask go;
    do {
        asm volatile("s_add_u32 %0, %0, 1" : "+s"(it) : : "scc");
        // node-independent work first (it overlaps the wait for this trip's node)
        const float tx = r.px * r.cx - r.bx;             // N:67-70
        const float ty = r.py * r.cy - r.by;
        const float tz = r.pz * r.cz - r.bz;
        const float tc_max = fminf(fminf(tx, ty), tz);
        const float tv_max = vmin(r.t_max, tc_max);
        const float half = r.sexp * 0.5f;                // N:111-116
        const lmask cx = LM_OF(center(half, r.cx, tx) > r.t_min);
        const lmask cy = LM_OF(center(half, r.cy, ty) > r.t_min);
        const lmask cz = LM_OF(center(half, r.cz, tz) > r.t_min);
        const lmask lx = LM_OF(tx <= tc_max), ly = LM_OF(ty <= tc_max), lz = LM_OF(tz <= tc_max);
        const lmask in_span = LM_OF(r.t_min <= tv_max), below_h = LM_OF(tc_max < r.h);
        // this trip's node (N:60-62): popped from the stack, or loaded during the last trip
        const uint2 nd = LM_ON(popped) ? nd_pop : pf;
        const uint32_t cm = nd.x << sh;                  // valid bit -> bit 31, leaf bit -> bit 23
        const lmask descend = act & LM_OF((int32_t)cm < 0) & in_span;
        const lmask leaf = LM_OF((cm & 0x00800000u) == 0u);
        const lmask hit = descend & leaf;                // N:93-94
        const lmask store = descend & ~leaf & below_h;
        const lmask push = descend & ~leaf;
        const lmask adv = act & ~descend;
        const uint32_t child = nd.y + (uint32_t)__builtin_popcount(cm & 0x007F0000u);
        // the next trip's node, as early as it is known: the child for PUSH lanes, this node
        // again for the others (a POP lane takes its node from the stack instead)
        pf = *(const uint2 *)((const char *)p.nodes + (uint32_t)((LM_ON(push) ? child : r.parent) << 3));
        if (LM_ON(store)) {                              // N:97-98, + the parent's node
            const uint32_t a = push_base + (__float_as_uint(r.sexp) >> SLOT_SH);
            const uint32_t tmw = MODE == 0 ? (uint32_t)cvt_i32((float)(int32_t)__float_as_uint(r.t_max))
                                           : __float_as_uint(r.t_max);
            asm volatile("ds_write2_b32 %0, %1, %2 offset1:1" : : "v"(a), "v"(r.parent), "v"(tmw) : "memory");
            asm volatile("ds_write2_b32 %0, %1, %2 offset1:1" : : "v"(a + node_bytes), "v"(nd.x), "v"(nd.y) : "memory");
        }
        const lmask sx = adv & lx;                       // N:122-125
        const lmask sy = adv & ly;
        const lmask sz = adv & lz;
        const float se = r.sexp;
        const float delta = LM_ON(push) ? half : -se;
        const float ox = r.px, oy = r.py, oz = r.pz;
        const lmask mvx = (push & cx) | sx, mvy = (push & cy) | sy, mvz = (push & cz) | sz;
        const float qx = r.px + (LM_ON(mvx) ? delta : 0.0f);
        const float qy = r.py + (LM_ON(mvy) ? delta : 0.0f);
        const float qz = r.pz + (LM_ON(mvz) ? delta : 0.0f);
        const int mv = lanes_to_idx(mvx, mvy, mvz);
        const lmask pop = adv & LM_OF((mv & ~(sh ^ oct)) != 0);   // N:130-131
        sh = (LM_ON(push) ? oct : sh) ^ mv;
        if (LM_ON(push)) {
            r.parent = child;
            r.h = tc_max;
            r.t_max = tv_max;
            r.sexp = half;
        }
        r.t_min = LM_ON(adv) ? tc_max : r.t_min;
        r.px = qx; r.py = qy; r.pz = qz;
        lmask out = 0;
        if (pop != 0) {                                  // N:134-154
            const uint32_t diff = (__float_as_uint(ox) ^ __float_as_uint(qx)) |
                                  (__float_as_uint(oy) ^ __float_as_uint(qy)) |
                                  (__float_as_uint(oz) ^ __float_as_uint(qz));
            const uint32_t fd = __float_as_uint((float)diff);
            const uint32_t ef = __builtin_amdgcn_ubfe(fd, 23, 8);   // scale + 127
            const int scale = (int)ef - 127;
            const uint32_t slot = min(ef, e_max) * STRIDE;
            const uint2 e = stk_pop[slot];
            nd_pop = stk_pop[nodes_off + slot];
            const uint32_t keep = 0xFFFFFFFFu << scale;
            const uint32_t bx_ = __builtin_amdgcn_ubfe(__float_as_uint(qx), scale, 1);
            const uint32_t by_ = __builtin_amdgcn_ubfe(__float_as_uint(qy), scale, 1);
            const uint32_t bz_ = __builtin_amdgcn_ubfe(__float_as_uint(qz), scale, 1);
            const bool pl = LM_ON(pop);
            r.sexp = pl ? __uint_as_float((ef << 23) - (23u << 23)) : r.sexp;
            r.parent = pl ? e.x : r.parent;
            r.t_max = pl ? __uint_as_float(e.y) : r.t_max;
            const uint32_t k = pl ? keep : 0xFFFFFFFFu;
            r.px = __uint_as_float(__float_as_uint(r.px) & k);
            r.py = __uint_as_float(__float_as_uint(r.py) & k);
            r.pz = __uint_as_float(__float_as_uint(r.pz) & k);
            r.h = pl ? 0.0f : r.h;
            sh = pl ? (int)(bx_ | (by_ << 1) | (bz_ << 2)) ^ oct : sh;
            out = pop & LM_OF(scale >= S_MAX);
        }
        popped = pop;
        act &= ~(hit | out);
        asm volatile("s_cmp_lt_u32 %1, %2\n\ts_cselect_b64 %0, %3, 0" : "=s"(go) : "s"(it), "n"(MAX_ITERS), "s"(act) : "scc");
    } while (go != 0);
    r.idx = sh ^ oct;
    r.trips = it;
    if (LM_ON(act)) r.flags |= 2u;                       // still tracing after MAX_ITERS trips
}

// Everything one finished primary ray writes.
struct Record {
    uint32_t w[6];      // the svo_hit words; w[0..2] = the compact record
    float rgb[3];       // Result colour (alpha 1)
    float pos[3];       // bestHit.position (misses: 0, CreateRayHit)
    unsigned long long key;   // voxel key (misses: all ones)
};

// N:158-186 hit decode + R:93-127 Shade.  (x, gy): the pixel, for the hit
// position's ray origin (recomputed, not kept live through the loop).
__device__ __forceinline__ void record(const LaunchParams &p, const Ray &r, int x, int gy, Record &o) {
    o.pos[0] = o.pos[1] = o.pos[2] = 0.0f;
    o.key = ~0ull;
    if (r.scale >= S_MAX) {
        o.w[0] = 0xFFFFFFFFu;
        o.w[1] = (r.flags & 0xFFFFu) << 16;
        o.w[2] = 0x7F800000u;
        o.w[3] = 0u; o.w[4] = 0u; o.w[5] = 0u;
        sky(r.dir_y, o.rgb);
        return;
    }
    const float t_min = r.t_min * 32.0f;                  // N:163
    const int hit_idx = r.idx ^ r.octant_mask ^ 7;        // N:176
    const uint2 a = p.att[r.parent];                      // N:177-178
    float n[3];
    decode_normal(a.y >> 16, n);
    normalize3(n);
    o.w[0] = r.parent;
    o.w[1] = (uint32_t)hit_idx | ((uint32_t)r.scale << 8) | (((r.flags | 1u) & 0xFFFFu) << 16);
    o.w[2] = (uint32_t)__float_as_int(t_min * 64.0f);    // N:171
    o.w[3] = (uint32_t)__float_as_int(n[0]);
    o.w[4] = (uint32_t)__float_as_int(n[1]);
    o.w[5] = (uint32_t)__float_as_int(n[2]);
    o.rgb[0] = o.rgb[1] = o.rgb[2] = 0.0f;
    if (p.out.rgba || p.out.rgba8 || p.out.rgb8 || p.out.accum) {
        float alb[3];
        decode_dxt(a.x, a.y, hit_idx, alb);
        shade_hit(p.cam, n, alb, o.rgb);
    }
    if (p.out.position || p.out.voxel) {
        // N:165-174: undo the mirroring, then clamp the (x32-scaled, reference quirk)
        // hit point into the voxel and scale it by 64.  Voxel key: the un-mirrored
        // corner's mantissa bits at the leaf scale (exact: positions are dyadic).
        float org[3], dir[3];
        camera_ray(p.cam, p.width, p.height, x, gy, org, dir);
        const float se = r.scale_exp2;
        float q[3] = { r.px, r.py, r.pz };
        unsigned long long key = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (((r.octant_mask >> k) & 1) == 0) q[k] = (3.0f - se) - q[k];
            const float hp = to_svo(org[k]) + t_min * dir[k];
            const float lo = q[k] + 0.00000001f;
            const float hi = (q[k] + se) - 0.00000001f;
            const float c = fminf(fmaxf(hp, lo), hi);
            o.pos[k] = (c - 1.5f) * 64.0f;
            key |= (unsigned long long)((__float_as_uint(q[k]) & 0x7FFFFFu) >> r.scale) << (21 * k);
        }
        o.key = key;
    }
}

// Output stores are non-temporal (global_store ... nt): the frame's 40-84 MB of records and
// colours stream through L2 once, and with the default policy they evict the node pool's lines
// there -- a trip whose node fetch misses L1 (most wave trips have one such lane) then waits on
// the Infinity Cache instead of L2.  C3 flyover kernel 0.1066 -> 0.1030 ms, Main pose -0.8 %
// (profiles/r03n_ab_nt_stores.txt).
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// The one-sample route's read of the accumulation (0 elsewhere; a non-temporal load measured 3 %
// slower).
__device__ __forceinline__ float4 accum_load(const LaunchParams &p, size_t i) {
    if (!p.out.accum) return make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    return p.out.accum[i];
}

// d0: out.accum[i] when out.accum is set, loaded by the caller right after its trace and before
// `record`, so its memory latency overlaps the attachment fetch of the shading instead of following
// it (loaded before the trace it would hold up the first trip: loads retire in order)
__device__ __forceinline__ void store_outputs(const Outputs &out, size_t i, const Record &o,
                                              float4 d0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f)) {
    // the words as scalars first: vectors built straight from the array kept it in private memory
    // in render_seg_kernel
    const uint32_t w0 = o.w[0], w1 = o.w[1], w2 = o.w[2], w3 = o.w[3], w4 = o.w[4], w5 = o.w[5];
    if (out.hits) {
        u32x2 *dst = reinterpret_cast<u32x2 *>(out.hits + i);
        __builtin_nontemporal_store(u32x2{w0, w1}, dst + 0);
        __builtin_nontemporal_store(u32x2{w2, w3}, dst + 1);
        __builtin_nontemporal_store(u32x2{w4, w5}, dst + 2);
    }
    if (out.compact)
        // a 3-vector is 16 bytes apart in arrays: address the 12-byte record explicitly
        __builtin_nontemporal_store(u32x3{w0, w1, w2}, reinterpret_cast<u32x3 *>(out.compact + 3 * i));
    if (out.rgba)
        __builtin_nontemporal_store(f32x4{o.rgb[0], o.rgb[1], o.rgb[2], 1.0f}, reinterpret_cast<f32x4 *>(out.rgba + i));
    float dr = o.rgb[0], dg = o.rgb[1], db = o.rgb[2];   // the colour the display words carry
    if (out.accum) {   // accumulate_kernel's blend (AddShader.shader:44-47), the Result alpha is a
        const float a = out.acc_a, b = out.acc_b;
        dr = o.rgb[0] * a + d0.x * b;
        dg = o.rgb[1] * a + d0.y * b;
        db = o.rgb[2] * a + d0.z * b;
        const float dw = a * a + d0.w * b;
        __builtin_nontemporal_store(f32x4{dr, dg, db, dw}, reinterpret_cast<f32x4 *>(out.accum + i));
    }
    if (out.rgba8 || out.rgb8) {
        const uint32_t w = pack_rgba8(dr, dg, db);
        if (out.rgba8) __builtin_nontemporal_store(w, out.rgba8 + i);
        if (out.rgb8) {
            uint8_t *d = out.rgb8 + 3 * i;
            d[0] = (uint8_t)w;
            d[1] = (uint8_t)(w >> 8);
            d[2] = (uint8_t)(w >> 16);
        }
    }
    if (out.position)
        __builtin_nontemporal_store(f32x4{o.pos[0], o.pos[1], o.pos[2], 0.0f}, reinterpret_cast<f32x4 *>(out.position + i));
    if (out.voxel) __builtin_nontemporal_store(o.key, out.voxel + i);
}

// Shadow ray of a primary hit (the reference's test is commented
// out at RaytraceCompute.compute:105-112): world hit point P = o + (t / 64) d (t =
// the record's 2048 t_svo), origin P + 0.001 n, direction -L.  == orc_shadow_ray.
__device__ __forceinline__ void shadow_ray(const LaunchParams &p, int x, int y, uint32_t w_t, uint32_t w_nx,
                                           uint32_t w_ny, uint32_t w_nz, float so[3], float sd[3]) {
    float org[3], dir[3];
    camera_ray(p.cam, p.width, p.height, x, y, org, dir);
    const float tw = __int_as_float((int32_t)w_t) * (1.0f / 64.0f);
    const float n[3] = { __int_as_float((int32_t)w_nx), __int_as_float((int32_t)w_ny), __int_as_float((int32_t)w_nz) };
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float pk = org[k] + tw * dir[k];
        so[k] = pk + n[k] * 0.001f;
        sd[k] = -p.cam.light[k];
    }
}

__device__ __forceinline__ int global_row(const LaunchParams &p, int lr) {
    const int j = lr / p.band_rows;
    const int in = lr - j * p.band_rows;
    if (p.band_cycle == 0) return (j * p.band_count + p.band_rank) * p.band_rows + in;
    const int c = j / p.band_cnt;
    return (c * p.band_cycle + (int)p.band_pos[j - c * p.band_cnt]) * p.band_rows + in;
}

__device__ __forceinline__ size_t out_index(const LaunchParams &p, int lr, int gy, int x) {
    return (size_t)(p.out.frame_layout ? gy : lr) * (size_t)p.width + (size_t)x;
}

// ------------------------------------------------------------- segmented rays
// One ray's traversal split into K t-segments that run side by side (VERDICT r4 item 1:
// a heavy tile's wave is a serial chain of up to ~270 trips that bounds a frame split over N
// GPUs; modelled first, tools/segment_model.py).  Segment k of a ray with
// starts t_1 .. t_{K-1} (any floats, NaN included: the result never depends on them, only the
// balance does) runs the lean loop from the cube entry with three changes:
//   * SKIP: a non-leaf child it would descend into whose exit tc_max is below t_k lies wholly
//     before t_k.  The lane instead takes the state the loop has after descending into it and
//     popping back -- the stack entry that PUSH stores (N:97-98, also when h allows it), t_max
//     through the HLSL float2 round trip (N:141-143), h = 0 (N:153) -- and ADVANCEs past it.
//     Every ADVANCE inside such a subtree has t_min <= its tc_max < t_k (the corner times
//     p * coef - bias are monotone in p, so a sub-cell's exit cannot pass its parent's), so the
//     lane follows the continuous loop's own path, state for state, minus those subtrees.
//   * ARM: a hit (N:93-94) counts only once the lane is armed: segment 0 from the start,
//     segment k at the first ADVANCE whose new t_min >= t_k (before it, a leaf is stepped past).
//   * STOP: segment k ends, without a hit, at the first ADVANCE whose new t_min >= t_{k+1} --
//     the very event that arms segment k + 1 on the same path.
// The ray's record is that of its first segment that did not stop (a hit, or the ray left
// the cube): the segments before it covered everything up to its arming event without a hit.
// Bit-identical to the continuous loop in both stack modes (tests/test_gpu_seg.py against the
// oracle, with real and with random starts).
// SEGS = false: one segment from t_start with no stop (a beam start): no STOP test
// and no per-lane trip bookkeeping.
// COUNT: per-lane descriptor fetches in r.fetches, with the HLSL re-fetch of a zero descriptor
// (trace_lean's COUNT form; svo_count_fetches under SVO_OPT_COUNT_BEAM).
// Lanes k of each KG-lane segment group (lanes KG r .. KG r + KG - 1 = ray r) that have a lane
// j < k of their group in m: an exclusive prefix OR inside the groups, on the wave's lane mask.
template <int KG>
__device__ __forceinline__ lmask after_in_group(lmask m) {
    constexpr lmask NOT0 = KG == 4 ? 0xEEEEEEEEEEEEEEEEull : 0xFEFEFEFEFEFEFEFEull;   // not a group's lane 0
    m |= (m << 1) & NOT0;
    m |= (m << 2) & (KG == 4 ? 0xCCCCCCCCCCCCCCCCull : 0xFCFCFCFCFCFCFCFCull);
    if (KG == 8) m |= (m << 4) & 0xF0F0F0F0F0F0F0F0ull;
    return (m << 1) & NOT0;
}

// KG (segmented parts: the group size K): a segment whose group has an earlier segment that ended
// holding the record (a hit or the cube exit, not a STOP) ends too -- the record is that earlier
// segment's whatever it would find (the first segment that did not stop), and its trips, stack and
// state are never read (seg_part: only segments up to the record holder's feed the rebalance and
// the tile cost).  Saves the walk of the segments past a hit that comes before their stored starts
// (a jittered sample, a moving camera: the starts are one frame old).
template <int MODE, bool FETCH_ALL, bool SEGS = true, bool COUNT = false, int KG = 0>
__device__ __forceinline__ void trace_seg(const LaunchParams &p, FRay &r, uint2 *__restrict__ stk, float t_start,
                                          float t_stop, bool armed0, uint32_t &n_lane, uint32_t &armed_at,
                                          bool &stopped_lane) {
    constexpr int STRIDE = TILE;
    const int slots = p.slots;
    for (int s = 0; s < slots; ++s) stk[s * STRIDE] = make_uint2(0u, 0u);
    const int scale_lo = S_MAX - slots;
    lmask act = LM_OF(true);
    lmask armed = LM_OF(armed0), stopped = 0, cached = 0, recs = 0;
    const int oct = r.octant_mask | 16;
    int sh = r.idx ^ oct;
    const uint32_t stk_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint2 *)stk;
    constexpr uint32_t SLOT = (uint32_t)(STRIDE * sizeof(uint2));
    constexpr int SLOT_SH = 23 - 9;
    const uint32_t push_base = stk_base - (uint32_t)(104 + scale_lo) * SLOT;
    const uint2 *stk_pop = stk - (127 + scale_lo) * STRIDE;
    const uint32_t e_max = (uint32_t)(127 + scale_lo + slots - 1);
    int it = 0;
    n_lane = 0;
    armed_at = 0;
    asm volatile("" : "+v"(r.parent), "+v"(r.cd16), "+v"(r.first));
    lmask go;
    do {
        asm volatile("s_add_u32 %0, %0, 1" : "+s"(it) : : "scc");
        const lmask need = FETCH_ALL ? ~(lmask)0 : act & ~cached;
        if (FETCH_ALL || LM_ON(need)) {
            const uint2 nd = *(const uint2 *)((const char *)p.nodes + (uint32_t)(r.parent << 3));
            r.cd16 = nd.x;
            r.first = nd.y;
            if (COUNT) r.fetches += 1u;
        }
        cached |= COUNT ? (need & LM_OF((r.cd16 | r.first) != 0u)) : need;
        const float tx = r.px * r.cx - r.bx;             // N:67-70
        const float ty = r.py * r.cy - r.by;
        const float tz = r.pz * r.cz - r.bz;
        const float tc_max = fminf(fminf(tx, ty), tz);
        const float tv_max = vmin(r.t_max, tc_max);
        const float half = r.sexp * 0.5f;
        const lmask cx = LM_OF(center(half, r.cx, tx) > r.t_min);
        const lmask cy = LM_OF(center(half, r.cy, ty) > r.t_min);
        const lmask cz = LM_OF(center(half, r.cz, tz) > r.t_min);
        const lmask lx = LM_OF(tx <= tc_max), ly = LM_OF(ty <= tc_max), lz = LM_OF(tz <= tc_max);
        const lmask in_span = LM_OF(r.t_min <= tv_max), below_h = LM_OF(tc_max < r.h);
        const lmask before = LM_OF(tc_max < t_start);    // SKIP test (NaN start: never)
        // ARM / STOP tests on the ADVANCE's new t_min.  Without segments (a beam start: finite or -inf,
        // never NaN; tc_max is never NaN, a min of three corner times of which at most two are NaN)
        // arming is the complement of the SKIP test: one compare fewer per trip
        const lmask arm_now = SEGS ? LM_OF(tc_max >= t_start) : ~before;
        const lmask stop_now = SEGS ? LM_OF(tc_max >= t_stop) : (lmask)0;
        const uint32_t cm = r.cd16 << sh;
        const lmask descend = act & LM_OF((int32_t)cm < 0) & in_span;
        const lmask leaf = LM_OF((cm & 0x00800000u) == 0u);
        const lmask inner = descend & ~leaf;
        const lmask skip = inner & before;
        const lmask hit = descend & leaf & armed;        // N:93-94, armed lanes only
        const lmask push = inner & ~skip;
        const lmask store = inner & below_h;             // PUSH's stack write, also for a SKIP
        const lmask adv = act & ~(hit | push);           // incl. SKIP lanes and unarmed leaves
        if (LM_ON(store)) {                              // N:97-98
            const uint32_t a = push_base + (__float_as_uint(r.sexp) >> SLOT_SH);
            const uint32_t tmw = MODE == 0 ? (uint32_t)cvt_i32((float)(int32_t)__float_as_uint(r.t_max))
                                           : __float_as_uint(r.t_max);
            asm volatile("ds_write2_b32 %0, %1, %2 offset1:1" : : "v"(a), "v"(r.parent), "v"(tmw) : "memory");
        }
        const lmask sx = adv & lx;                       // N:122-125
        const lmask sy = adv & ly;
        const lmask sz = adv & lz;
        const float se = r.sexp;
        const float delta = LM_ON(push) ? half : -se;
        const float ox = r.px, oy = r.py, oz = r.pz;
        const lmask mvx = (push & cx) | sx, mvy = (push & cy) | sy, mvz = (push & cz) | sz;
        const float qx = r.px + (LM_ON(mvx) ? delta : 0.0f);
        const float qy = r.py + (LM_ON(mvy) ? delta : 0.0f);
        const float qz = r.pz + (LM_ON(mvz) ? delta : 0.0f);
        const int mv = lanes_to_idx(mvx, mvy, mvz);
        const lmask pop = adv & LM_OF((mv & ~(sh ^ oct)) != 0);
        const uint32_t child = r.first + (uint32_t)__builtin_popcount(cm & 0x007F0000u);
        sh = (LM_ON(push) ? oct : sh) ^ mv;
        if (LM_ON(push)) {
            r.parent = child;
            r.h = tc_max;
            r.t_max = tv_max;
            r.sexp = half;
        }
        if (skip != 0) {   // back at this node's level as after a POP (N:141-153)
            if (LM_ON(skip)) {
                if (MODE == 0) r.t_max = __int_as_float(cvt_i32((float)(int32_t)__float_as_uint(r.t_max)));
                r.h = 0.0f;
            }
        }
        r.t_min = LM_ON(adv) ? tc_max : r.t_min;
        const lmask armed_new = adv & arm_now & ~armed;
        if (armed_new != 0) {
            if (SEGS && LM_ON(armed_new)) armed_at = (uint32_t)it;
            armed |= armed_new;
        }
        const lmask stop = SEGS ? adv & stop_now : (lmask)0;
        cached &= ~(push | pop);
        r.px = qx; r.py = qy; r.pz = qz;
        lmask out = 0;
        if (pop != 0) {                                  // N:134-154
            const uint32_t diff = (__float_as_uint(ox) ^ __float_as_uint(qx)) |
                                  (__float_as_uint(oy) ^ __float_as_uint(qy)) |
                                  (__float_as_uint(oz) ^ __float_as_uint(qz));
            const uint32_t fd = __float_as_uint((float)diff);
            const uint32_t ef = __builtin_amdgcn_ubfe(fd, 23, 8);
            const int scale = (int)ef - 127;
            const uint2 e = stk_pop[min(ef, e_max) * STRIDE];
            const uint32_t keep = 0xFFFFFFFFu << scale;
            const uint32_t bx_ = __builtin_amdgcn_ubfe(__float_as_uint(qx), scale, 1);
            const uint32_t by_ = __builtin_amdgcn_ubfe(__float_as_uint(qy), scale, 1);
            const uint32_t bz_ = __builtin_amdgcn_ubfe(__float_as_uint(qz), scale, 1);
            const bool pl = LM_ON(pop);
            r.sexp = pl ? __uint_as_float((ef << 23) - (23u << 23)) : r.sexp;
            r.parent = pl ? e.x : r.parent;
            r.t_max = pl ? __uint_as_float(e.y) : r.t_max;
            const uint32_t k = pl ? keep : 0xFFFFFFFFu;
            r.px = __uint_as_float(__float_as_uint(r.px) & k);
            r.py = __uint_as_float(__float_as_uint(r.py) & k);
            r.pz = __uint_as_float(__float_as_uint(r.pz) & k);
            r.h = pl ? 0.0f : r.h;
            sh = pl ? (int)(bx_ | (by_ << 1) | (bz_ << 2)) ^ oct : sh;
            out = pop & LM_OF(scale >= S_MAX);
        }
        const lmask fin = act & (hit | out | stop);
        if (fin != 0) {
            if (SEGS && LM_ON(fin)) n_lane = (uint32_t)it;
            stopped |= stop;                             // STOP before the cube exit of the same trip
            act &= ~fin;
            if (KG > 1) {                                // the group's later segments: nothing to find
                recs |= fin & ~stop;
                act &= ~after_in_group<KG>(recs);
            }
        }
        asm volatile("s_cmp_lt_u32 %1, %2\n\ts_cselect_b64 %0, %3, 0" : "=s"(go) : "s"(it), "n"(MAX_ITERS), "s"(act) : "scc");
    } while (go != 0);
    if (LM_ON(act)) {   // still tracing after MAX_ITERS trips (unreachable for a tree of depth <= 13)
        r.flags |= 2u;
        if (SEGS) n_lane = (uint32_t)it;
    }
    stopped_lane = LM_ON(stopped);
    r.idx = sh ^ oct;
    r.trips = it;
}


// ------------------------------------------------------------- beam starts
// The start of a primary ray of pixel (x, gy) (global row) under a launch's beam starts
// (DESIGN.md 3.1d): the min of its tile's, super tile's and the global lower bound, less a margin
// for rounding.  The bound d is exact geometry (the distance from the camera to the nearest box
// that can hold a voxel on the ray); the loop's hit t is a corner time p * coef - bias in f32,
// whose error is at most ~2 ulps of its larger term, 2 ulp(2 |coef| + |bias|) -- a quarter of the
// margin (2 |coef| + |bias|) 2^-20 summed over the axes -- plus the relative error of d (2^-16).  A ray parallel to an axis (|coef| = inf) starts at -inf: everything
// as without a beam.  Returns -inf without beam starts.
__device__ __forceinline__ float beam_start(const LaunchParams &p, const FRay &f, int x, int gy) {
    if (!p.tile_start) return -__builtin_inff();
    // an entry of this launch's generation holds its distance, any other is +inf (beam_splat_kernel)
    const unsigned long long k = min(min(p.tile_start[(gy >> 3) * p.ts_tiles_x + (x >> 3)],
                                         p.tile_start[p.ts_super_off + (gy >> 6) * p.ts_super_x + (x >> 6)]),
                                     p.tile_start[p.ts_global_off]);
    const float d = (uint32_t)(k >> 32) == ~p.ts_gen ? __uint_as_float((uint32_t)k) : __builtin_inff();
    const float m = (2.0f * (fabsf(f.cx) + fabsf(f.cy) + fabsf(f.cz)) + fabsf(f.bx) + fabsf(f.by) + fabsf(f.bz)) *
                    0x1p-20f;
    const float s = d * (1.0f - 0x1p-16f) - m;
    return s == s ? s : -__builtin_inff();
}

// The lean loop from a beam start (trace_seg, one segment, no stop): a lane whose cube entry lies
// at or past the start is armed from the first trip and runs the continuous loop.
template <int MODE, bool FA, bool COUNT = false>
__device__ __forceinline__ void trace_beam(const LaunchParams &p, FRay &f, uint2 *__restrict__ stk, float start) {
    uint32_t n_lane, armed_at;
    bool stopped;
    trace_seg<MODE, FA, false, COUNT>(p, f, stk, start, __builtin_inff(), f.t_min >= start, n_lane, armed_at, stopped);
}

// ------------------------------------------------------------- tile kernel
// Interleaved XCD column strips (xcd_remap 2).  Workgroups b with b % 8 == x
// land on XCD x (MI355X_MICROARCH.md "Workgroup dispatch"); tile column c
// belongs to XCD c % 8, so XCD x's private 4 MB L2 only caches the nodes seen
// through its own columns while every XCD samples the whole screen (sky and
// terrain alike).  Needs the tile columns to be a multiple of 8 (the host
// checks).  e = position within the XCD's share, column-major.
// strips STRIP_K tile columns wide: XCD x owns columns c with (c / K) % 8 == x
__device__ __forceinline__ int strip_col(int x, int m) {
    constexpr int K = STRIP_K;
    return K == 1 ? m * 8 + x : (m / K) * (8 * K) + x * K + (m % K);
}
__device__ __forceinline__ int strip_tile(int x, int e, int tiles_x, int tiles_y) {
    const int m = e / tiles_y, row = e - m * tiles_y;
    return row * tiles_x + strip_col(x, m);
}

// FA: the lean loop's unpredicated node loads (p.fetch_all) -- a separate
// instantiation, so each form keeps its own register allocation (both loops in
// one kernel took 82 SGPRs: 7 waves/SIMD, MI355X_MICROARCH.md occupancy table)
// SH: the shadow pass fused into the same wave -- after its primary rays the wave
// traces one shadow ray per hit lane, and the tile's recorded cost is the sum of
// both, so one cost-ordered launch balances the whole frame.
// COUNT: the instrumented launch (per-ray descriptor fetch counts, no outputs).
// LAT: the latency form of the loop (trace_lat) for launches that leave wave slots empty;
// twice the LDS (the stack entries keep their node).
template <int MODE, bool COUNT, bool FA = false, bool SH = false, bool LAT = false>
// SGPR budget: at .sgpr_count 80 (what the compiler chose unbounded) the hardware admitted only 7
// of these one-wave workgroups per SIMD (wave ids 0-6, 28 per CU in the per-wave HW_ID log,
// profiles/r03t_*), though the compiler's and the API's occupancy said 8; capped at 72 it needs 70,
// spills nothing, and 8 waves per SIMD are resident (C3 frame -2 %, profiles/r03t_ab_sgpr_cap.txt).
#ifndef SVO_NUM_SGPR
#define SVO_NUM_SGPR 72
#endif
__global__ __launch_bounds__(TILE) __attribute__((amdgpu_num_sgpr(SVO_NUM_SGPR))) void render_tile_kernel(LaunchParams p, int tiles_x) {
    extern __shared__ uint2 stk_base[];   // [p.slots][64] (LAT: twice, the nodes behind)
    const int lane = threadIdx.x;
    const uint32_t t_entry = !COUNT && p.wave_log ? (uint32_t)__builtin_amdgcn_s_memrealtime() : 0u;
    const int n_tiles = (int)gridDim.x;
    const int t = p.tile_order ? (int)p.tile_order[blockIdx.x]
                : p.xcd_remap == 2 ? strip_tile((int)blockIdx.x % 8, (int)blockIdx.x / 8, tiles_x, n_tiles / tiles_x)
                                   : (int)blockIdx.x;
    const int bx = t % tiles_x, by = t / tiles_x;
    const int x = bx * 8 + (lane & 7);
    const int lr = by * 8 + (lane >> 3);
    if (x >= p.width || lr >= p.local_rows) return;
    if (p.tile_order && p.prio) {
        // issue priority by the previous launch's cost class: the heaviest tiles
        // bound the launch, so their waves win issue arbitration on a busy SIMD
        const uint32_t n = gridDim.x;
        const bool strips = p.xcd_remap == 2;
        const uint32_t b = strips ? blockIdx.x / 8 : blockIdx.x;
        const uint32_t *bound = strips ? p.tile_order + n + 4 + 4 * (blockIdx.x % 8) : p.tile_order + n;
        if (b < bound[0]) __builtin_amdgcn_s_setprio(3);
        else if (b < bound[1]) __builtin_amdgcn_s_setprio(2);
        else if (b < bound[2]) __builtin_amdgcn_s_setprio(1);
    }
    const int gy = global_row(p, lr);
    Ray r;
    {
        float org[3], dir[3];
        camera_ray(p.cam, p.width, p.height, x, gy, org, dir);
        setup_ray(org, dir, r);
    }
    uint2 *stk = stk_base + lane;
    uint32_t t0 = 0;
    if (!COUNT && p.wave_log) t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    FRay f;
    to_fray(r, f);
    LeanDiag dg;
    if (COUNT) {
        if (p.tile_start) trace_beam<MODE, false, true>(p, f, stk, beam_start(p, f, x, gy));   // SVO_OPT_COUNT_BEAM
        else trace_lean<MODE, true, false, false, true>(p, f, stk);
    }
    else if (LAT) trace_lat<MODE>(p, f, stk);
    else if (!SH && p.wave_log) {
        if (p.guard) trace_lean<MODE, true, true>(p, f, stk, &dg);
        else trace_lean<MODE, false, true>(p, f, stk, &dg);
    }
    else if (p.guard) trace_lean<MODE, true>(p, f, stk);
    else if (p.tile_start) trace_beam<MODE, FA>(p, f, stk, beam_start(p, f, x, gy));
    else trace_lean<MODE, false, false, FA>(p, f, stk);
    from_fray(f, r);
    if (COUNT) {
        p.out.fetches[(size_t)lr * (size_t)p.width + (size_t)x] = r.fetches;
        return;
    }
    const float4 acc = accum_load(p, out_index(p, lr, gy, x));
    Record o;
    record(p, r, x, gy, o);
    int trips = f.trips;
    if (SH) {
        const bool hit = r.scale < S_MAX;
        const uint64_t hits = __ballot(hit);
        if (hits) {
            if (hit) {   // exec = the hit lanes: the lean loop's lanes are exactly these
                float so[3], sd[3];
                shadow_ray(p, x, gy, o.w[2], o.w[3], o.w[4], o.w[5], so, sd);
                Ray rs;
                setup_ray(so, sd, rs);
                FRay fs;
                to_fray(rs, fs);
                if (p.guard) trace_lean<MODE, true>(p, fs, stk);
                else trace_lean<MODE, false, false, FA>(p, fs, stk);
                from_fray(fs, rs);
                if (rs.scale < S_MAX) {   // occluded: flag bit 3, black Result (R:109-111)
                    o.w[1] |= 8u << 16;
                    o.rgb[0] = o.rgb[1] = o.rgb[2] = 0.0f;
                }
                trips += fs.trips;
            }
            trips = __shfl(trips, __ffsll((long long)hits) - 1);   // primary + shadow trips of the wave
        }
    }
    if (p.out.hitmask) {   // the tile's hit lanes, for the sparse band payload
        const uint64_t hm = __ballot(r.scale < S_MAX);
        if (lane == 0) p.out.hitmask[t] = hm;
    }
    if (p.tile_cost && (!SH || lane == 0)) p.tile_cost[t] = (uint16_t)min(trips, 65535);
    if (p.wave_log && lane == 0) {   // 100 MHz constant clock, tile, XCC_ID
        uint32_t *w = p.wave_log + WAVE_LOG_WORDS * (size_t)blockIdx.x;
        w[8] = t_entry;
        w[10] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID: wave, SIMD, CU, SH, SE
        w[0] = t0;
        w[1] = (uint32_t)__builtin_amdgcn_s_memrealtime();
        w[2] = (uint32_t)t;   // the tile (band-local, row-major)
        w[3] = ((uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xFFu) | ((uint32_t)f.trips << 8);
        w[4] = (uint32_t)dg.loop_cycles;
        w[5] = (uint32_t)dg.fetch_cycles;
        w[6] = dg.fetch_trips;
        w[7] = dg.pop_trips;
    }
    store_outputs(p.out, out_index(p, lr, gy, x), o, acc);
    if (p.wave_log && lane == 0) p.wave_log[WAVE_LOG_WORDS * (size_t)blockIdx.x + 9] = (uint32_t)__builtin_amdgcn_s_memrealtime();
}

// a ray's K segments are K consecutive lanes (K = 4 or 8, wave-uniform)
__device__ __forceinline__ int group_min(int v, int K) {
    v = min(v, __shfl_xor(v, 1));
    v = min(v, __shfl_xor(v, 2));
    if (K == 8) v = min(v, __shfl_xor(v, 4));
    return v;
}
__device__ __forceinline__ float group_get(float v, int K, int j) {
    return __shfl(v, (int)(threadIdx.x & ~(uint32_t)(K - 1)) + j);
}
__device__ __forceinline__ uint32_t group_get(uint32_t v, int K, int j) {
    return (uint32_t)__shfl((int)v, (int)(threadIdx.x & ~(uint32_t)(K - 1)) + j);
}

// The next frame's starts of one ray from this frame's K segments: the continuous trips each
// segment took after arming (segment 0: all of its trips) put the cumulative share at its start
// t_k; the new start at fraction e / 8 (e = 1..7, whatever K the next trace uses) is where the
// cumulative share reaches e / 8 of the total, linear in t between the points (t_entry, 0),
// (t_k, share before k), (t_end, total).  Only the balance of the next trace depends on it.
// `slot`: this wave's dead stack (LDS, one uint2 per lane): each lane parks (its share, its
// start) there, and lane 0 of the group walks the K entries in order -- no per-lane arrays, so
// the kernel keeps the lean loop's register budget.  Returns false if the ray gave no information.
__device__ __forceinline__ void seg_rebalance(uint2 *slot, float t_entry, float t_start, float t_end, uint32_t c,
                                              int f, int K, float tot, float *hint8, bool store) {
    const int lane = (int)threadIdx.x, k = lane & (K - 1);
    // a start past the ray's end carries nothing: it sits at the end
    slot[lane] = make_uint2(k <= f ? c : 0u, __float_as_uint(k == 0 ? t_entry : k > f ? t_end : t_start));
    // lane 0 of each group reads its group's other lanes' entries below: the writes must have landed
    // (the workgroup is this one wave; the compiler cannot see the cross-lane dependence)
    __syncthreads();
    if (k != 0 || !store) return;
    if (!(tot > 0.0f)) {   // no information: the next trace splits the cube span evenly
        hint8[0] = __int_as_float(0x7FC00000);
        return;
    }
    const uint2 *g = slot + lane;   // the group's K entries
    int m = 0;
    float cum = 0.0f, cm = (float)g[0].x, t0 = t_entry, prev = 0.0f;
    float t1 = K > 1 ? __uint_as_float(g[1].y) : t_end;
    for (int e = 1; e < SEG_KMAX; ++e) {
        const float target = tot * ((float)e / (float)SEG_KMAX);
        while (m < K - 1 && cum + cm < target) {   // the segment holding the target
            cum += cm;
            ++m;
            cm = (float)g[m].x;
            t0 = t1;
            t1 = m + 1 < K ? __uint_as_float(g[m + 1].y) : t_end;
        }
        const float fr = cm > 0.0f ? fminf(fmaxf((target - cum) / cm, 0.0f), 1.0f) : 0.0f;
        const float v = t0 + fr * (t1 - t0);
        prev = e > 1 ? fmaxf(v, prev) : v;
        hint8[e - 1] = prev;
    }
}

// Start of the segment at fraction e / 8 of the ray's trace (e = 0 or 8: none, NaN): the
// pixel's stored starts, an even split of the cube span before it has any, or (tests,
// p.seg_scramble) a hash -- unordered, NaN, +-inf or outside the cube.
__device__ __forceinline__ float seg_start(const LaunchParams &p, const float *hint8, bool have, size_t hi, int e,
                                           float t_entry, float t_exit) {
    if (e <= 0 || e >= SEG_KMAX) return __int_as_float(0x7FC00000);
    const float span = t_exit - t_entry;
    if (p.seg_scramble) {
        uint32_t hsh = (uint32_t)hi * 0x9E3779B1u ^ p.seg_scramble * 0x85EBCA77u ^ (uint32_t)e * 0x27D4EB2Fu;
        hsh ^= hsh >> 15; hsh *= 0x2C1B3C6Du; hsh ^= hsh >> 12; hsh *= 0x297A2D39u; hsh ^= hsh >> 15;
        const uint32_t sel = hsh & 15u;
        const float u = (float)(hsh >> 8) * (1.0f / 16777216.0f);
        return sel == 0 ? __int_as_float(0x7FC00000) : sel == 1 ? __int_as_float(0x7F800000)
             : sel == 2 ? __int_as_float(0xFF800000) : t_entry + (1.4f * u - 0.2f) * span;
    }
    return have ? hint8[e - 1] : t_entry + ((float)e / (float)SEG_KMAX) * span;
}

// Cost-ordered launch whose order (launch_order_strips with seg_cap > 0) lists each XCD's
// heaviest tiles as K part entries (K = 4 or 8 by cost class): part q traces 64 / K rays of its
// tile -- rows q * 8 / K onward -- as K segments each (lanes K r .. K r + K - 1 = ray r), and
// writes every output of those pixels from the lane of the segment that holds the record.  Every
// other entry is one tile, traced as in render_tile_kernel (lean loop, primary rays).  A part's
// chain is its longest segment: ~1/K of the tile's continuous chain plus the walk to t_k.  LAT:
// whole tiles take the latency form (trace_lat, twice the LDS).
// Part `part` of a tile traced as K segments per ray (render_seg_kernel; K a template constant so
// the part's wave-uniform values need no SGPRs across the traversal loop).
// Diagnostics (SVO_WAVE_LOG, p.wave_log != null): per workgroup of render_seg_kernel, at blockIdx.x:
// [0] trace start, [1] trace end, [8] entry (s_memrealtime, 100 MHz), [2] the order entry,
// [3] XCC_ID | the wave's trips << 8, [9] lane 0's end (after the rebalance, before a part's record
// stores; after its stores for a whole tile) (the band-floor decomposition, tools/band_floor.py).
// The stamps are a template flag (LOG, launched only when p.wave_log is set): compiled into the
// product kernel behind a runtime test they cost C4's launch 4-5 % (profiles/r06_seg_log_ab.json).
__device__ __forceinline__ void seg_log(const LaunchParams &p, int slot, uint32_t v) {
    if (threadIdx.x == 0) p.wave_log[WAVE_LOG_WORDS * (size_t)blockIdx.x + slot] = v;
}
__device__ __forceinline__ uint32_t now_100mhz() { return (uint32_t)__builtin_amdgcn_s_memrealtime(); }

template <int MODE, bool FA, int K, bool LOG>
__device__ __forceinline__ void seg_part(const LaunchParams &p, uint2 *__restrict__ stk_base, int t, int part, int bx,
                                         int by) {
    const int lane = threadIdx.x;
    uint2 *stk = stk_base + lane;
    constexpr int R = TILE / K;                // rays of this part: rows part * R / 8 .. of the tile
    const int k = lane & (K - 1), ri = lane / K;
    const int x_ = bx * 8 + (ri & 7);
    const int lr_ = by * 8 + part * (R / 8) + (ri >> 3);
    const bool inside = x_ < p.width && lr_ < p.local_rows;   // outside lanes trace a copy, store nothing
    const int x = min(x_, p.width - 1), lr = min(lr_, p.local_rows - 1);
    const int gy = global_row(p, lr);
    Ray r;
    {
        float org[3], dir[3];
        camera_ray(p.cam, p.width, p.height, x, gy, org, dir);
        setup_ray(org, dir, r);
    }
    FRay f;
    to_fray(r, f);
    // segment 0 starts at the beam start (-inf without one); the even split and the rebalance
    // then spread the segments over the part of the ray after it
    const float bs = beam_start(p, f, x, gy);
    const float t_entry = fmaxf(r.t_min, bs), t_exit = r.t_max;
    // the pixel's starts at fractions e / 8 of its trace (8 floats: e = 1..7 + spare); segment k of
    // K runs from fraction k / K to (k + 1) / K
    const size_t hi = (size_t)lr * (size_t)p.width + (size_t)x;
    float *hint8 = p.seg_hint ? reinterpret_cast<float *>(p.seg_hint + 2 * hi) : nullptr;   // null: even splits
    const int e0 = k * (SEG_KMAX / K), e1 = e0 + SEG_KMAX / K;   // 0 and 8: none
    // NaN: none yet.  A lane outside the frame (a copy of an edge pixel, which may belong to another
    // part of this tile traced by another workgroup) takes the even split: it reads no hint
    const bool have = inside && hint8 && hint8[0] == hint8[0];
    const float t_start = seg_start(p, hint8, have, hi, e0, t_entry, t_exit);
    const float t_stop = seg_start(p, hint8, have, hi, e1, t_entry, t_exit);
    uint32_t n_lane, armed_at;
    bool stopped;
    if (LOG) seg_log(p, 0, now_100mhz());
    trace_seg<MODE, FA, true, false, K>(p, f, stk, k == 0 ? bs : t_start, t_stop, k == 0 && r.t_min >= bs, n_lane, armed_at,
                        stopped);
    if (LOG) {
        seg_log(p, 1, now_100mhz());
        seg_log(p, 3, ((uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xFFu) | ((uint32_t)f.trips << 8));
    }
    from_fray(f, r);
    // the record holder: the first segment that did not stop (the last one never stops)
    const int fsel = group_min(stopped ? K : k, K);
    const bool writer = k == fsel;
    const uint32_t c = k == 0 ? n_lane : n_lane - armed_at;   // continuous trips after arming
    const float t_end = group_get(r.scale < S_MAX ? r.t_min : t_exit, K, fsel);
    uint32_t tot = k <= fsel ? c : 0u;   // the ray's continuous trips, its tile_cost share
    tot += (uint32_t)__shfl_xor((int)tot, 1);
    tot += (uint32_t)__shfl_xor((int)tot, 2);
    if (K == 8) tot += (uint32_t)__shfl_xor((int)tot, 4);
    seg_rebalance(stk_base, t_entry, t_start, t_end, c, fsel, K, (float)tot, hint8, inside && hint8);
    if (p.tile_cost) {
        uint32_t m = inside ? tot : 0u;
        for (int d = K; d < TILE; d <<= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d));
        if (lane == 0) {
            p.part_cost[SEG_KMAX * (size_t)t + part] = (uint16_t)min(m, (uint32_t)(SEG_COST_FLAG - 1));
            if (part == 0) p.tile_cost[t] = (uint16_t)(SEG_COST_FLAG | K);
        }
    }
    if (p.out.hitmask) {   // this part's R pixels: bits part * R .. part * R + R - 1 of the tile's mask
        // OR of the ray's group: the writer lane's hit, gathered into lane K r, then one ballot
        uint32_t hit_w = (writer && inside && r.scale < S_MAX) ? 1u : 0u;
        hit_w |= (uint32_t)__shfl_xor((int)hit_w, 1);
        hit_w |= (uint32_t)__shfl_xor((int)hit_w, 2);
        if (K == 8) hit_w |= (uint32_t)__shfl_xor((int)hit_w, 4);
        const uint64_t hm = __ballot(k == 0 && hit_w != 0);   // bit K r = ray r
        uint32_t bits = 0;
#pragma unroll
        for (int j = 0; j < R; ++j) bits |= (uint32_t)((hm >> (K * j)) & 1ull) << j;
        if (lane == 0) {
            if (K == 4) reinterpret_cast<uint16_t *>(p.out.hitmask)[4 * (size_t)t + part] = (uint16_t)bits;
            else reinterpret_cast<uint8_t *>(p.out.hitmask)[8 * (size_t)t + part] = (uint8_t)bits;
        }
    }
    if (LOG) seg_log(p, 9, now_100mhz());
    if (!writer || !inside) return;
    const float4 acc = accum_load(p, out_index(p, lr, gy, x));
    Record o;
    record(p, r, x, gy, o);
    store_outputs(p.out, out_index(p, lr, gy, x), o, acc);
}

template <int MODE, bool FA, bool LAT, bool LOG>
// VGPR budget: unbounded, the compiler gave this kernel 68-70 VGPRs -- 7 waves per SIMD (a wave needs
// <= 64 for 8, MI355X_MICROARCH.md occupancy table).  Asking for 8 waves per EU fits it in 64 VGPRs at
// the cost of one spilled dword, stored and reloaded outside the traversal loop (tools/kernel_resources.py).
#ifndef SVO_SEG_WAVES_PER_EU
#define SVO_SEG_WAVES_PER_EU 8
#endif
__global__ __launch_bounds__(TILE) __attribute__((amdgpu_num_sgpr(SVO_NUM_SGPR), amdgpu_waves_per_eu(SVO_SEG_WAVES_PER_EU, 8)))
void render_seg_kernel(LaunchParams p, int tiles_x) {
    extern __shared__ uint2 stk_base[];
    const int lane = threadIdx.x;
    const uint32_t t_in = LOG ? now_100mhz() : 0u;
    const uint32_t entry = p.tile_order[blockIdx.x];
    if (LOG) {
        seg_log(p, 8, t_in);
        seg_log(p, 2, entry);
    }
    if (entry == SEG_EMPTY) return;
    const int t = (int)(entry & 0x0FFFFFFFu);
    const int code = (int)(entry >> 28);   // 0: a whole tile; 1..4: part of a K = 4 tile; 5..12: K = 8
    if (p.prio) {
        const uint32_t *bound = p.tile_order + gridDim.x + 4 + 4 * (blockIdx.x % 8);
        const uint32_t b = blockIdx.x / 8;
        if (b < bound[0]) __builtin_amdgcn_s_setprio(3);
        else if (b < bound[1]) __builtin_amdgcn_s_setprio(2);
        else if (b < bound[2]) __builtin_amdgcn_s_setprio(1);
    }
    const int bx = t % tiles_x, by = t / tiles_x;
    uint2 *stk = stk_base + lane;
    if (code == 0) {   // render_tile_kernel's primary-ray path
        const int x = bx * 8 + (lane & 7);
        const int lr = by * 8 + (lane >> 3);
        if (x >= p.width || lr >= p.local_rows) return;
        const int gy = global_row(p, lr);
        Ray r;
        {
            float org[3], dir[3];
            camera_ray(p.cam, p.width, p.height, x, gy, org, dir);
            setup_ray(org, dir, r);
        }
        FRay f;
        to_fray(r, f);
        if (LOG) seg_log(p, 0, now_100mhz());
        if (LAT) trace_lat<MODE>(p, f, stk);
        else if (p.tile_start) trace_beam<MODE, FA>(p, f, stk, beam_start(p, f, x, gy));
        else trace_lean<MODE, false, false, FA>(p, f, stk);
        if (LOG) {
            seg_log(p, 1, now_100mhz());
            seg_log(p, 3, ((uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xFFu) | ((uint32_t)f.trips << 8));
        }
        from_fray(f, r);
        const float4 acc = accum_load(p, out_index(p, lr, gy, x));
        Record o;
        record(p, r, x, gy, o);
        if (p.out.hitmask) {
            const uint64_t hm = __ballot(r.scale < S_MAX);
            if (lane == 0) p.out.hitmask[t] = hm;
        }
        if (p.tile_cost) p.tile_cost[t] = (uint16_t)min(f.trips, (int)(SEG_COST_FLAG - 1));
        store_outputs(p.out, out_index(p, lr, gy, x), o, acc);
        if (LOG) seg_log(p, 9, now_100mhz());
        return;
    }
    if (code <= 4) seg_part<MODE, FA, 4, LOG>(p, stk_base, t, code - 1, bx, by);
    else seg_part<MODE, FA, 8, LOG>(p, stk_base, t, code - 5, bx, by);
}

// ------------------------------------------------------------- samples in flight
// svo_render_samples: the reference's frame loop is a stream of independent jittered samples,
// each blended into the display target (_PixelOffset = (Random.value, Random.value) per frame,
// RaytracingMaster.cs:35; _Sample blend and _currentSample++, :70-73, AddShader.shader:44-47).
// One launch traces S of them: workgroup = 8x8 tile (cost-ordered like render_tile_kernel),
// wave k = sample k.  A launch then holds S times the waves behind each heavy tile, so the
// heaviest wave -- which bounds a one-sample launch of a small band -- is
// overlapped by the other samples' work instead of draining alone.  After tracing, each wave
// parks its colour in its own (dead) stack region, and wave 0 blends the S colours into the
// accumulation in sample order with accumulate_kernel's arithmetic (bit-identical to S
// consecutive svo_accumulate calls), then stores the display words.
template <int MODE, bool FA>
__global__ __launch_bounds__(TILE * MAX_SAMPLES) __attribute__((amdgpu_num_sgpr(SVO_NUM_SGPR)))
void render_samples_kernel(LaunchParams p, int tiles_x) {
    extern __shared__ uint2 stk_base[];   // [sample][p.slots][64]
    const int lane = threadIdx.x & (TILE - 1);
    const int k = threadIdx.x / TILE;     // this wave's sample
    const int n_tiles = (int)gridDim.x;
    const int t = p.tile_order ? (int)p.tile_order[blockIdx.x]
                : p.xcd_remap == 2 ? strip_tile((int)blockIdx.x % 8, (int)blockIdx.x / 8, tiles_x, n_tiles / tiles_x)
                                   : (int)blockIdx.x;
    const int bx = t % tiles_x, by = t / tiles_x;
    // a lane out of the frame traces a copy of an inside pixel and stores nothing: every lane of
    // every wave reaches the barrier below (no reliance on partially exited waves)
    const bool inside = bx * 8 + (lane & 7) < p.width && by * 8 + (lane >> 3) < p.local_rows;
    const int x = min(bx * 8 + (lane & 7), p.width - 1);
    const int lr = min(by * 8 + (lane >> 3), p.local_rows - 1);
    if (p.tile_order && p.prio) {
        const uint32_t n = gridDim.x;
        const bool strips = p.xcd_remap == 2;
        const uint32_t b = strips ? blockIdx.x / 8 : blockIdx.x;
        const uint32_t *bound = strips ? p.tile_order + n + 4 + 4 * (blockIdx.x % 8) : p.tile_order + n;
        if (b < bound[0]) __builtin_amdgcn_s_setprio(3);
        else if (b < bound[1]) __builtin_amdgcn_s_setprio(2);
        else if (b < bound[2]) __builtin_amdgcn_s_setprio(1);
    }
    const int gy = global_row(p, lr);
    Ray r;
    {
        Camera cam = p.cam;
        cam.px_off[0] = p.sample_off[k][0];
        cam.px_off[1] = p.sample_off[k][1];
        float org[3], dir[3];
        camera_ray(cam, p.width, p.height, x, gy, org, dir);
        setup_ray(org, dir, r);
    }
    const size_t region = (size_t)max(p.slots, 2) * TILE;   // >= 64 float4: the colours below
    uint2 *stk = stk_base + (size_t)k * region + lane;
    // wave 0 loads its pixels' accumulation before tracing, so the load's latency is hidden by
    // the trace instead of holding the wave's slot at its end
    float4 dprev = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (k == 0 && inside) dprev = p.accum[out_index(p, lr, gy, x)];
    FRay f;
    to_fray(r, f);
    if (p.guard) trace_lean<MODE, true>(p, f, stk);
    else if (p.tile_start) trace_beam<MODE, FA>(p, f, stk, beam_start(p, f, x, gy));
    else trace_lean<MODE, false, false, FA>(p, f, stk);
    from_fray(f, r);
    Record o;
    record(p, r, x, gy, o);   // p.out.rgba is set (the accumulation), so the hit is shaded
    if (k == 0 && lane == 0 && p.tile_cost) p.tile_cost[t] = (uint16_t)min(f.trips, 65535);
    // the colour into this wave's own stack region (dead now; 16 B per lane <= the stack's share)
    float4 *col = reinterpret_cast<float4 *>(stk_base + (size_t)k * region);
    col[lane] = make_float4(o.rgb[0], o.rgb[1], o.rgb[2], 1.0f);
    __syncthreads();
    if (k != 0 || !inside) return;
    const size_t i = out_index(p, lr, gy, x);
    float4 d = dprev;
    for (int j = 0; j < p.samples; ++j) {   // accumulate_kernel's blend, sample j after sample j - 1
        const float4 c = reinterpret_cast<const float4 *>(stk_base + (size_t)j * region)[lane];
        const float a = p.blend_a[j], b = p.blend_b[j];
        d.x = c.x * a + d.x * b;
        d.y = c.y * a + d.y * b;
        d.z = c.z * a + d.z * b;
        d.w = a * a + d.w * b;
    }
    // the write streams out (33 MB at 1080p): non-temporal, so it does not evict the node pool from
    // L2 (store_outputs); the read above keeps the default policy (prefetched, non-temporal +2-8 %)
    __builtin_nontemporal_store(f32x4{d.x, d.y, d.z, d.w}, reinterpret_cast<f32x4 *>(p.accum + i));
    if (p.accum8 || p.accum_rgb8) {
        const uint32_t w = pack_rgba8(d.x, d.y, d.z);
        if (p.accum8) __builtin_nontemporal_store(w, p.accum8 + i);
        if (p.accum_rgb8) {
            uint8_t *c = p.accum_rgb8 + 3 * i;
            c[0] = (uint8_t)w;
            c[1] = (uint8_t)(w >> 8);
            c[2] = (uint8_t)(w >> 16);
        }
    }
}

// ------------------------------------------------------------- shadow pass
// Two-pass form (svo_config.shadow_form 1): one shadow ray per primary hit, read
// back from the primary pass's records (svo_hit or compact); an occluded pixel
// gets flag bit 3 and a black Result (R:109-111) in every output.  Same 8x8
// tiles as the primary pass, cost-ordered by its own recorded trip counts.
template <int MODE, bool FA = false>
__global__ __launch_bounds__(TILE) void shadow_tile_kernel(LaunchParams p, int tiles_x) {
    extern __shared__ uint2 stk_base[];
    const int lane = threadIdx.x;
    const int t = p.shadow_order ? (int)p.shadow_order[blockIdx.x]
                : p.xcd_remap == 2 ? strip_tile((int)blockIdx.x % 8, (int)blockIdx.x / 8, tiles_x, (int)gridDim.x / tiles_x)
                                   : (int)blockIdx.x;
    if (p.shadow_order && p.prio) {
        const bool strips = p.xcd_remap == 2;
        const uint32_t *bound = strips ? p.shadow_order + gridDim.x + 4 + 4 * (blockIdx.x % 8) : p.shadow_order + gridDim.x;
        const uint32_t b = strips ? blockIdx.x / 8 : blockIdx.x;
        if (b < bound[0]) __builtin_amdgcn_s_setprio(3);
        else if (b < bound[1]) __builtin_amdgcn_s_setprio(2);
        else if (b < bound[2]) __builtin_amdgcn_s_setprio(1);
    }
    const int x = (t % tiles_x) * 8 + (lane & 7);
    const int lr = (t / tiles_x) * 8 + (lane >> 3);
    const bool inside = x < p.width && lr < p.local_rows;
    const int gy = inside ? global_row(p, lr) : 0;
    const size_t i = out_index(p, lr, gy, x);
    uint32_t w1 = 0, w2 = 0;
    float n[3] = {0.0f, 0.0f, 0.0f};
    if (inside) {
        if (p.out.hits) {
            const uint2 *rec = reinterpret_cast<const uint2 *>(p.out.hits + i);
            const uint2 a = rec[0], b = rec[1], c = rec[2];
            w1 = a.y; w2 = b.x;
            n[0] = __uint_as_float(b.y); n[1] = __uint_as_float(c.x); n[2] = __uint_as_float(c.y);
        } else {
            const uint3 c = reinterpret_cast<const uint3 *>(p.out.compact)[i];
            w1 = c.y; w2 = c.z;
            if ((w1 >> 16) & 1u) {
                const uint2 a = p.att[c.x];
                decode_normal(a.y >> 16, n);
                normalize3(n);
            }
        }
    }
    const bool hit = (w1 >> 16) & 1u;
    const bool any_hit = __ballot(hit) != 0;   // whole wave, before any lane leaves
    if (p.shadow_cost && lane == 0 && !any_hit) p.shadow_cost[t] = 0;
    if (!hit) return;
    float so[3], sd[3];
    shadow_ray(p, x, gy, w2, __float_as_uint(n[0]), __float_as_uint(n[1]), __float_as_uint(n[2]), so, sd);
    Ray r;
    setup_ray(so, sd, r);
    uint2 *stk = stk_base + lane;
    FRay f;   // the primary rays' lean loop (one wave of shadow rays per tile, parallel directions)
    to_fray(r, f);
    if (p.guard) trace_lean<MODE, true>(p, f, stk);
    else trace_lean<MODE, false, false, FA>(p, f, stk);
    from_fray(f, r);
    if (p.shadow_cost) p.shadow_cost[t] = (uint16_t)min(f.trips, 65535);   // same value from every tracing lane
    if (r.scale < S_MAX) {   // occluded
        const uint32_t nw1 = w1 | (8u << 16);
        if (p.out.hits) reinterpret_cast<uint32_t *>(p.out.hits + i)[1] = nw1;
        if (p.out.compact) p.out.compact[3 * i + 1] = nw1;
        if (p.out.rgba) p.out.rgba[i] = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
        if (p.out.rgba8) p.out.rgba8[i] = 255u << 24;
        if (p.out.rgb8) {
            uint8_t *d = p.out.rgb8 + 3 * i;
            d[0] = d[1] = d[2] = 0;
        }
    }
}

// Compacted form (svo_config.shadow_form 2): the primary pass's
// hit masks are scanned and its hit pixels packed into a dense list in tile order
// (pack_hits_kernel<INDEX>, the sparse payload's ballot + prefix sum), and one wave
// traces 64 consecutive list entries.  The grid covers every pixel; waves past the
// device-side hit count return at once.
template <int MODE, bool FA = false>
__global__ __launch_bounds__(TILE) void shadow_list_kernel(LaunchParams p, const uint32_t *__restrict__ list,
                                                           const uint32_t *__restrict__ count) {
    extern __shared__ uint2 stk_base[];
    const int lane = (int)threadIdx.x;
    const uint32_t k = blockIdx.x * TILE + (uint32_t)lane;
    const uint32_t n = *count;
    if (blockIdx.x * TILE >= n || k >= n) return;
    const uint32_t px = list[k];
    const int x = (int)(px % (uint32_t)p.width), lr = (int)(px / (uint32_t)p.width);
    const int gy = global_row(p, lr);
    const size_t i = out_index(p, lr, gy, x);
    uint32_t w1, w2;
    float nrm[3];
    if (p.out.hits) {
        const uint2 *rec = reinterpret_cast<const uint2 *>(p.out.hits + i);
        const uint2 a = rec[0], b = rec[1], c = rec[2];
        w1 = a.y; w2 = b.x;
        nrm[0] = __uint_as_float(b.y); nrm[1] = __uint_as_float(c.x); nrm[2] = __uint_as_float(c.y);
    } else {
        const uint3 c = reinterpret_cast<const uint3 *>(p.out.compact)[i];
        w1 = c.y; w2 = c.z;
        const uint2 a = p.att[c.x];
        decode_normal(a.y >> 16, nrm);
        normalize3(nrm);
    }
    float so[3], sd[3];
    shadow_ray(p, x, gy, w2, __float_as_uint(nrm[0]), __float_as_uint(nrm[1]), __float_as_uint(nrm[2]), so, sd);
    Ray r;
    setup_ray(so, sd, r);
    uint2 *stk = stk_base + lane;
    FRay f;
    to_fray(r, f);
    if (p.guard) trace_lean<MODE, true>(p, f, stk);
    else trace_lean<MODE, false, false, FA>(p, f, stk);
    from_fray(f, r);
    if (r.scale < S_MAX) {   // occluded
        const uint32_t nw1 = w1 | (8u << 16);
        if (p.out.hits) reinterpret_cast<uint32_t *>(p.out.hits + i)[1] = nw1;
        if (p.out.compact) p.out.compact[3 * i + 1] = nw1;
        if (p.out.rgba) p.out.rgba[i] = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
        if (p.out.rgba8) p.out.rgba8[i] = 255u << 24;
        if (p.out.rgb8) {
            uint8_t *d = p.out.rgb8 + 3 * i;
            d[0] = d[1] = d[2] = 0;
        }
    }
}

// ---------------------------------------------------------- frame assembly
// svo_assemble_frame: one thread per pixel of the frame (one row per grid y).
// Row y belongs to band b = y / band_rows and, round-robin, to part m = b % n_parts
// at local row (b / n_parts) * band_rows + y % band_rows (part_of_row: also the
// weighted deal).  Parts are read where
// they lie: a peer device's memory over xGMI (peer access), or this device's.
// Part and part-local row of frame row y (round-robin or weighted deal).
__device__ __forceinline__ int part_of_row(const AssembleParams &a, int y, int *lr) {
    const int band = y / a.band_rows;
    int m, lband;
    if (a.cycle == 0) {
        m = band % a.n_parts;
        lband = band / a.n_parts;
    } else {
        const int c = band / a.cycle, pos = band - c * a.cycle;
        m = a.owner[pos];
        lband = c * a.cnt[m] + a.idx[pos];
    }
    *lr = lband * a.band_rows + (y - band * a.band_rows);
    return m;
}

// One pixel of a sparse part (svo_rt.h layout): a hit's colour from the part, a miss's
// sky computed here from the camera (the render kernel's miss branch).
__device__ __forceinline__ uint32_t sparse_pixel(const AssembleParams &a, int m, int lr, int x, int y) {
    const int tiles_x = (a.width + 7) / 8;
    const int t = (lr >> 3) * tiles_x + (x >> 3);
    const int bit = ((lr & 7) << 3) | (x & 7);
    const unsigned long long *masks = reinterpret_cast<const unsigned long long *>(a.parts[m]);
    const unsigned long long mk = masks[t];
    if ((mk >> bit) & 1ull) {
        const uint32_t *offsets = reinterpret_cast<const uint32_t *>(masks + a.n_tiles[m]);
        const uint32_t k = offsets[t] + (uint32_t)__popcll(mk & ((1ull << bit) - 1ull));
        const uint8_t *c = reinterpret_cast<const uint8_t *>(offsets + a.n_tiles[m] + 1) + 3 * (size_t)k;
        return (uint32_t)c[0] | ((uint32_t)c[1] << 8) | ((uint32_t)c[2] << 16) | (255u << 24);
    }
    float org[3], dir[3], rgb[3];
    camera_ray(a.cam, a.width, a.height, x, y, org, dir);
    sky(dir[1], rgb);
    return pack_rgba8(rgb[0], rgb[1], rgb[2]);
}

__global__ __launch_bounds__(256) void assemble_kernel(AssembleParams a) {
    const int x = (int)(blockIdx.x * 256 + threadIdx.x);
    const int y = (int)blockIdx.y;
    if (x >= a.width) return;
    int lr;
    const int m = part_of_row(a, y, &lr);
    if (m == a.skip_part) return;
    const size_t src = (size_t)lr * (size_t)a.width + (size_t)x;
    const size_t dst = (size_t)y * (size_t)a.width + (size_t)x;
    if (a.part_format == PART_RGBA8) {
        a.out.rgba8[dst] = reinterpret_cast<const uint32_t *>(a.parts[m])[src];
        return;
    }
    if (a.part_format == PART_RGB8) {
        const uint8_t *c = reinterpret_cast<const uint8_t *>(a.parts[m]) + 3 * src;
        a.out.rgba8[dst] = (uint32_t)c[0] | ((uint32_t)c[1] << 8) | ((uint32_t)c[2] << 16) | (255u << 24);
        return;
    }
    if (a.part_format == PART_SPARSE_RGB8) {
        a.out.rgba8[dst] = sparse_pixel(a, m, lr, x, y);
        return;
    }
    const uint3 c = reinterpret_cast<const uint3 *>(a.parts[m])[src];
    if (a.out.compact) reinterpret_cast<uint3 *>(a.out.compact)[dst] = c;
    if (!a.out.hits && !a.out.rgba && !a.out.rgba8) return;
    const bool hit = (c.y >> 16) & 1u;
    float n[3] = {0.0f, 0.0f, 0.0f}, rgb[3];
    if (hit) {   // the render kernel's decode + Shade on the display device's replica
        const uint2 at = c.x < a.n_nodes ? a.att[c.x] : make_uint2(0u, 0u);
        decode_normal(at.y >> 16, n);
        normalize3(n);
        if (a.out.rgba || a.out.rgba8) {
            if ((c.y >> 16) & 8u) {
                rgb[0] = rgb[1] = rgb[2] = 0.0f;
            } else {
                float alb[3];
                decode_dxt(at.x, at.y, (int)(c.y & 0xFFu), alb);
                shade_hit(a.cam, n, alb, rgb);
            }
        }
    } else if (a.out.rgba || a.out.rgba8) {
        float org[3], dir[3];
        camera_ray(a.cam, a.width, a.height, x, y, org, dir);
        sky(dir[1], rgb);
    }
    if (a.out.hits) {
        uint2 *d = reinterpret_cast<uint2 *>(a.out.hits + dst);
        d[0] = make_uint2(c.x, c.y);
        d[1] = make_uint2(c.z, __float_as_uint(n[0]));
        d[2] = make_uint2(__float_as_uint(n[1]), __float_as_uint(n[2]));
    }
    if (a.out.rgba) a.out.rgba[dst] = make_float4(rgb[0], rgb[1], rgb[2], 1.0f);
    if (a.out.rgba8) a.out.rgba8[dst] = pack_rgba8(rgb[0], rgb[1], rgb[2]);
}

}  // namespace

// Diagnostics only (env SVO_LDS_PAD=<bytes>, read once): extra LDS per render workgroup, to
// lower the resident waves per CU in occupancy sweeps; never set by callers.
static size_t lds_pad() {
    static const size_t pad = [] {
        const char *v = std::getenv("SVO_LDS_PAD");
        return v ? (size_t)std::strtoul(v, nullptr, 10) : (size_t)0;
    }();
    return pad;
}

template <int MODE, bool COUNT>
static hipError_t launch_variant(const LaunchParams &p, hipStream_t stream) {
    const int bx = (p.width + 7) / 8, by = (p.local_rows + 7) / 8;
    const size_t lds = (size_t)p.slots * TILE * sizeof(uint2) + lds_pad();
    const dim3 grid((unsigned)(bx * by)), block(TILE);
    if (!COUNT && p.samples > 0) {   // samples in flight: S waves per tile, S stacks (>= 1 KB each: the colours)
        const size_t per = (size_t)std::max(p.slots, 2) * TILE * sizeof(uint2);
        const dim3 sblock((unsigned)(TILE * p.samples));
        if (p.fetch_all && !p.guard)
            hipLaunchKernelGGL((render_samples_kernel<MODE, true>), grid, sblock, per * p.samples, stream, p, bx);
        else
            hipLaunchKernelGGL((render_samples_kernel<MODE, false>), grid, sblock, per * p.samples, stream, p, bx);
        return hipGetLastError();
    }
    if (!COUNT && p.seg > 0) {   // segmented heavy tiles (the order was built with seg_cap = p.seg)
        const dim3 sgrid((unsigned)order_strips_grid(bx * by, p.seg, p.seg_kmax));
        if (p.lat && p.wave_log)
            hipLaunchKernelGGL((render_seg_kernel<MODE, true, true, true>), sgrid, block, 2 * lds, stream, p, bx);
        else if (p.lat)
            hipLaunchKernelGGL((render_seg_kernel<MODE, true, true, false>), sgrid, block, 2 * lds, stream, p, bx);
        else if (p.fetch_all && p.wave_log)
            hipLaunchKernelGGL((render_seg_kernel<MODE, true, false, true>), sgrid, block, lds, stream, p, bx);
        else if (p.fetch_all)
            hipLaunchKernelGGL((render_seg_kernel<MODE, true, false, false>), sgrid, block, lds, stream, p, bx);
        else if (p.wave_log)
            hipLaunchKernelGGL((render_seg_kernel<MODE, false, false, true>), sgrid, block, lds, stream, p, bx);
        else
            hipLaunchKernelGGL((render_seg_kernel<MODE, false, false, false>), sgrid, block, lds, stream, p, bx);
        return hipGetLastError();
    }
    if (COUNT)
        hipLaunchKernelGGL((render_tile_kernel<MODE, true>), grid, block, lds, stream, p, bx);
    else if (p.lat)   // latency form (svo_rt.hip launch decides): the stack entries keep their node
        hipLaunchKernelGGL((render_tile_kernel<MODE, false, false, false, true>), grid, block, 2 * lds, stream, p, bx);
    else if (p.shadows == 2) {   // shadow pass fused into the primary launch
        if (p.fetch_all && !p.guard)
            hipLaunchKernelGGL((render_tile_kernel<MODE, false, true, true>), grid, block, lds, stream, p, bx);
        else
            hipLaunchKernelGGL((render_tile_kernel<MODE, false, false, true>), grid, block, lds, stream, p, bx);
    } else if (p.fetch_all && !p.guard)
        hipLaunchKernelGGL((render_tile_kernel<MODE, false, true>), grid, block, lds, stream, p, bx);
    else
        hipLaunchKernelGGL((render_tile_kernel<MODE, false>), grid, block, lds, stream, p, bx);
    return hipGetLastError();
}

// ---------------------------------------------------------- tile order
// Stable-free 4-class partition of the tiles by recorded cost, heaviest class
// first: class 0 = cost >= max/2, 1 = >= max/4, 2 = >= max/8, 3 = the rest.
// Only the start order of the heavy tiles matters (they bound the launch; the
// light ones fill in behind), so a partition does what a sort would
// (tools/wave_log.py: any order that dispatches the >= max/2 tiles first
// reaches the longest-wave bound).  One workgroup; every tile's cost is read
// with 16-byte loads into registers (32 per thread per chunk), classes are
// counted with ballots, positions come from mbcnt ranks: no atomics.
constexpr int ORDER_THREADS = 1024, ORDER_PER = 32, ORDER_CHUNK = ORDER_THREADS * ORDER_PER;

__device__ __forceinline__ void order_load(const uint16_t *cost, int chunk, int tid, uint32_t v[ORDER_PER / 2]) {
    const uint4 *src = reinterpret_cast<const uint4 *>(cost + (size_t)chunk * ORDER_CHUNK + (size_t)tid * ORDER_PER);
#pragma unroll
    for (int q = 0; q < ORDER_PER / 8; ++q) {
        const uint4 w = src[q];
        v[4 * q + 0] = w.x; v[4 * q + 1] = w.y; v[4 * q + 2] = w.z; v[4 * q + 3] = w.w;
    }
}

__global__ __launch_bounds__(ORDER_THREADS) void order_tiles_kernel(const uint16_t *__restrict__ cost,
                                                                    uint32_t *__restrict__ order, int n,
                                                                    uint32_t *stats) {
    constexpr int NW = ORDER_THREADS / 64, NC = 4;
    __shared__ uint32_t red[NW], red_sum[NW];
    __shared__ uint32_t cnt[NC][NW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n_chunks = (n + ORDER_CHUNK - 1) / ORDER_CHUNK;
    uint32_t v[ORDER_PER / 2];   // two 16-bit costs per word
    // ---- max cost
    uint32_t mx = 0, sum = 0;
    for (int c = 0; c < n_chunks; ++c) {
        order_load(cost, c, tid, v);
#pragma unroll
        for (int e = 0; e < ORDER_PER; ++e) {
            const int i = c * ORDER_CHUNK + tid * ORDER_PER + e;
            const uint32_t k = (v[e >> 1] >> ((e & 1) * 16)) & 0x7FFFu;   // (no SEG_COST_FLAG in this mode)
            if (i < n) {
                mx = max(mx, k);
                sum += k;
            }
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, d));
        sum += (uint32_t)__shfl_xor((int)sum, d);
    }
    if (lane == 0) {
        red[wave] = mx;
        red_sum[wave] = sum;
    }
    __syncthreads();
    mx = 0;
    sum = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        mx = max(mx, red[w]);
        sum += red_sum[w];
    }
    // the loop-form statistics (as order_strips_kernel's, all of it under "XCD 0")
    if (stats && tid < 8) {
        stats[2 * tid] = tid == 0 ? mx : 0u;
        stats[2 * tid + 1] = tid == 0 ? sum : 0u;
    }
    // class of a cost (NC = invalid element)
    auto cls = [mx](uint32_t k) { return 2 * k >= mx ? 0 : 4 * k >= mx ? 1 : 8 * k >= mx ? 2 : 3; };
    // ---- per-wave class counts
    uint32_t count[NC] = {0, 0, 0, 0};
    for (int c = 0; c < n_chunks; ++c) {
        if (n_chunks > 1) order_load(cost, c, tid, v);
#pragma unroll
        for (int e = 0; e < ORDER_PER; ++e) {
            const int i = c * ORDER_CHUNK + tid * ORDER_PER + e;
            const int k = i < n ? cls((v[e >> 1] >> ((e & 1) * 16)) & 0x7FFFu) : NC;
#pragma unroll
            for (int q = 0; q < NC; ++q) count[q] += (uint32_t)__popcll(__ballot(k == q));
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < NC; ++q) cnt[q][wave] = count[q];
    }
    __syncthreads();
    uint32_t run[NC];
    uint32_t before = 0;
#pragma unroll
    for (int q = 0; q < NC; ++q) {
        uint32_t mine = before;
        for (int w = 0; w < NW; ++w) {
            if (w < wave) mine += cnt[q][w];
            before += cnt[q][w];
        }
        run[q] = mine;
        if (tid == 0) order[n + q] = before;   // class boundaries: end of class q in the order
    }
    // ---- scatter
    for (int c = 0; c < n_chunks; ++c) {
        if (n_chunks > 1) order_load(cost, c, tid, v);
#pragma unroll
        for (int e = 0; e < ORDER_PER; ++e) {
            const int i = c * ORDER_CHUNK + tid * ORDER_PER + e;
            const int k = i < n ? cls((v[e >> 1] >> ((e & 1) * 16)) & 0x7FFFu) : NC;
            uint32_t pos = 0;
#pragma unroll
            for (int q = 0; q < NC; ++q) {
                const uint64_t m = __ballot(k == q);
                if (k == q) pos = run[q] + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                run[q] += (uint32_t)__popcll(m);
            }
            if (k < NC) order[pos] = (uint32_t)i;
        }
    }
}

size_t order_cost_capacity(int n_tiles) {
    return ((size_t)n_tiles + ORDER_CHUNK - 1) / ORDER_CHUNK * ORDER_CHUNK;
}

// XCD strips (remap 2): workgroup x orders the tiles of XCD x's column strips
// (see strip_tile) heaviest class first and writes them to the block positions
// b = 8 j + x; the per-XCD class ends (in units of j) go to order[n + 4 + 4 x + c].
// stats (nullable, host-visible): [2 x] = the max and [2 x + 1] = the sum of XCD x's tile
// costs -- the launch's heaviest wave and its total wave trips, which the host uses to pick
// the loop form of the next launches (svo_rt.hip launch).
__global__ __launch_bounds__(ORDER_THREADS) void order_strips_kernel(const uint16_t *__restrict__ cost_in,
                                                                     uint32_t *__restrict__ order, int n, int tiles_x,
                                                                     uint32_t *stats, int seg_cap,
                                                                     const uint16_t *__restrict__ part_cost,
                                                                     int seg_kpack, int spread) {
    __shared__ uint32_t red[ORDER_THREADS / 64], red_sum[ORDER_THREADS / 64];
    constexpr int NC = 6;
    __shared__ uint32_t cnt[NC], base[NC + 1], rank[NC], segs[NC];
    const int x = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int len = n / 8, tiles_y = n / tiles_x;
    const int L = len + (seg_kmax_of(seg_kpack) - 1) * seg_cap;   // every XCD's list length (grid = 8 L)
    // a segmented tile's parts recorded their own continuous-equivalent trips (render_seg_kernel)
    auto cost_at = [&](int t) -> uint32_t {
        const uint32_t k = cost_in[t];
        if (!(k & SEG_COST_FLAG) || !part_cost) return k & 0x7FFFu;
        const uint4 q = *reinterpret_cast<const uint4 *>(part_cost + SEG_KMAX * (size_t)t);
        uint32_t m = max(max(q.x & 0xFFFFu, q.x >> 16), max(q.y & 0xFFFFu, q.y >> 16));
        if ((k & 15u) == 8u) m = max(m, max(max(q.z & 0xFFFFu, q.z >> 16), max(q.w & 0xFFFFu, q.w >> 16)));
        return m;
    };
    // position e of this XCD's list is (column c = e / tiles_y, row e % tiles_y) of its
    // strips (strip_tile); the threads walk it in steps of ORDER_THREADS with one
    // division at the start instead of integer divisions per element (11.6 -> 9.7 us
    // per launch at 1080p)
    const int dc = ORDER_THREADS / tiles_y, dr = ORDER_THREADS % tiles_y;
    struct Walk { int e, c, r; };
    auto start = [&]() { return Walk{tid, tid / tiles_y, tid % tiles_y}; };
    auto next = [&](Walk &w) {
        w.e += ORDER_THREADS; w.c += dc; w.r += dr;
        if (w.r >= tiles_y) { w.r -= tiles_y; w.c += 1; }
    };
    auto tile_of = [&](const Walk &w) { return w.r * tiles_x + strip_col(x, w.c); };
    // spread (a moving camera: the costs are a few frames old and the heavy tiles have drifted by up to
    // a tile on screen): a tile's class is that of the heaviest of it and its 8 neighbours
    auto class_cost = [&](const Walk &w) -> uint32_t {
        const int col = strip_col(x, w.c);
        if (!spread) return cost_at(w.r * tiles_x + col);
        uint32_t m = 0;
        for (int dy = -1; dy <= 1; ++dy) {
            const int r = w.r + dy;
            if (r < 0 || r >= tiles_y) continue;
            for (int dx = -1; dx <= 1; ++dx) {
                const int c = col + dx;
                if (c >= 0 && c < tiles_x) m = max(m, cost_at(r * tiles_x + c));
            }
        }
        return m;
    };
    uint32_t mx = 0, sum = 0;
    for (Walk w = start(); w.e < len; next(w)) {
        const uint32_t k = cost_at(tile_of(w));
        mx = max(mx, k);
        sum += k;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, d));
        sum += (uint32_t)__shfl_xor((int)sum, d);
    }
    if (lane == 0) {
        red[wave] = mx;
        red_sum[wave] = sum;
    }
    if (tid < NC) cnt[tid] = 0;
    __syncthreads();
    mx = 0;
    sum = 0;
#pragma unroll
    for (int w = 0; w < ORDER_THREADS / 64; ++w) {
        mx = max(mx, red[w]);
        sum += red_sum[w];
    }
    if (stats && tid == 0) {
        stats[2 * x] = mx;
        stats[2 * x + 1] = sum;
    }
    // six classes, the top half split three ways so the very heaviest tiles are the
    // XCD's first dispatches (they bound the launch); the render kernel's s_setprio
    // classes are >= 1/2, >= 1/4, >= 1/8 of the XCD's max and the rest
    auto cls = [mx](uint32_t k) {
        return 8 * k >= 7 * mx ? 0 : 4 * k >= 3 * mx ? 1 : 2 * k >= mx ? 2 : 4 * k >= mx ? 3 : 8 * k >= mx ? 4 : 5;
    };
    for (Walk w = start(); w.e < len; next(w)) atomicAdd(&cnt[cls(class_cost(w))], 1u);
    __syncthreads();
    const int G = 8 * L;   // the grid, and where the class ends go
    if (tid == 0) {
        // seg_cap > 0: the tiles of the classes seg_kpack segments (heaviest first, at most seg_cap
        // per XCD) take K consecutive slots each, one per part
        uint32_t run = 0, left = (uint32_t)seg_cap;
        for (int c = 0; c < NC; ++c) {
            const uint32_t kc = (uint32_t)(seg_kpack >> (4 * c)) & 15u;
            segs[c] = kc > 1 ? min(cnt[c], left) : 0u;
            left -= segs[c];
            base[c] = run;
            rank[c] = 0;
            run += cnt[c] + (kc > 1 ? kc - 1 : 0u) * segs[c];
            if (c >= 2) order[G + 4 + 4 * x + (c - 2)] = run;   // prio class ends
        }
        base[NC] = run;
        if (x == 0) for (int c = 0; c < 4; ++c) order[G + c] = 0;   // global bounds unused in this mode
    }
    __syncthreads();
    for (Walk w = start(); w.e < len; next(w)) {
        const int t = tile_of(w);
        const int c = cls(class_cost(w));
        const uint32_t r = atomicAdd(&rank[c], 1u);
        const uint32_t kc = (uint32_t)(seg_kpack >> (4 * c)) & 15u;
        if (r < segs[c]) {
            const uint32_t j = base[c] + kc * r;
            const uint32_t code0 = kc == 4 ? 1u : 5u;   // part q: code0 + q
            for (uint32_t q = 0; q < kc; ++q) order[(size_t)(j + q) * 8 + x] = (uint32_t)t | ((code0 + q) << 28);
        } else {
            const uint32_t j = base[c] + (kc > 1 ? kc - 1 : 0u) * segs[c] + r;
            order[(size_t)j * 8 + x] = (uint32_t)t;
        }
    }
    for (int j = (int)base[NC] + tid; j < L; j += ORDER_THREADS) order[(size_t)j * 8 + x] = SEG_EMPTY;
}

hipError_t launch_order_strips(const uint16_t *cost, uint32_t *order, int n_tiles, int tiles_x, hipStream_t stream,
                               uint32_t *stats, int seg_cap, const uint16_t *part_cost, int seg_kpack, int spread) {
    if (n_tiles <= 0) return hipSuccess;
    if (seg_cap > 0 && (n_tiles / tiles_x) * tiles_x != n_tiles) return hipErrorInvalidValue;
    for (int c = 0; c < 6; ++c) {
        const int kc = (seg_kpack >> (4 * c)) & 15;
        if (kc != 0 && kc != 4 && kc != 8) return hipErrorInvalidValue;
    }
    if (seg_cap > 0 && ((size_t)order_strips_grid(n_tiles, seg_cap, seg_kmax_of(seg_kpack)) >> 28) != 0)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(order_strips_kernel, dim3(8), dim3(ORDER_THREADS), 0, stream, cost, order, n_tiles, tiles_x,
                       stats, seg_cap, part_cost, seg_kpack, spread);
    return hipGetLastError();
}

hipError_t launch_order_tiles(const uint16_t *cost, uint32_t *order, int n_tiles, hipStream_t stream,
                              uint32_t *stats) {
    if (n_tiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(order_tiles_kernel, dim3(1), dim3(ORDER_THREADS), 0, stream, cost, order, n_tiles, stats);
    return hipGetLastError();
}

// ---------------------------------------------------------- accumulation
// AddShader.shader:44-47 + Blend SrcAlpha OneMinusSrcAlpha (:10), driven by
// RaytracingMaster.cs:70-73: dst = src * a + dst * (1 - a), a = 1/(sample+1),
// on all four channels (the source alpha is a).  Pure HBM streaming: 16 B read
// of the sample + 16 B read and 16 B write of the accumulation per pixel,
// float4 per lane, grid-stride.
__global__ __launch_bounds__(256) void accumulate_kernel(float4 *__restrict__ dst, const float4 *__restrict__ src,
                                                         size_t n, float a, float b) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float4 s = src[i];
        float4 d = dst[i];
        d.x = s.x * a + d.x * b;
        d.y = s.y * a + d.y * b;
        d.z = s.z * a + d.z * b;
        d.w = a * a + d.w * b;
        dst[i] = d;
    }
}

hipError_t launch_accumulate(float4 *dst, const float4 *src, size_t n_px, uint32_t sample, int num_cus,
                             hipStream_t stream) {
    if (n_px == 0) return hipSuccess;
    const float a = 1.0f / ((float)sample + 1.0f);
    const float b = 1.0f - a;
    const size_t want = (n_px + 255) / 256;
    const unsigned blocks = (unsigned)std::min<size_t>(want, (size_t)num_cus * 16);
    hipLaunchKernelGGL(accumulate_kernel, dim3(blocks), dim3(256), 0, stream, dst, src, n_px, a, b);
    return hipGetLastError();
}

// svo_render_progressive_async (svo_config.readback 1): the packed display words pushed into the
// plugin's mapped pinned host buffer by a kernel (PCIe writes from every workgroup) instead of
// one DMA copy; 16 B per lane, grid-stride, non-temporal stores.
__global__ __launch_bounds__(256) void push_host_kernel(const uint4 *__restrict__ src, uint4 *__restrict__ dst,
                                                        size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        const uint4 v = src[i];
        __builtin_nontemporal_store(v.x, &dst[i].x);
        __builtin_nontemporal_store(v.y, &dst[i].y);
        __builtin_nontemporal_store(v.z, &dst[i].z);
        __builtin_nontemporal_store(v.w, &dst[i].w);
    }
}

hipError_t launch_push_host(const void *src, void *dst_mapped, size_t bytes, int blocks, hipStream_t stream) {
    if (bytes == 0) return hipSuccess;
    const size_t n16 = bytes / 16;   // callers pass multiples of 16 bytes (whole frames of 4-byte words, padded)
    hipLaunchKernelGGL(push_host_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                       reinterpret_cast<const uint4 *>(src), reinterpret_cast<uint4 *>(dst_mapped), n16);
    return hipGetLastError();
}

// Display RGBA8 of an RGBA32F frame (the accumulated Result): saturate, * 255,
// round half up per colour channel, opaque alpha.  == orc_pack_rgba8.
__global__ __launch_bounds__(256) void pack_rgba8_kernel(const float4 *__restrict__ src, uint32_t *__restrict__ dst,
                                                         size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float4 c = src[i];
        auto q = [](float v) {
            v = fminf(fmaxf(v, 0.0f), 1.0f);
            v = v * 255.0f;
            return (uint32_t)(v + 0.5f);
        };
        dst[i] = q(c.x) | (q(c.y) << 8) | (q(c.z) << 16) | (255u << 24);
    }
}

// The same words without their constant alpha, 3 bytes per pixel (Unity TextureFormat.RGB24):
// 4 pixels per lane -> 3 dwords, so the stores stay whole and aligned; a tail of < 4 pixels
// is written bytewise by the last lane.
__global__ __launch_bounds__(256) void pack_rgb8_kernel(const float4 *__restrict__ src, uint8_t *__restrict__ dst,
                                                        size_t n) {
    auto q = [](float v) {
        v = fminf(fmaxf(v, 0.0f), 1.0f);
        v = v * 255.0f;
        return (uint32_t)(v + 0.5f);
    };
    const size_t groups = n / 4, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < groups; g += stride) {
        uint32_t b[12];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 c = src[4 * g + j];
            b[3 * j] = q(c.x);
            b[3 * j + 1] = q(c.y);
            b[3 * j + 2] = q(c.z);
        }
        uint32_t *d = reinterpret_cast<uint32_t *>(dst + 12 * g);
#pragma unroll
        for (int w = 0; w < 3; ++w) d[w] = b[4 * w] | (b[4 * w + 1] << 8) | (b[4 * w + 2] << 16) | (b[4 * w + 3] << 24);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (size_t i = 4 * groups; i < n; ++i) {
            const float4 c = src[i];
            dst[3 * i] = (uint8_t)q(c.x);
            dst[3 * i + 1] = (uint8_t)q(c.y);
            dst[3 * i + 2] = (uint8_t)q(c.z);
        }
}

hipError_t launch_pack_rgb8(const float4 *src, uint8_t *dst, size_t n_px, int num_cus, hipStream_t stream) {
    if (n_px == 0) return hipSuccess;
    const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>((n_px / 4 + 255) / 256, (size_t)num_cus * 16));
    hipLaunchKernelGGL(pack_rgb8_kernel, dim3(blocks), dim3(256), 0, stream, src, dst, n_px);
    return hipGetLastError();
}

hipError_t launch_pack_rgba8(const float4 *src, uint32_t *dst, size_t n_px, int num_cus, hipStream_t stream) {
    if (n_px == 0) return hipSuccess;
    const unsigned blocks = (unsigned)std::min<size_t>((n_px + 255) / 256, (size_t)num_cus * 16);
    hipLaunchKernelGGL(pack_rgba8_kernel, dim3(blocks), dim3(256), 0, stream, src, dst, n_px);
    return hipGetLastError();
}

// RGBA8 / RGB8 parts: pure data movement (4 or 3 B read + 4 B written per pixel), so
// 4 pixels per lane and the row's band arithmetic once per workgroup (row =
// blockIdx.y).  Needs width % 4 == 0 (16-byte aligned RGBA rows, 4-byte aligned RGB
// groups in every part and in the frame).
__global__ __launch_bounds__(256) void assemble_rgba8_kernel(AssembleParams a) {
    const int y = (int)blockIdx.y;
    int lr;
    const int m = part_of_row(a, y, &lr);
    if (m == a.skip_part) return;
    const int q = (int)(blockIdx.x * 256 + threadIdx.x);   // 4-pixel group of the row
    if (4 * q >= a.width) return;
    uint4 *dst = reinterpret_cast<uint4 *>(a.out.rgba8 + (size_t)y * (size_t)a.width);
    if (a.part_format == PART_RGB8) {   // 12 bytes (4 x RGB) -> 16 (4 x RGBA, alpha 255)
        const uint32_t *row = reinterpret_cast<const uint32_t *>(a.parts[m]) + (size_t)lr * (size_t)(3 * a.width / 4);
        const uint32_t w0 = row[3 * q], w1 = row[3 * q + 1], w2 = row[3 * q + 2];
        const uint32_t A = 255u << 24;
        dst[q] = make_uint4((w0 & 0xFFFFFFu) | A, (w0 >> 24) | ((w1 & 0xFFFFu) << 8) | A,
                            (w1 >> 16) | ((w2 & 0xFFu) << 16) | A, (w2 >> 8) | A);
        return;
    }
    if (a.part_format == PART_SPARSE_RGB8) {   // 4 pixels of one tile row: one mask, one offset
        const int x = 4 * q;
        dst[q] = make_uint4(sparse_pixel(a, m, lr, x, y), sparse_pixel(a, m, lr, x + 1, y),
                            sparse_pixel(a, m, lr, x + 2, y), sparse_pixel(a, m, lr, x + 3, y));
        return;
    }
    const uint4 *src = reinterpret_cast<const uint4 *>(reinterpret_cast<const uint32_t *>(a.parts[m]) +
                                                       (size_t)lr * (size_t)a.width);
    dst[q] = src[q];
}

// ------------------------------------------------------ sparse hit payload
// Two launches over the band's n tiles (svo_rt.h layout).
// (1) tile_scan_local: one workgroup per chunk of SCAN_THREADS tiles scans the masks'
//     popcounts (wave prefix by shuffles, then across the 16 waves in LDS) into the
//     part's scratch tail: L[t] = hits before t within its chunk, S[c] = chunk c's total.
// (2) pack_hits: one thread per pixel; a 256-pixel row segment spans 32 tiles, so at
//     most two chunks: the workgroup sums S over the chunks before its first one and
//     every pixel gets offset(t) = L[t] + its chunk's prefix.  A tile's first pixel
//     writes offset(t) into the part's head (the last tile also the count), a hit pixel
//     its 3 bytes to slot offset(t) + the tile's hit lanes before it.
constexpr int SCAN_THREADS = 1024;
constexpr int PACK_THREADS = 256;

struct SparseLayout {   // byte offsets of a part (svo_rt.h SVO_SPARSE_*)
    size_t offsets, rgb, scratch;
};
// elem: bytes per packed hit (3: RGB payload, 4: pixel index of the compacted shadow pass)
__host__ __device__ inline SparseLayout sparse_layout(int n, int n_px, int elem = 3) {
    SparseLayout l;
    l.offsets = 8 * (size_t)n;
    l.rgb = 12 * (size_t)n + 4;
    l.scratch = (l.rgb + (size_t)elem * (size_t)n_px + 3) & ~(size_t)3;
    return l;
}

__global__ __launch_bounds__(SCAN_THREADS) void tile_scan_local_kernel(const unsigned long long *__restrict__ masks,
                                                                       int n, uint32_t *__restrict__ local,
                                                                       uint32_t *__restrict__ sums,
                                                                       uint32_t *__restrict__ count) {
    __shared__ uint32_t wave_sum[SCAN_THREADS / 64];
    const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int i = (int)blockIdx.x * SCAN_THREADS + tid;
    const uint32_t c = i < n ? (uint32_t)__popcll(masks[i]) : 0u;
    uint32_t incl = c;   // inclusive prefix within the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)incl, d);
        if (lane >= d) incl += v;
    }
    if (lane == 63) wave_sum[wave] = incl;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (int w = 0; w < SCAN_THREADS / 64; ++w) {
        const uint32_t v = wave_sum[w];
        if (w < wave) before += v;
        total += v;
    }
    if (i < n) local[i] = before + incl - c;
    if (tid == 0) sums[blockIdx.x] = total;
    if (n == 0 && tid == 0) *count = 0u;   // an empty band: no pack workgroup writes it
}

// INDEX: pack the hit pixels' band-local indices (lr * width + x, 4 bytes) instead of
// their RGB -- the compacted shadow pass's hit list.
template <bool INDEX>
__global__ __launch_bounds__(PACK_THREADS) void pack_hits_kernel(const uint8_t *__restrict__ rgb8, int width,
                                                                 int local_rows, uint8_t *__restrict__ part) {
    __shared__ uint32_t wsum[PACK_THREADS / 64];
    const int tiles_x = (width + 7) / 8;
    const int n = tiles_x * ((local_rows + 7) / 8);
    const SparseLayout L = sparse_layout(n, width * local_rows, INDEX ? 4 : 3);
    const unsigned long long *masks = reinterpret_cast<const unsigned long long *>(part);
    uint32_t *offsets = reinterpret_cast<uint32_t *>(part + L.offsets);
    const uint32_t *local = reinterpret_cast<const uint32_t *>(part + L.scratch);
    const uint32_t *sums = local + n;
    const int lr = (int)blockIdx.y;
    const int x0 = (int)blockIdx.x * PACK_THREADS;
    const int c0 = ((lr >> 3) * tiles_x + (x0 >> 3)) / SCAN_THREADS;   // the segment's first chunk
    uint32_t v = 0;
    for (int c = (int)threadIdx.x; c < c0; c += PACK_THREADS) v += sums[c];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += (uint32_t)__shfl_xor((int)v, d);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
    __syncthreads();
    const uint32_t prefix0 = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    const int x = x0 + (int)threadIdx.x;
    if (x >= width) return;
    const int t = (lr >> 3) * tiles_x + (x >> 3);
    const int bit = ((lr & 7) << 3) | (x & 7);
    const unsigned long long mk = masks[t];
    const uint32_t off = local[t] + prefix0 + (t / SCAN_THREADS > c0 ? sums[c0] : 0u);
    if (bit == 0) {
        offsets[t] = off;
        if (t == n - 1) offsets[n] = off + (uint32_t)__popcll(mk);   // the band's hit count
    }
    if (!((mk >> bit) & 1ull)) return;
    const uint32_t k = off + (uint32_t)__popcll(mk & ((1ull << bit) - 1ull));
    if (INDEX) {
        reinterpret_cast<uint32_t *>(part + L.rgb)[k] = (uint32_t)lr * (uint32_t)width + (uint32_t)x;
        return;
    }
    const uint8_t *src = rgb8 + 3 * ((size_t)lr * (size_t)width + (size_t)x);
    uint8_t *dst = part + L.rgb + 3 * (size_t)k;
    dst[0] = src[0];
    dst[1] = src[1];
    dst[2] = src[2];
}

template <bool INDEX>
static hipError_t launch_pack(const uint8_t *rgb8, int width, int local_rows, void *part, hipStream_t stream) {
    if (width <= 0 || local_rows < 0) return hipSuccess;
    const int n = ((width + 7) / 8) * ((local_rows + 7) / 8);
    const int chunks = (n + SCAN_THREADS - 1) / SCAN_THREADS;
    uint8_t *p = reinterpret_cast<uint8_t *>(part);
    const SparseLayout L = sparse_layout(n, width * local_rows, INDEX ? 4 : 3);
    uint32_t *local = reinterpret_cast<uint32_t *>(p + L.scratch);
    hipLaunchKernelGGL(tile_scan_local_kernel, dim3(chunks > 0 ? chunks : 1), dim3(SCAN_THREADS), 0, stream,
                       reinterpret_cast<const unsigned long long *>(p), n, local, local + n,
                       reinterpret_cast<uint32_t *>(p + L.offsets) + n);
    if (local_rows > 0) {
        const dim3 grid((unsigned)((width + PACK_THREADS - 1) / PACK_THREADS), (unsigned)local_rows);
        hipLaunchKernelGGL(pack_hits_kernel<INDEX>, grid, dim3(PACK_THREADS), 0, stream, rgb8, width, local_rows, p);
    }
    return hipGetLastError();
}

hipError_t launch_pack_hits(const uint8_t *rgb8, int width, int local_rows, void *part, hipStream_t stream) {
    return launch_pack<false>(rgb8, width, local_rows, part, stream);
}

size_t shadow_list_bytes(int width, int local_rows) {
    const int n = ((width + 7) / 8) * ((local_rows + 7) / 8);
    return sparse_layout(n, width * local_rows, 4).scratch + 4 * (size_t)n + 4 * (size_t)((n + SCAN_THREADS - 1) / SCAN_THREADS);
}

hipError_t launch_assemble(const AssembleParams &a, hipStream_t stream) {
    if (a.width <= 0 || a.height <= 0) return hipSuccess;
    if ((a.part_format == PART_RGBA8 || a.part_format == PART_RGB8 || a.part_format == PART_SPARSE_RGB8) &&
        a.width % 4 == 0) {
        const dim3 grid((unsigned)((a.width / 4 + 255) / 256), (unsigned)a.height);
        hipLaunchKernelGGL(assemble_rgba8_kernel, grid, dim3(256), 0, stream, a);
        return hipGetLastError();
    }
    const dim3 grid((unsigned)((a.width + 255) / 256), (unsigned)a.height);
    hipLaunchKernelGGL(assemble_kernel, grid, dim3(256), 0, stream, a);
    return hipGetLastError();
}

// ------------------------------------------------------------- beam splat
// One thread per box of the pool's splat list (svo_rt.hip build_beam_boxes): the box's Euclidean
// distance from the camera bounds from below the t at which any ray can enter it, so that
// distance is min-ed into every 8x8 tile whose rays can reach the box -- those whose pixel area
// (any offset in [0, 1]) meets the box's screen projection.  The projection is the bounding box of
// the projected corners, after clipping the box to the part in front of the camera (q_z > eps:
// the edges crossing that plane add their crossing points).  A box a tile's rays miss only costs
// that tile a lower start; a box they can reach is never left out, so every tile's value is <=
// the hit t of each of its rays (exact).
// Entries are 64-bit keys (~gen << 32 | distance bits): a launch's keys are below every older
// launch's, so one atomic min both replaces a stale entry and keeps the nearest box -- no fill
// pass; a reader takes an entry of another generation as +inf.  The list is in Morton order, so
// a workgroup's boxes cover a compact patch of the screen: their tiles are min-ed in an LDS window
// first and each touched tile costs one global atomic per workgroup (device-scope atomics from
// every XCD to one address serialise: one atomic per box-tile pair took 72 us per C3 frame).
#ifndef SVO_SPLAT_THREADS
#define SVO_SPLAT_THREADS 512
#endif
constexpr int SPLAT_THREADS = SVO_SPLAT_THREADS, SPLAT_WIN = 8192;

// no read first: a returning load before each atomic put a full memory round trip into every
// iteration of the flush loop (24 us per C3 frame); the atomic alone returns nothing to wait for
__device__ __forceinline__ void beam_min(unsigned long long *a, unsigned long long key, uint32_t diag = 0) {
    if (!(diag & 1)) atomicMin(a, key);
}

// One box of the splat list: kind 0 (no ray reaches it), 1 (tiles [tx0, tx1] x [ty0, ty1]), 2 (the
// super tiles over them) or 3 (the global word), and its distance from the camera.
__device__ __forceinline__ void beam_box(const BeamParams &b, uint32_t i, int &kind, int &tx0, int &ty0, int &tx1,
                                         int &ty1, float &dist) {
    kind = 0;
    tx0 = ty0 = 0;
    tx1 = ty1 = -1;
    dist = 0.0f;
    const uint2 e = b.boxes[i];
    const int dep = (int)(e.y >> 16);
    const float size = __uint_as_float((uint32_t)(127 - dep) << 23);   // 2^-depth
    const float lo[3] = {1.0f + (float)(e.x & 0xFFFFu) * size, 1.0f + (float)(e.x >> 16) * size,
                         1.0f + (float)(e.y & 0xFFFFu) * size};   // exact (17 significant bits)
    float rel[3], d2 = 0.0f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        rel[k] = lo[k] - b.org[k];
        const float m = fmaxf(fmaxf(rel[k], -(rel[k] + size)), 0.0f);   // gap to the box along axis k
        d2 += m * m;
    }
    dist = __builtin_amdgcn_sqrtf(d2);   // 1 ulp: inside the render's 2^-16 margin
    // outside a side plane of the view frustum (the planes sit a pixel outside the frame): no ray
    const float span = fabsf(rel[0]) + fabsf(rel[1]) + fabsf(rel[2]) + 3.0f * size;
    bool in = true;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float *n = b.plane[j];
        const float top = n[0] * rel[0] + n[1] * rel[1] + n[2] * rel[2] +
                          size * (fmaxf(n[0], 0.0f) + fmaxf(n[1], 0.0f) + fmaxf(n[2], 0.0f));
        in = in && !(top < -1e-5f * span);
    }
    // the box's corners in (fx, fy, 1)-space, q = Minv (P - o), by increments; its projection is the
    // hull of the corners' (qx / qz, qy / qz) when every corner lies in front of the camera
    float q0[3], g[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        q0[r] = b.minv[3 * r] * rel[0] + b.minv[3 * r + 1] * rel[1] + b.minv[3 * r + 2] * rel[2];
#pragma unroll
        for (int k = 0; k < 3; ++k) g[k][r] = b.minv[3 * r + k] * size;
    }
    float zmin = __builtin_inff(), zmax = -__builtin_inff();
    float x0 = __builtin_inff(), x1 = -__builtin_inff(), y0 = __builtin_inff(), y1 = -__builtin_inff();
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const float qx = q0[0] + ((c & 1) ? g[0][0] : 0.0f) + ((c & 2) ? g[1][0] : 0.0f) + ((c & 4) ? g[2][0] : 0.0f);
        const float qy = q0[1] + ((c & 1) ? g[0][1] : 0.0f) + ((c & 2) ? g[1][1] : 0.0f) + ((c & 4) ? g[2][1] : 0.0f);
        const float qz = q0[2] + ((c & 1) ? g[0][2] : 0.0f) + ((c & 2) ? g[1][2] : 0.0f) + ((c & 4) ? g[2][2] : 0.0f);
        zmin = fminf(zmin, qz);
        zmax = fmaxf(zmax, qz);
        const float rz = __builtin_amdgcn_rcpf(qz);   // 1 ulp: far inside the pixel margin below
        x0 = fminf(x0, qx * rz); x1 = fmaxf(x1, qx * rz);
        y0 = fminf(y0, qy * rz); y1 = fmaxf(y1, qy * rz);
    }
    in = in && zmax > 0.0f;   // else wholly behind the camera
    if (in && dist <= 1e-3f * size) {   // the camera at the box: every ray
        kind = 3;
    } else if (in && zmin > 1e-5f * zmax) {   // wholly in front: the corners' hull (x0 .. y1 above)
    } else if (in) {
        // across the camera plane (rare: near the camera): the corners in front of q_z = eps and the
        // crossing points of the edges through that plane
        float qx[8], qy[8], qz[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const float sx = (c & 1) ? size : 0.0f, sy = (c & 2) ? size : 0.0f, sz = (c & 4) ? size : 0.0f;
            qx[c] = b.minv[0] * (rel[0] + sx) + b.minv[1] * (rel[1] + sy) + b.minv[2] * (rel[2] + sz);
            qy[c] = b.minv[3] * (rel[0] + sx) + b.minv[4] * (rel[1] + sy) + b.minv[5] * (rel[2] + sz);
            qz[c] = b.minv[6] * (rel[0] + sx) + b.minv[7] * (rel[1] + sy) + b.minv[8] * (rel[2] + sz);
        }
        const float eps = zmax * 1e-5f;
        x0 = y0 = __builtin_inff();
        x1 = y1 = -__builtin_inff();
        for (int c = 0; c < 8; ++c) {
            if (qz[c] > eps) {
                const float fx = qx[c] / qz[c], fy = qy[c] / qz[c];
                x0 = fminf(x0, fx); x1 = fmaxf(x1, fx); y0 = fminf(y0, fy); y1 = fmaxf(y1, fy);
            }
            for (int bit = 1; bit < 8; bit <<= 1) {   // the 12 edges (c, c | bit), c without bit
                if (c & bit) continue;
                const int d = c | bit;
                if ((qz[c] > eps) == (qz[d] > eps)) continue;
                const float s = (eps - qz[c]) / (qz[d] - qz[c]);
                const float fx = (qx[c] + s * (qx[d] - qx[c])) / eps, fy = (qy[c] + s * (qy[d] - qy[c])) / eps;
                x0 = fminf(x0, fx); x1 = fmaxf(x1, fx); y0 = fminf(y0, fy); y1 = fmaxf(y1, fy);
            }
        }
        x0 -= fabsf(x0) * 1e-5f; x1 += fabsf(x1) * 1e-5f;   // the corner and clipping roundings
        y0 -= fabsf(y0) * 1e-5f; y1 += fabsf(y1) * 1e-5f;
    }
    if (in && kind == 0) {
        const float mg = 0.05f;   // pixels: rounding of the projection and of the rays' own u, v
        x0 -= mg; y0 -= mg; x1 += mg; y1 += mg;
        if (x1 >= 0.0f && y1 >= 0.0f && x0 <= (float)b.width && y0 <= (float)b.height) {
            tx0 = (int)(fmaxf(x0, 0.0f) * 0.125f);
            ty0 = (int)(fmaxf(y0, 0.0f) * 0.125f);
            tx1 = min((int)(fminf(x1, (float)b.width) * 0.125f), b.tiles_x - 1);
            ty1 = min((int)(fminf(y1, (float)b.height) * 0.125f), b.tiles_y - 1);
            if (tx1 >= tx0 && ty1 >= ty0) {
                const int nt = (tx1 - tx0 + 1) * (ty1 - ty0 + 1);
                const int ns = ((tx1 >> 3) - (tx0 >> 3) + 1) * ((ty1 >> 3) - (ty0 >> 3) + 1);
                kind = nt <= 32 ? 1 : ns <= 32 ? 2 : 3;
            }
        }
    }
}

constexpr int SPLAT_PER = 1;   // boxes per thread (4: 14.9 us per C3 frame against 8.9 with 1)

__global__ __launch_bounds__(SPLAT_THREADS) void beam_splat_kernel(BeamParams b) {
    __shared__ uint32_t win[SPLAT_WIN];
    __shared__ int rect[4];
    const unsigned long long gen = (unsigned long long)(~b.gen) << 32;
    unsigned long long *const ts = b.tile_start;
    int kind[SPLAT_PER], tx0[SPLAT_PER], ty0[SPLAT_PER], tx1[SPLAT_PER], ty1[SPLAT_PER];
    float dist[SPLAT_PER];
    const uint32_t base = blockIdx.x * (SPLAT_THREADS * SPLAT_PER) + threadIdx.x;
#pragma unroll
    for (int k = 0; k < SPLAT_PER; ++k) {
        const uint32_t i = base + k * SPLAT_THREADS;
        kind[k] = 0;
        if (i < b.n_boxes) beam_box(b, i, kind[k], tx0[k], ty0[k], tx1[k], ty1[k], dist[k]);
    }
    // the workgroup's tile window: reduced across the wave first (every lane on the same 4 LDS words
    // serialises: ~8 us per C3 frame), then one LDS atomic per wave
    if (threadIdx.x == 0) {
        rect[0] = rect[1] = 0x7FFFFFFF;
        rect[2] = rect[3] = -1;
    }
    __syncthreads();
    {
        int a0 = 0x7FFFFFFF, a1 = 0x7FFFFFFF, a2 = -1, a3 = -1;
#pragma unroll
        for (int k = 0; k < SPLAT_PER; ++k)
            if (kind[k] == 1) {
                a0 = min(a0, tx0[k]); a1 = min(a1, ty0[k]); a2 = max(a2, tx1[k]); a3 = max(a3, ty1[k]);
            }
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            a0 = min(a0, __shfl_xor(a0, d));
            a1 = min(a1, __shfl_xor(a1, d));
            a2 = max(a2, __shfl_xor(a2, d));
            a3 = max(a3, __shfl_xor(a3, d));
        }
        if ((threadIdx.x & 63) == 0 && a2 >= 0) {
            atomicMin(&rect[0], a0);
            atomicMin(&rect[1], a1);
            atomicMax(&rect[2], a2);
            atomicMax(&rect[3], a3);
        }
    }
    __syncthreads();
    const int rx0 = rect[0], ry0 = rect[1], rw = rect[2] - rect[0] + 1, rh = rect[3] - rect[1] + 1;
    const bool lds = rect[2] >= 0 && rw * rh <= SPLAT_WIN;   // workgroup-uniform
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lds)   // rows by wave, columns by lane: no division
        for (int r = wave; r < rh; r += SPLAT_THREADS / 64)
            for (int c = lane; c < rw; c += 64) win[r * rw + c] = 0x7F800000u;   // +inf
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SPLAT_PER; ++k) {
        const unsigned long long key = gen | __float_as_uint(dist[k]);
        if (kind[k] == 1) {
            for (int ty = ty0[k]; ty <= ty1[k]; ++ty)
                for (int tx = tx0[k]; tx <= tx1[k]; ++tx) {
                    if (lds) {
                        if (!(b.diag & 2)) atomicMin(&win[(ty - ry0) * rw + (tx - rx0)], __float_as_uint(dist[k]));
                    } else beam_min(ts + ty * b.tiles_x + tx, key, b.diag);
                }
        } else if (kind[k] == 2) {
            for (int sy = ty0[k] >> 3; sy <= ty1[k] >> 3; ++sy)
                for (int sx = tx0[k] >> 3; sx <= tx1[k] >> 3; ++sx)
                    beam_min(ts + b.super_off + sy * b.super_x + sx, key, b.diag);
        } else if (kind[k] == 3) {
            beam_min(ts + b.global_off, key, b.diag);
        }
    }
    __syncthreads();
    if (lds)
        for (int r = wave; r < rh; r += SPLAT_THREADS / 64)
            for (int c = lane; c < rw; c += 64) {
                const uint32_t v = win[r * rw + c];
                if (v != 0x7F800000u) beam_min(ts + (ry0 + r) * b.tiles_x + rx0 + c, gen | v, b.diag);
            }
}

hipError_t launch_beam_splat(const BeamParams &b, hipStream_t stream) {
    if (b.n_boxes == 0) return hipSuccess;
    const uint32_t per_wg = SPLAT_THREADS * SPLAT_PER;
    hipLaunchKernelGGL(beam_splat_kernel, dim3((b.n_boxes + per_wg - 1u) / per_wg), dim3(SPLAT_THREADS), 0, stream, b);
    return hipGetLastError();
}

template <int MODE>
static hipError_t launch_shadows(const LaunchParams &p, hipStream_t stream) {
    const int bx = (p.width + 7) / 8, by = (p.local_rows + 7) / 8;
    const size_t lds = (size_t)p.slots * TILE * sizeof(uint2);
    if (p.fetch_all && !p.guard)
        hipLaunchKernelGGL((shadow_tile_kernel<MODE, true>), dim3((unsigned)(bx * by)), dim3(TILE), lds, stream, p, bx);
    else
        hipLaunchKernelGGL((shadow_tile_kernel<MODE>), dim3((unsigned)(bx * by)), dim3(TILE), lds, stream, p, bx);
    return hipGetLastError();
}

// svo_beam_starts (diagnostics): every pixel's primary-ray start under the launch's beam starts --
// beam_start of the ray render_tile_kernel traces (-inf without beam starts), band layout.
__global__ __launch_bounds__(256) void beam_starts_kernel(LaunchParams p) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)p.width * (size_t)p.local_rows) return;
    const int x = (int)(i % (size_t)p.width), lr = (int)(i / (size_t)p.width);
    const int gy = global_row(p, lr);
    Ray r;
    float org[3], dir[3];
    camera_ray(p.cam, p.width, p.height, x, gy, org, dir);
    setup_ray(org, dir, r);
    FRay f;
    to_fray(r, f);
    p.out.starts[i] = beam_start(p, f, x, gy);
}

hipError_t launch_render(const LaunchParams &p, int stack_mode, hipStream_t stream, hipEvent_t primary_start,
                         hipEvent_t primary_end) {
    // primary_start / primary_end (nullable): events around the primary-ray kernel only
    if (p.out.starts) {
        const size_t n = (size_t)p.width * (size_t)p.local_rows;
        hipLaunchKernelGGL(beam_starts_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, p);
        return hipGetLastError();
    }
    const bool count = p.out.fetches != nullptr;
    hipError_t e = hipSuccess;
    if (primary_start && (e = hipEventRecord(primary_start, stream)) != hipSuccess) return e;
    if (stack_mode == 0)
        e = count ? launch_variant<0, true>(p, stream) : launch_variant<0, false>(p, stream);
    else
        e = count ? launch_variant<1, true>(p, stream) : launch_variant<1, false>(p, stream);
    if (e != hipSuccess) return e;
    if (primary_end && (e = hipEventRecord(primary_end, stream)) != hipSuccess) return e;
    if (!count && p.shadows == 1 && (p.out.hits || p.out.compact))
        return stack_mode == 0 ? launch_shadows<0>(p, stream) : launch_shadows<1>(p, stream);
    if (!count && p.shadows == 3 && (p.out.hits || p.out.compact) && p.out.hitmask) {
        // compacted shadow pass: the hit list in the scratch whose head the primary filled
        if ((e = launch_pack<true>(nullptr, p.width, p.local_rows, p.out.hitmask, stream)) != hipSuccess) return e;
        const int n = ((p.width + 7) / 8) * ((p.local_rows + 7) / 8);
        const SparseLayout L = sparse_layout(n, p.width * p.local_rows, 4);
        const uint8_t *base = reinterpret_cast<const uint8_t *>(p.out.hitmask);
        const uint32_t *list = reinterpret_cast<const uint32_t *>(base + L.rgb);
        const uint32_t *cnt = reinterpret_cast<const uint32_t *>(base + L.offsets) + n;
        const size_t lds = (size_t)p.slots * TILE * sizeof(uint2);
        const dim3 grid((unsigned)(((size_t)p.width * (size_t)p.local_rows + TILE - 1) / TILE));
        LaunchParams q = p;
        q.out.hitmask = nullptr;
        if (stack_mode == 0) {
            if (p.fetch_all && !p.guard) hipLaunchKernelGGL((shadow_list_kernel<0, true>), grid, dim3(TILE), lds, stream, q, list, cnt);
            else hipLaunchKernelGGL((shadow_list_kernel<0>), grid, dim3(TILE), lds, stream, q, list, cnt);
        } else {
            if (p.fetch_all && !p.guard) hipLaunchKernelGGL((shadow_list_kernel<1, true>), grid, dim3(TILE), lds, stream, q, list, cnt);
            else hipLaunchKernelGGL((shadow_list_kernel<1>), grid, dim3(TILE), lds, stream, q, list, cnt);
        }
        return hipGetLastError();
    }
    return hipSuccess;
}

}  // namespace svo
