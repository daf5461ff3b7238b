// svo_traverse.h -- per-pixel SVO primary-ray kernel for gfx950 (wave64).
//
// Restates, for the GPU, Assets/Shaders/RaytraceCompute.compute:143-168
// (CSMain), :129-141 (CreateCameraRay), :93-127 (Shade) and
// Assets/Shaders/NVIDIASVO.compute:12-198 (IntersectSVO, Laine & Karras 2010)
// of the reference.  Not a transcription of the HLSL dispatch: one wave64
// covers an 8x8 pixel tile, the traversal stack lives in LDS laid out
// [slot][lane] (conflict-free ds_read_b64 / ds_write_b64), a node fetch is one
// 8-byte load, and never-written stack entries read as zero through a
// per-lane written-slot bit mask instead of a per-ray LDS clear.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

namespace svo {

constexpr int S_MAX = 23;          // NVIDIASVO.compute:2
constexpr int MAX_ITERS = 65536;   // safety net, identical in oracle/svo_oracle.c
constexpr int BLOCK = 256;         // 4 waves, 16x16 pixels

struct Camera {
    float c2w[16];        // Unity Matrix4x4, column-major
    float inv_proj[16];
    float px_off[2];
    float light[4];
};

struct Hit {              // == svo_hit
    uint32_t parent;
    uint8_t hit_idx;
    uint8_t hit_scale;
    uint16_t flags;
    float t;
    float nx, ny, nz;
};
static_assert(sizeof(Hit) == 24, "hit record layout");

struct LaunchParams {
    const uint2 *nodes;
    const uint2 *att;
    uint32_t n_nodes;     // pool size (index bound for fetches of HLSL-rounded parents)
    Camera cam;
    int width, height;
    int band_rows, band_rank, band_count, local_rows;
    int slots;            // stack slots = depth - 1 (scales [23 - slots, 22])
    Hit *hits;            // nullable
    float4 *rgba;         // nullable
    uint32_t *fetches;    // nullable (instrumented launch)
    int refill_at;        // persistent kernel: refill idle lanes when fewer than this still trace
    int blocks_per_cu;    // persistent kernel: grid = CUs x this
    int xcd_remap;        // tile kernel: give each XCD a contiguous screen band
    int flat;             // 1: branch-flattened iteration (default), 0: branchy reference form
    int block;            // tile kernel workgroup size: 64 (one 8x8 wave) or 256 (16x16 pixels)
    int shadows;          // one shadow ray per primary hit: 1 = second pass (needs hits), 2 = fused into the primary launch
    uint32_t *wave_log;   // diagnostics (env SVO_WAVE_LOG): per wave {t0, t1, HW_ID, XCC_ID | trips << 8,
                          //   loop cycles, fetch-wait cycles, fetch trips, pop trips} (instrumented loop)
    // Cost-ordered dispatch (64-thread tile kernel): block b traces 8x8 tile
    // tile_order[b] (null = b) and records its wave trip count in tile_cost.
    const uint32_t *tile_order;   // n_tiles entries + 4 class boundaries
    uint16_t *tile_cost;
    int prio;                     // s_setprio by cost class (env SVO_PRIO)
    int guard;                    // lean loop: stack-overflow test and HLSL parent round trip needed
    int fetch_all;                // lean loop (!guard): every lane loads its node every trip
    int strip_w;                  // xcd_remap 2: tile columns per super-column
    // The same cost-ordered dispatch for the shadow pass (its own costs and order).
    const uint32_t *shadow_order;
    uint16_t *shadow_cost;
};

// Order the tiles by recorded cost, most expensive class first, into `order`
// (one workgroup, no atomics), followed by the 4 cumulative class sizes
// (order must hold n_tiles + 4 entries).  Placement only: any order gives
// identical results.  `cost` must hold order_cost_capacity(n_tiles) entries (the tail
// beyond n_tiles is read, never used).
hipError_t launch_order_tiles(const uint16_t *cost, uint32_t *order, int n_tiles, hipStream_t stream);
size_t order_cost_capacity(int n_tiles);
// The same per XCD strip (xcd_remap 2): order must hold n_tiles + 36 entries.
hipError_t launch_order_strips(const uint16_t *cost, uint32_t *order, int n_tiles, int tiles_x, int strip_w,
                               hipStream_t stream);

// Progressive accumulation (AddShader blend) of an RGBA32F sample frame.
hipError_t launch_accumulate(float4 *dst, const float4 *src, size_t n_px, uint32_t sample, int num_cus,
                             hipStream_t stream);

// kernel: 0 = tile (one lane per pixel), 1 = persistent (wave-level ray refill).
// counter: 16-byte device work counter (persistent kernel), num_cus: CU count.
hipError_t launch_render(const LaunchParams &p, int stack_mode, hipStream_t stream, int kernel,
                         uint32_t *counter, int num_cus, hipEvent_t primary_start = nullptr,
                         hipEvent_t primary_end = nullptr);

}  // namespace svo
