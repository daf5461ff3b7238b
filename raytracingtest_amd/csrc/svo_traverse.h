// svo_traverse.h -- per-pixel SVO primary-ray kernel for gfx950 (wave64).
//
// Restates, for the GPU, Assets/Shaders/RaytraceCompute.compute:143-168
// (CSMain), :129-141 (CreateCameraRay), :93-127 (Shade) and
// Assets/Shaders/NVIDIASVO.compute:12-198 (IntersectSVO, Laine & Karras 2010)
// of the reference.  Not a transcription of the HLSL dispatch: one wave64
// covers an 8x8 pixel tile, the traversal stack lives in LDS laid out
// [slot][lane] (conflict-free ds_write2_b32 / ds_read_b64), a node fetch is one
// 8-byte load, and the per-lane branch conditions are wave lane masks in SGPRs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

namespace svo {

constexpr int S_MAX = 23;          // NVIDIASVO.compute:2
constexpr int MAX_ITERS = 65536;   // safety net, identical in oracle/svo_oracle.c
constexpr int TILE = 64;           // one wave64 = one 8x8 pixel tile
constexpr int MAX_PARTS = 64;      // band parts one assemble launch reads (devices / ranks)
constexpr int WAVE_LOG_WORDS = 12;   // per-wave record of the SVO_WAVE_LOG diagnostics
constexpr int MAX_CYCLE = 256;     // bands per cycle of a weighted band deal (svo_band.cycle)
constexpr int MAX_SAMPLES = 8;     // jittered samples one svo_render_samples launch traces per tile
// XCD column strips are STRIP_K tile columns wide (svo_kernel.hip strip_col; compile-time knob
// -DSVO_STRIP_K for A/Bs: 2 and 3 within noise of 1, 5 and 6 +3 %, profiles/r03n_ab_strip_width.txt)
#ifdef SVO_STRIP_K
constexpr int STRIP_K = SVO_STRIP_K;
#else
constexpr int STRIP_K = 1;
#endif

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

// Every per-pixel output of one launch (device pointers, each nullable).  Index =
// local row * width + x (band layout) or global row * width + x (frame layout).
struct Outputs {
    Hit *hits;                 // svo_hit, 24 B
    float4 *rgba;              // Result (RGBA32F)
    uint32_t *rgba8;           // display RGBA8
    uint32_t *compact;         // svo_hit_compact: 3 words = the first 12 bytes of svo_hit
    float4 *position;          // bestHit.position (NVIDIASVO.compute:172-174), w = 0
    unsigned long long *voxel; // voxel key
    uint8_t *rgb8;             // display RGB, 3 bytes per pixel (the RGBA8 word's low bytes)
    unsigned long long *hitmask;   // per 8x8 tile of the render's rows (band-local tile index
                                   // (lr / 8) * tiles_x + x / 8): the wave's ballot of its hit lanes
    uint32_t *fetches;         // instrumented launch: descriptor fetches per ray
    float *starts;             // diagnostics (svo_beam_starts): each primary ray's beam start, nothing else
    int frame_layout;          // 1: index by global row (full-frame buffers)
    // one sample blended into an RGBA32F accumulation (svo_render_samples with S = 1: the one-sample
    // launch itself, AddShader's blend in its epilogue): accum = colour * acc_a + accum * acc_b,
    // and rgba8 / rgb8 then carry the BLENDED colour
    float4 *accum;
    float acc_a, acc_b;
};

struct LaunchParams {
    const uint2 *nodes;
    const uint2 *att;
    uint32_t n_nodes;     // pool size (index bound for fetches of HLSL-rounded parents)
    Camera cam;
    int width, height;
    int band_rows, band_rank, band_count, local_rows;
    // weighted deal (band_cycle > 0): this render's j-th band is band
    // (j / band_cnt) * band_cycle + band_pos[j % band_cnt]; 0 = round-robin
    int band_cycle, band_cnt;
    uint8_t band_pos[MAX_CYCLE];
    int slots;            // stack slots = depth - 1 (scales [23 - slots, 22])
    Outputs out;
    int xcd_remap;        // 2: interleaved XCD column strips, 0: raster
    int shadows;          // one shadow ray per primary hit: 1 = second pass (needs hits), 2 = fused into the primary
                          // launch, 3 = second pass over the compacted hit list (needs hits + out.hitmask scratch)
    uint32_t *wave_log;   // diagnostics (env SVO_WAVE_LOG): per wave {t0, t1, tile, XCC_ID | trips << 8,
                          //   loop cycles, push-only | advance-only trips << 16, fetch trips, pop trips,
                          //   wave entry, wave exit (after its stores), 2 spare} (WAVE_LOG_WORDS)
    // Cost-ordered dispatch: block b traces 8x8 tile tile_order[b] (null = b)
    // and records its wave trip count in tile_cost.
    const uint32_t *tile_order;   // n_tiles entries + 36 class boundaries
    uint16_t *tile_cost;
    int prio;                     // s_setprio by cost class (svo_config.issue_priority)
    int guard;                    // lean loop: stack-overflow test and HLSL parent round trip needed
    int fetch_all;                // lean loop (!guard): every lane loads its node every trip
    int lat;                      // latency form of the loop (trace_lat; !guard, primary rays only)
    // The same cost-ordered dispatch for the two-pass shadow form (its own costs and order).
    const uint32_t *shadow_order;
    uint16_t *shadow_cost;
    // Samples in flight (svo_render_samples): samples > 0 traces that many jittered samples of
    // every tile in ONE launch -- a workgroup per tile, wave k = sample k with pixel offset
    // sample_off[k] -- and blends them in order into accum (AddShader, _Sample = first + k:
    // dst = src * blend_a[k] + dst * blend_b[k]), then writes the blended frame's display words.
    int samples;
    float sample_off[MAX_SAMPLES][2];
    float blend_a[MAX_SAMPLES], blend_b[MAX_SAMPLES];
    float4 *accum;             // RGBA32F accumulation (out_index layout), read and written
    uint32_t *accum8;          // display RGBA8 of the blended pixels (nullable)
    uint8_t *accum_rgb8;       // the same as 3-byte RGB, the band payload (nullable)
    // Segmented heavy tiles (svo_kernel.hip render_seg_kernel; seg != 0 only with an order built
    // by launch_order_strips(..., seg_cap > 0)): an order entry t | code << 28 is part q of tile t
    // traced as K t-segments per ray (code 1 + q for K = 4, 5 + q for K = 8; lanes K r .. K r + K - 1
    // = ray r's segments); 0xFFFFFFFF is an empty slot.  seg_hint: per pixel (band-local lr * width
    // + x) two float4, the starts at fractions 1/8 .. 7/8 of the ray's last segmented trace (NaN:
    // none), rewritten by every such trace; part_cost: per tile SEG_KMAX entries, each part's
    // continuous-equivalent trips (the tile's tile_cost then holds SEG_COST_FLAG | K).
    // seg = the order's seg_cap (0: no segmented tiles), seg_kmax its largest K.
    int seg, seg_kmax;
    float4 *seg_hint;
    uint16_t *part_cost;
    uint32_t seg_scramble;     // tests (svo_config.seg_scramble): != 0 replaces every start by a hash of
                               // (pixel, this value) -- unordered, NaN, +-inf, outside the cube
    // Beam starts (null: none).  tile_start[ty * ts_tiles_x + tx] for the 8x8 tile
    // (tx, ty) of the FULL frame (global rows), tile_start[ts_super_off + sy * ts_super_x + sx] for
    // its 64x64 super tile and tile_start[ts_global_off]: the minimum is a lower bound of the
    // distance (SVO-space t) at which any primary ray through the tile, at any pixel offset in
    // [0, 1], can first hit a voxel (beam_splat_kernel).  A primary ray starts there, minus a
    // rounding margin, in trace_seg's exact skip form.
    // Entries are keys ~gen << 32 | distance bits (beam_splat_kernel); one of another generation
    // than ts_gen reads as +inf.
    const unsigned long long *tile_start;
    int ts_tiles_x, ts_super_x, ts_super_off, ts_global_off;
    uint32_t ts_gen;
};

constexpr int SEG_KMAX = 8;                 // segments per ray: 4 (a lane quad) or 8, by cost class
constexpr uint16_t SEG_COST_FLAG = 0x8000;  // tile_cost of a segmented tile (| its K): read part_cost
constexpr uint32_t SEG_EMPTY = 0xFFFFFFFFu; // order slot with nothing to trace

// Re-interleave the band parts of a split frame on the display device
// (svo_assemble_frame): part m holds the rows of bands b with b % n_parts == m,
// in increasing y, as 12-byte compact records (PART_COMPACT) or RGBA8 words
// (PART_RGBA8).  Compact parts are expanded into every requested output: the
// normal and the Result colour are rebuilt from the display device's own SVO
// replica and camera with the render kernel's arithmetic (bit-identical).
enum { PART_COMPACT = 0, PART_RGBA8 = 1, PART_RGB8 = 2, PART_SPARSE_RGB8 = 3 };
struct AssembleParams {
    const uint2 *att;
    uint32_t n_nodes;     // a parent outside the pool reads attachment words 0
    Camera cam;
    int width, height, band_rows, n_parts, part_format, skip_part;
    const void *parts[MAX_PARTS];
    // weighted deal (cycle > 0): band b belongs to part owner[b % cycle] and is that
    // part's band (b / cycle) * cnt[part] + idx[b % cycle]; 0 = round-robin
    int cycle;
    uint8_t owner[MAX_CYCLE], idx[MAX_CYCLE];
    int cnt[MAX_PARTS];
    // PART_SPARSE_RGB8: part m = [n_tiles[m] hit masks (u64)][n_tiles[m] + 1 tile offsets (u32)]
    // [3-byte RGB of the hit pixels, tile by tile, lanes in order] (svo_rt.h, svo_pack_hits)
    uint32_t n_tiles[MAX_PARTS];
    Outputs out;          // frame layout
};

// Order the tiles by recorded cost, most expensive class first, into `order`
// (one workgroup, no atomics), followed by the 4 cumulative class sizes
// (order must hold n_tiles + 4 entries).  Placement only: any order gives
// identical results.  `cost` must hold order_cost_capacity(n_tiles) entries (the tail
// beyond n_tiles is read, never used).  stats (nullable, 16 words, host-visible): the
// max [0] and sum [1] of the tiles' costs, [2..15] zero (launch_order_strips' layout).
hipError_t launch_order_tiles(const uint16_t *cost, uint32_t *order, int n_tiles, hipStream_t stream,
                              uint32_t *stats = nullptr);
size_t order_cost_capacity(int n_tiles);
// The same per XCD strip (xcd_remap 2): order must hold order_strips_entries(n_tiles, seg_cap)
// entries.  stats (nullable, 16 words, host-visible memory): per XCD x the max [2 x] and the
// sum [2 x + 1] of its tiles' costs.  seg_cap > 0: each XCD's tiles of cost >= half its
// heaviest (at most seg_cap of them, heaviest classes first) are listed as SEG_K quarter
// entries for render_seg_kernel, the lists padded to one length with SEG_EMPTY; a segmented
// tile's cost is the max of its part_cost entries.  The render grid is then
// order_strips_grid(n_tiles, seg_cap) workgroups.
// seg_kpack: the K of cost class c (>= 7/8, 3/4, 1/2, 1/4, 1/8 of the XCD's max, rest) in bits
// 4 c .. 4 c + 3: 0 = not segmented, 4 or 8.
hipError_t launch_order_strips(const uint16_t *cost, uint32_t *order, int n_tiles, int tiles_x, hipStream_t stream,
                               uint32_t *stats = nullptr, int seg_cap = 0, const uint16_t *part_cost = nullptr,
                               int seg_kpack = 0, int spread = 0);
// spread != 0: each tile is classed by the heaviest cost of its 3x3 neighbourhood (costs recorded a few
// frames before, while the camera moves); the stats stay those of the tiles themselves.
__host__ __device__ inline int seg_kmax_of(int kpack) {
    int m = 1;
    for (int c = 0; c < 6; ++c) {
        const int k = (kpack >> (4 * c)) & 15;
        m = k > m ? k : m;
    }
    return m;
}
inline int order_strips_grid(int n_tiles, int seg_cap, int kmax) { return n_tiles + 8 * (kmax - 1) * seg_cap; }
inline size_t order_strips_entries(int n_tiles, int seg_cap, int kmax = SEG_KMAX) {
    return (size_t)order_strips_grid(n_tiles, seg_cap, kmax) + 36;
}

// Beam starts of one launch: every box of the pool's splat list (the nodes at
// the splat depth and the leaves above it, svo_rt.hip build_beam_boxes) is projected onto the
// screen, and its distance from the camera min-ed into every 8x8 tile its projection touches
// (a 64x64 super tile or the one global word when it touches more than 32), as the key
// ~gen << 32 | distance bits: no fill pass, stale entries lose every min (tiles_x * tiles_y +
// super_x * super_y + 1 entries; gen > 0, the buffer all-ones when first allocated).
struct BeamParams {
    const uint2 *boxes;    // (x | y << 16, z | depth << 16): box [1 + i 2^-depth, 1 + (i + 1) 2^-depth]^3
    uint32_t n_boxes;
    unsigned long long *tile_start;
    uint32_t gen;
    uint32_t diag;         // diagnostics (env SVO_BEAM_DIAG): 1 no global atomics, 2 no LDS window either
    int tiles_x, tiles_y, super_x, super_y, super_off, global_off;
    int width, height;
    float org[3];          // camera origin in SVO space, bit-identical to the render's
    float minv[9];         // row-major inverse of M: unnormalised ray direction = M (fx, fy, 1), fx, fy
                           // continuous pixel coordinates (pixel x, offset o: fx = x + o)
    float minv_abs[3];     // sum_k |minv[r][k]| per row r, rounded up: a box's half extents in q-space
    float plane[4][3];     // the view frustum's side planes through the camera, normals pointing in
};
hipError_t launch_beam_splat(const BeamParams &b, hipStream_t stream);

// Progressive accumulation (AddShader blend) of an RGBA32F sample frame.
hipError_t launch_accumulate(float4 *dst, const float4 *src, size_t n_px, uint32_t sample, int num_cus,
                             hipStream_t stream);

hipError_t launch_assemble(const AssembleParams &a, hipStream_t stream);

// Sparse hit payload of a band (svo_rt.h layout): `part` holds the n tile masks; write the
// tile offsets (exclusive scan of the masks' popcounts, count last) and pack the 3-byte RGB
// of every hit pixel of the band's dense `rgb8` behind them.  Three launches.
hipError_t launch_pack_hits(const uint8_t *rgb8, int width, int local_rows, void *part, hipStream_t stream);
// Scratch bytes of the compacted shadow pass (shadows == 3): hit masks, tile offsets, count,
// the hit pixels' band-local indices and the scan's scratch; LaunchParams.out.hitmask points at it.
size_t shadow_list_bytes(int width, int local_rows);

// Copy `bytes` (a multiple of 16) of device memory into mapped pinned host memory with a kernel.
hipError_t launch_push_host(const void *src, void *dst_mapped, size_t bytes, int blocks, hipStream_t stream);

// Display RGB, 3 bytes per pixel, of an RGBA32F frame (svo_render_progressive_async, RGB8).
hipError_t launch_pack_rgb8(const float4 *src, uint8_t *dst, size_t n_px, int num_cus, hipStream_t stream);

// Display RGBA8 words of an RGBA32F frame (svo_render_progressive).
hipError_t launch_pack_rgba8(const float4 *src, uint32_t *dst, size_t n_px, int num_cus, hipStream_t stream);

hipError_t launch_render(const LaunchParams &p, int stack_mode, hipStream_t stream, hipEvent_t primary_start = nullptr,
                         hipEvent_t primary_end = nullptr);

}  // namespace svo
