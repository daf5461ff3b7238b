// svo_rt.hip -- MI355X (gfx950) sparse-voxel-octree primary-ray caster.
//
// C-ABI plugin (include/svo_rt.h) replacing the reference's Unity host driver
// RaytracingMaster.cs + the HLSL compute kernel RaytraceCompute.compute /
// NVIDIASVO.compute / AttachmentLookup.compute (reference repo paths).
//
// Device data layout (DESIGN.md "Data layout in HBM"):
//   nodes : uint2[N]  .x = valid8 << 8 | nonleaf8,  .y = absolute index of the
//           first non-leaf child.  One 8-byte load per descriptor fetch.  The
//           reference's 16-bit RELATIVE pointer (NaiveCreator.cs:164-165) is
//           resolved to absolute at upload, so pools deeper than 16-bit
//           pointers allow use the same kernel.
//   att   : uint2[N]  .x = colorA565 | colorB565 << 16, .y = choices16 | normal16 << 16
//           (NaiveCreator.cs:189-191), one 8-byte load per hit.
//
// Numerics: compiled with -ffp-contract=off and correctly rounded f32 div/sqrt
// so every expression rounds exactly as the strict-IEEE oracle (oracle/).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "svo_rt.h"
#include "svo_traverse.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

#define HIP_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess)                                                          \
            return fail(SVO_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

struct Upload {
    size_t offset, count;
    int depth;
    bool external;   // has child links outside its own range (sub-SVO linking)
    bool tree;       // every node reached once from the upload's first node (no sharing, no cycles)
};

}  // namespace

struct svo_ctx {
    int device = 0;
    size_t capacity = 0;
    size_t n_nodes = 0;
    uint2 *d_nodes = nullptr;
    uint2 *d_att = nullptr;
    int32_t *d_stage = nullptr;   // staging for V1 descriptor conversion
    size_t stage_cap = 0;
    hipStream_t stream = nullptr;
    svo::Camera cam{};
    bool cam_set = false;
    std::vector<Upload> uploads;
    int depth = 0;
    bool depth_exact = false;        // see recompute_depth
    // host-path output scratch
    void *d_out_hits = nullptr;
    void *d_out_rgba = nullptr;
    size_t out_cap_px = 0;
    uint32_t *d_counter = nullptr;   // persistent-kernel work counter (16 B, zeroed per launch)
    int num_cus = 256;
    int kernel = 0;                  // 0 = tile (default), 1 = persistent; env SVO_KERNEL=tile|persistent
    int refill_at = 40;              // env SVO_REFILL
    int blocks_per_cu = 8;           // env SVO_BLOCKS_PER_CU
    int xcd_remap = 2;               // env SVO_XCD_REMAP: 2 interleaved column strips (default), 1 row bands, 0 off
    int strip_w = 1;                 // env SVO_STRIP_W: tile columns per strip (xcd_remap 2)
    int flat = 4;                    // env SVO_FLAT: 4 lean V2 (default), 3 lean, 1 flat, 0 branchy
    int block = 64;                  // env SVO_BLOCK (64 | 256)
    uint32_t options = 0;            // svo_set_options
    // SVO_OPT_KERNEL_TIMING: event pairs around the primary kernel of each launch
    std::vector<std::pair<hipEvent_t, hipEvent_t>> timing_events;   // recorded, not yet read
    std::vector<std::pair<hipEvent_t, hipEvent_t>> timing_free;     // reusable
    uint32_t *d_wave_log = nullptr;  // diagnostics: env SVO_WAVE_LOG=<file> (tile kernel, SVO_FLAT=3)
    size_t wave_log_cap = 0;
    // Cost-ordered tile dispatch: every launch records each 8x8 tile's trip
    // count; the order kernel, enqueued right behind it, turns them into the
    // heaviest-first dispatch order of the next launch at the same geometry.
    int tile_order = 1;              // env SVO_TILE_ORDER=0 disables
    int prio = 1;                    // env SVO_PRIO=0: no issue priority by cost class
    int shadow_order_enabled = 1;    // env SVO_SHADOW_ORDER=0: shadow tiles in plain strip order
    int fetch_all = -1;              // env SVO_FETCH_ALL=0|1 (default: by pool size, see launch)
    int fused_shadows = 1;           // env SVO_FUSED_SHADOWS=0: shadow rays as a second launch
    int order_every = 8;             // env SVO_ORDER_EVERY: rebuild the order every k-th launch (~20 us one-CU kernel)
    unsigned long long order_launches = 0;
    uint16_t *d_tile_cost = nullptr;
    uint32_t *d_tile_order = nullptr;
    uint16_t *d_shadow_cost = nullptr;   // the shadow pass's own costs and order
    uint32_t *d_shadow_order = nullptr;
    long long shadow_order_key = -1;
    unsigned long long shadow_launches = 0;
    size_t tile_cap = 0;
    long long order_key = -1;        // geometry d_tile_order was built for (-1: none)
    hipStream_t order_stream = nullptr;   // stream of the last order kernel (a launch elsewhere syncs it first)
    bool order_pending = false;
};

namespace {

// V1 (relative, int32) -> device node (absolute, uint2).  NaiveCreator.cs:184-187.
__global__ void convert_v1_kernel(const int32_t *__restrict__ desc, uint2 *__restrict__ nodes,
                                  size_t n, uint32_t base) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t cd = (uint32_t)desc[i];
    uint32_t self = base + (uint32_t)i;
    uint2 o;
    o.x = cd & 0xFFFFu;
    o.y = cd ? self + (cd >> 16) : 0u;   // node == 0 <=> descriptor word == 0 (HLSL re-fetch test)
    nodes[base + i] = o;
}

// Host-side level walk: validates every non-leaf child index and returns the
// number of descriptor levels reachable from the upload's first node.
int walk_depth(const uint32_t *lo, const uint32_t *first, size_t n, size_t base, size_t pool_n,
               int *depth_out, bool *external_out, bool *tree_out, std::string *err) {
    *tree_out = true;
    std::vector<uint8_t> seen(n, 0);
    std::vector<uint32_t> cur{0}, nxt;
    int depth = 0;
    bool external = false;
    if (n == 0) { *depth_out = 0; *external_out = false; return 0; }
    seen[0] = 1;
    while (!cur.empty()) {
        ++depth;
        if (depth > 22) { *err = "node pool deeper than 22 levels (s_max = 23)"; return -1; }
        nxt.clear();
        for (uint32_t li : cur) {
            uint32_t m = lo[li] & 0xFFu;
            uint32_t f = first[li];
            int rank = 0;
            for (int c = 0; c < 8; ++c) {
                if (!((m >> c) & 1u)) continue;
                uint64_t child = (uint64_t)f + (uint64_t)rank++;
                if (child >= pool_n) {
                    *err = "child pointer of node " + std::to_string(base + li) + " -> " +
                           std::to_string(child) + " outside the pool (" + std::to_string(pool_n) + ")";
                    return -1;
                }
                if (child < base || child >= base + n) { external = true; continue; }
                uint32_t cl = (uint32_t)(child - base);
                if (seen[cl]) { *tree_out = false; continue; }   // shared subtrees are legal (DAG)
                seen[cl] = 1;
                nxt.push_back(cl);
            }
        }
        cur.swap(nxt);
    }
    *depth_out = depth;
    *external_out = external;
    return 0;
}

void recompute_depth(svo_ctx *ctx) {
    int root_depth = 0, other = 0;
    bool ext = false;
    for (const Upload &u : ctx->uploads) {
        if (u.offset == 0) root_depth = std::max(root_depth, u.depth);
        else other = std::max(other, u.depth);
        ext = ext || u.external;
    }
    ctx->depth = root_depth + (ext ? other : 0);
    if (ctx->depth > 22) ctx->depth = 22;
    // A single self-contained tree at offset 0: every descent path has at most
    // `depth` levels, so the traversal stack cannot overflow while parents are
    // exact (the kernel may then drop its overflow guard).
    ctx->depth_exact = ctx->uploads.size() == 1 && ctx->uploads[0].offset == 0 && !ctx->uploads[0].external &&
                       ctx->uploads[0].tree && ctx->depth <= 22 && root_depth == ctx->depth;
}

int record_upload(svo_ctx *ctx, const uint32_t *lo, const uint32_t *first, size_t n, size_t base) {
    std::string err;
    int depth = 0;
    bool ext = false, tree = true;
    size_t pool_n = std::max(ctx->n_nodes, base + n);
    if (walk_depth(lo, first, n, base, pool_n, &depth, &ext, &tree, &err) != 0) return fail(SVO_ERR_FORMAT, err);
    ctx->uploads.erase(std::remove_if(ctx->uploads.begin(), ctx->uploads.end(),
                                      [&](const Upload &u) { return u.offset == base; }),
                       ctx->uploads.end());
    ctx->uploads.push_back({base, n, depth, ext, tree});
    ctx->n_nodes = pool_n;
    recompute_depth(ctx);
    return SVO_OK;
}

int ensure_out(svo_ctx *ctx, size_t px) {
    if (px <= ctx->out_cap_px) return SVO_OK;
    if (ctx->d_out_hits) hipFree(ctx->d_out_hits);
    if (ctx->d_out_rgba) hipFree(ctx->d_out_rgba);
    ctx->d_out_hits = ctx->d_out_rgba = nullptr;
    ctx->out_cap_px = 0;
    HIP_TRY(hipMalloc(&ctx->d_out_hits, px * sizeof(svo_hit)));
    HIP_TRY(hipMalloc(&ctx->d_out_rgba, px * 4 * sizeof(float)));
    ctx->out_cap_px = px;
    return SVO_OK;
}

int band_rows_local(int height, const svo_band &b) {
    // rows y with (y / band_rows) % band_count == band_rank
    int rows = 0;
    for (int y0 = b.band_rank * b.band_rows; y0 < height; y0 += b.band_rows * b.band_count)
        rows += std::min(b.band_rows, height - y0);
    return rows;
}

int check_band(const svo_band *band, int height, svo_band *out) {
    svo_band b = band ? *band : svo_band{1, 0, 1};
    if (b.band_rows <= 0 || b.band_count <= 0 || b.band_rank < 0 || b.band_rank >= b.band_count)
        return fail(SVO_ERR_ARG, "invalid svo_band");
    if (b.band_count == 1) b.band_rows = height > 0 ? height : 1;
    *out = b;
    return SVO_OK;
}

int launch(svo_ctx *ctx, int width, int height, int stack_mode, const svo_band *band,
           void *d_rgba, void *d_hits, uint32_t *d_fetch, hipStream_t stream) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (width <= 0 || height <= 0) return fail(SVO_ERR_ARG, "width/height must be positive");
    if (stack_mode != SVO_STACK_HLSL && stack_mode != SVO_STACK_EXACT)
        return fail(SVO_ERR_ARG, "unknown stack mode");
    if (ctx->n_nodes == 0) return fail(SVO_ERR_STATE, "no node pool uploaded (svo_set_buffer)");
    if (!ctx->cam_set) return fail(SVO_ERR_STATE, "camera not set (svo_set_camera)");
    svo_band b;
    int rc = check_band(band, height, &b);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(ctx->device));
    svo::LaunchParams p;
    p.nodes = ctx->d_nodes;
    p.att = ctx->d_att;
    p.n_nodes = (uint32_t)std::min<size_t>(ctx->n_nodes, 0xFFFFFFFFu);
    p.cam = ctx->cam;
    p.width = width;
    p.height = height;
    p.band_rows = b.band_rows;
    p.band_rank = b.band_rank;
    p.band_count = b.band_count;
    p.local_rows = band_rows_local(height, b);
    p.slots = std::max(ctx->depth - 1, 1);
    // guard: stack-overflow test + HLSL parent round trip, needed unless the
    // pool is one tree of known depth whose parent indices are exact in f32
    // (and the lean loop's 32-bit node byte offsets need fewer than 2^29 nodes)
    p.guard = !ctx->depth_exact || (stack_mode == 0 && ctx->n_nodes > ((size_t)1 << 24)) ||
              ctx->n_nodes >= ((size_t)1 << 29);
    // unpredicated node loads pay off on pools below 2^24 nodes (C2, C3: 5-9 %) and
    // cost 6-12 % on the 25 M / 100 M-node C4 / C5 pools (svo_kernel.hip trace_lean)
    p.fetch_all = ctx->fetch_all >= 0 ? ctx->fetch_all : (ctx->n_nodes < ((size_t)1 << 24) ? 1 : 0);
    p.hits = reinterpret_cast<svo::Hit *>(d_hits);
    p.rgba = reinterpret_cast<float4 *>(d_rgba);
    p.fetches = d_fetch;
    p.refill_at = ctx->refill_at;
    p.blocks_per_cu = ctx->blocks_per_cu;
    p.xcd_remap = ctx->xcd_remap;
    p.strip_w = ctx->strip_w;
    if (p.xcd_remap == 2 && (ctx->block != 64 || ((width + 7) / 8) % (8 * p.strip_w) != 0)) p.xcd_remap = 0;
    p.flat = ctx->flat;
    p.block = ctx->block;
    p.shadows = (ctx->options & SVO_OPT_SHADOW_RAYS) ? 1 : 0;
    // fused shadow pass: the 64-thread lean V2 tile kernel with cost ordering (env SVO_FUSED_SHADOWS=0: two passes)
    if (p.shadows && ctx->fused_shadows && ctx->kernel == 0 && ctx->block == 64 && ctx->flat == 4) p.shadows = 2;
    if (p.local_rows == 0) return SVO_OK;
    if (p.shadows == 1 && !p.hits && !p.fetches) {   // the second shadow pass reads the primary hit records
        int rc2 = ensure_out(ctx, (size_t)p.local_rows * (size_t)width);
        if (rc2) return rc2;
        p.hits = reinterpret_cast<svo::Hit *>(ctx->d_out_hits);
    }
    p.wave_log = nullptr;
    p.tile_order = nullptr;
    p.tile_cost = nullptr;
    p.shadow_order = nullptr;
    p.shadow_cost = nullptr;
    p.prio = ctx->prio;
    const bool ordered = ctx->tile_order && ctx->kernel == 0 && ctx->flat >= 3 && ctx->block == 64 && !p.fetches;
    const int n_tiles = ((width + 7) / 8) * ((p.local_rows + 7) / 8);
    long long key = -1;
    if (ordered) {
        key = ((long long)width << 40) ^ ((long long)p.local_rows << 16) ^ ((long long)b.band_rows << 8) ^
              (long long)b.band_rank ^ ((long long)b.band_count << 4) ^ ((long long)ctx->xcd_remap << 60) ^ ((long long)ctx->strip_w << 52);
        if (ctx->tile_cap < (size_t)n_tiles) {
            HIP_TRY(hipDeviceSynchronize());   // a pending launch may still use the old buffers
            if (ctx->d_tile_cost) hipFree(ctx->d_tile_cost);
            if (ctx->d_tile_order) hipFree(ctx->d_tile_order);
            if (ctx->d_shadow_cost) hipFree(ctx->d_shadow_cost);
            if (ctx->d_shadow_order) hipFree(ctx->d_shadow_order);
            ctx->d_tile_cost = nullptr;
            ctx->d_tile_order = nullptr;
            ctx->d_shadow_cost = nullptr;
            ctx->d_shadow_order = nullptr;
            ctx->tile_cap = 0;
            ctx->order_key = -1;
            ctx->shadow_order_key = -1;
            const size_t cap = svo::order_cost_capacity(n_tiles);
            HIP_TRY(hipMalloc(&ctx->d_tile_cost, cap * sizeof(uint16_t)));
            HIP_TRY(hipMemset(ctx->d_tile_cost, 0, cap * sizeof(uint16_t)));
            HIP_TRY(hipMalloc(&ctx->d_tile_order, ((size_t)n_tiles + 36) * sizeof(uint32_t)));
            HIP_TRY(hipMalloc(&ctx->d_shadow_cost, cap * sizeof(uint16_t)));
            HIP_TRY(hipMemset(ctx->d_shadow_cost, 0, cap * sizeof(uint16_t)));
            HIP_TRY(hipMalloc(&ctx->d_shadow_order, ((size_t)n_tiles + 36) * sizeof(uint32_t)));
            ctx->tile_cap = (size_t)n_tiles;
        }
        if (const char *f = std::getenv("SVO_ORDER_FILE")) {   // experiments: a fixed host-made order
            if (ctx->order_key != key) {
                std::vector<uint32_t> h((size_t)n_tiles + 4, 0u);
                FILE *fp = std::fopen(f, "rb");
                if (!fp) return fail(SVO_ERR_ARG, std::string("SVO_ORDER_FILE: cannot open ") + f);
                const size_t got = std::fread(h.data(), sizeof(uint32_t), (size_t)n_tiles, fp);
                std::fclose(fp);
                if (got != (size_t)n_tiles) return fail(SVO_ERR_ARG, "SVO_ORDER_FILE: short file");
                std::vector<uint8_t> seen((size_t)n_tiles, 0);
                for (size_t i = 0; i < (size_t)n_tiles; ++i) {
                    if (h[i] >= (uint32_t)n_tiles || seen[h[i]]) return fail(SVO_ERR_ARG, "SVO_ORDER_FILE: not a permutation");
                    seen[h[i]] = 1;
                }
                HIP_TRY(hipMemcpy(ctx->d_tile_order, h.data(), h.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
                ctx->order_key = key;
            }
            p.tile_order = ctx->d_tile_order;
            p.tile_cost = nullptr;
        } else {
            p.tile_order = ctx->order_key == key ? ctx->d_tile_order : nullptr;
        }
        if (!std::getenv("SVO_ORDER_FILE")) p.tile_cost = ctx->d_tile_cost;
        if (p.shadows == 1 && ctx->shadow_order_enabled) {
            p.shadow_cost = ctx->d_shadow_cost;
            p.shadow_order = ctx->shadow_order_key == key ? ctx->d_shadow_order : nullptr;
        }
    }
    const char *log_path = std::getenv("SVO_WAVE_LOG");
    const size_t n_wave = (size_t)((width + 15) / 16) * (size_t)((p.local_rows + 15) / 16) * 4;   // >= any tiling
    if (log_path && !p.fetches) {
        if (ctx->wave_log_cap < n_wave) {
            if (ctx->d_wave_log) hipFree(ctx->d_wave_log);
            ctx->d_wave_log = nullptr;
            ctx->wave_log_cap = 0;
            HIP_TRY(hipMalloc(&ctx->d_wave_log, n_wave * 32));
            ctx->wave_log_cap = n_wave;
        }
        HIP_TRY(hipMemset(ctx->d_wave_log, 0, n_wave * 32));
        p.wave_log = ctx->d_wave_log;
    }
    hipStream_t s = stream ? stream : ctx->stream;
    // the cost/order buffers are shared by all launches of the context: launches
    // on one stream are ordered; switching streams waits for the last order kernel
    if (p.tile_cost && ctx->order_pending && ctx->order_stream != s) {
        HIP_TRY(hipStreamSynchronize(ctx->order_stream));
        ctx->order_pending = false;
    }
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    if ((ctx->options & SVO_OPT_KERNEL_TIMING) && !p.fetches) {
        if (ctx->timing_free.empty()) {
            HIP_TRY(hipEventCreate(&ev0));
            if (hipEventCreate(&ev1) != hipSuccess) {
                hipEventDestroy(ev0);
                return fail(SVO_ERR_HIP, "hipEventCreate");
            }
        } else {
            ev0 = ctx->timing_free.back().first;
            ev1 = ctx->timing_free.back().second;
            ctx->timing_free.pop_back();
        }
        ctx->timing_events.emplace_back(ev0, ev1);
    }
    hipError_t e = svo::launch_render(p, stack_mode, s, ctx->kernel, ctx->d_counter, ctx->num_cus, ev0, ev1);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("render launch: ") + hipGetErrorString(e));
    const bool refresh = p.tile_cost && (ctx->order_key != key || ctx->order_launches++ % ctx->order_every == 0);
    if (refresh) {   // the next launch at this geometry dispatches the heaviest tiles first
        e = p.xcd_remap == 2 ? svo::launch_order_strips(ctx->d_tile_cost, ctx->d_tile_order, n_tiles, (width + 7) / 8,
                                                        p.strip_w, s)
                                : svo::launch_order_tiles(ctx->d_tile_cost, ctx->d_tile_order, n_tiles, s);
        if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("tile order launch: ") + hipGetErrorString(e));
        ctx->order_stream = s;
        ctx->order_pending = true;
        ctx->order_key = key;
    }
    if (p.shadow_cost && (ctx->shadow_order_key != key || ctx->shadow_launches++ % ctx->order_every == 0)) {
        e = p.xcd_remap == 2 ? svo::launch_order_strips(ctx->d_shadow_cost, ctx->d_shadow_order, n_tiles, (width + 7) / 8,
                                                        p.strip_w, s)
                             : svo::launch_order_tiles(ctx->d_shadow_cost, ctx->d_shadow_order, n_tiles, s);
        if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("shadow order launch: ") + hipGetErrorString(e));
        ctx->order_stream = s;
        ctx->order_pending = true;
        ctx->shadow_order_key = key;
    }
    if (p.wave_log) {   // blocking dump of the last launch's per-wave record
        HIP_TRY(hipStreamSynchronize(s));
        std::vector<uint32_t> h(n_wave * 8);
        HIP_TRY(hipMemcpy(h.data(), ctx->d_wave_log, n_wave * 32, hipMemcpyDeviceToHost));
        if (FILE *f = std::fopen(log_path, "wb")) {
            std::fwrite(h.data(), 32, n_wave, f);
            std::fclose(f);
        }
    }
    return SVO_OK;
}

}  // namespace

extern "C" {

int svo_abi_version(void) { return 1; }

const char *svo_last_error(void) { return g_last_error.c_str(); }

int svo_create(int device, size_t capacity_nodes, svo_ctx **out) {
    if (!out) return fail(SVO_ERR_ARG, "out is null");
    *out = nullptr;
    if (capacity_nodes == 0 || capacity_nodes > (size_t)0xFFFFFFFFu)
        return fail(SVO_ERR_ARG, "capacity_nodes must be in [1, 2^32)");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(SVO_ERR_ARG, "device index out of range");
    HIP_TRY(hipSetDevice(device));
    svo_ctx *ctx = new (std::nothrow) svo_ctx();
    if (!ctx) return fail(SVO_ERR_ARG, "out of host memory");
    ctx->device = device;
    ctx->capacity = capacity_nodes;
    hipError_t e = hipMalloc(&ctx->d_nodes, capacity_nodes * sizeof(uint2));
    if (e == hipSuccess) e = hipMalloc(&ctx->d_att, capacity_nodes * sizeof(uint2));
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&ctx->d_counter, 256);
    if (e == hipSuccess) e = hipMemset(ctx->d_counter, 0, 256);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&ctx->num_cus, hipDeviceAttributeMultiprocessorCount, device);
    if (const char *k = std::getenv("SVO_KERNEL")) ctx->kernel = std::strcmp(k, "persistent") == 0 ? 1 : 0;
    if (const char *k = std::getenv("SVO_REFILL")) ctx->refill_at = std::max(0, std::min(64, std::atoi(k)));
    if (const char *k = std::getenv("SVO_XCD_REMAP")) ctx->xcd_remap = std::max(0, std::min(2, std::atoi(k)));
    if (const char *k = std::getenv("SVO_STRIP_W")) ctx->strip_w = std::max(1, std::atoi(k));
    if (const char *k = std::getenv("SVO_FLAT")) ctx->flat = std::max(0, std::min(4, std::atoi(k)));
    if (const char *k = std::getenv("SVO_TILE_ORDER")) ctx->tile_order = std::atoi(k) != 0;
    if (const char *k = std::getenv("SVO_PRIO")) ctx->prio = std::atoi(k) != 0;
    if (const char *k = std::getenv("SVO_SHADOW_ORDER")) ctx->shadow_order_enabled = std::atoi(k) != 0;
    if (const char *k = std::getenv("SVO_FETCH_ALL")) ctx->fetch_all = std::atoi(k) != 0 ? 1 : 0;
    if (const char *k = std::getenv("SVO_FUSED_SHADOWS")) ctx->fused_shadows = std::atoi(k) != 0;
    if (const char *k = std::getenv("SVO_ORDER_EVERY")) ctx->order_every = std::max(1, std::atoi(k));
    if (const char *k = std::getenv("SVO_BLOCK")) { const int b = std::atoi(k); ctx->block = (b == 256 || b == 128) ? b : 64; }
    if (const char *k = std::getenv("SVO_BLOCKS_PER_CU")) ctx->blocks_per_cu = std::max(1, std::min(64, std::atoi(k)));
    if (e != hipSuccess) {
        svo_destroy(ctx);
        return fail(SVO_ERR_HIP, std::string("svo_create: ") + hipGetErrorString(e));
    }
    *out = ctx;
    return SVO_OK;
}

int svo_set_buffer(svo_ctx *ctx, const int32_t *desc, size_t n_desc, const uint32_t *att,
                   size_t n_att, size_t dst_offset) {
    if (!ctx || (!desc && n_desc) || (!att && n_att)) return fail(SVO_ERR_ARG, "null argument");
    if (dst_offset + n_desc > ctx->capacity || 2 * dst_offset + n_att > 2 * ctx->capacity)
        return fail(SVO_ERR_CAPACITY, "upload exceeds node-pool capacity");
    if (n_att != 2 * n_desc) return fail(SVO_ERR_ARG, "attachments must hold 2 words per descriptor");
    if (n_desc == 0) return SVO_OK;
    // host-side validation walk on the absolute view
    std::vector<uint32_t> lo(n_desc), first(n_desc);
    for (size_t i = 0; i < n_desc; ++i) {
        uint32_t cd = (uint32_t)desc[i];
        lo[i] = cd & 0xFFFFu;
        first[i] = cd ? (uint32_t)(dst_offset + i) + (cd >> 16) : 0u;
    }
    int rc = record_upload(ctx, lo.data(), first.data(), n_desc, dst_offset);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(ctx->device));
    if (n_desc > ctx->stage_cap) {
        if (ctx->d_stage) hipFree(ctx->d_stage);
        ctx->d_stage = nullptr;
        ctx->stage_cap = 0;
        HIP_TRY(hipMalloc(&ctx->d_stage, n_desc * sizeof(int32_t)));
        ctx->stage_cap = n_desc;
    }
    HIP_TRY(hipMemcpyAsync(ctx->d_stage, desc, n_desc * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
    unsigned blocks = (unsigned)((n_desc + 255) / 256);
    hipLaunchKernelGGL(convert_v1_kernel, dim3(blocks), dim3(256), 0, ctx->stream, ctx->d_stage,
                       ctx->d_nodes, n_desc, (uint32_t)dst_offset);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(ctx->d_att + dst_offset, att, n_att * sizeof(uint32_t), hipMemcpyHostToDevice,
                           ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return SVO_OK;
}

int svo_set_buffer_v2(svo_ctx *ctx, const uint64_t *nodes, size_t n_nodes, const uint32_t *att,
                      size_t n_att, size_t dst_offset) {
    if (!ctx || (!nodes && n_nodes) || (!att && n_att)) return fail(SVO_ERR_ARG, "null argument");
    if (dst_offset + n_nodes > ctx->capacity) return fail(SVO_ERR_CAPACITY, "upload exceeds node-pool capacity");
    if (n_att != 2 * n_nodes) return fail(SVO_ERR_ARG, "attachments must hold 2 words per node");
    if (n_nodes == 0) return SVO_OK;
    std::vector<uint32_t> lo(n_nodes), first(n_nodes);
    for (size_t i = 0; i < n_nodes; ++i) {
        lo[i] = (uint32_t)nodes[i];
        first[i] = (uint32_t)(nodes[i] >> 32);
        if (lo[i] > 0xFFFFu) return fail(SVO_ERR_FORMAT, "v2 node low word must only hold the two masks");
    }
    int rc = record_upload(ctx, lo.data(), first.data(), n_nodes, dst_offset);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(ctx->device));
    static_assert(sizeof(uint2) == sizeof(uint64_t), "node layout");
    HIP_TRY(hipMemcpyAsync(ctx->d_nodes + dst_offset, nodes, n_nodes * sizeof(uint64_t), hipMemcpyHostToDevice,
                           ctx->stream));
    HIP_TRY(hipMemcpyAsync(ctx->d_att + dst_offset, att, n_att * sizeof(uint32_t), hipMemcpyHostToDevice,
                           ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return SVO_OK;
}

int svo_set_camera(svo_ctx *ctx, const float c2w[16], const float inv_proj[16], float px_off_x,
                   float px_off_y, const float light[4]) {
    if (!ctx || !c2w || !inv_proj || !light) return fail(SVO_ERR_ARG, "null argument");
    std::memcpy(ctx->cam.c2w, c2w, sizeof(ctx->cam.c2w));
    std::memcpy(ctx->cam.inv_proj, inv_proj, sizeof(ctx->cam.inv_proj));
    ctx->cam.px_off[0] = px_off_x;
    ctx->cam.px_off[1] = px_off_y;
    std::memcpy(ctx->cam.light, light, sizeof(ctx->cam.light));
    ctx->cam_set = true;
    return SVO_OK;
}

int svo_render(svo_ctx *ctx, int width, int height, int stack_mode, float *rgba_out, svo_hit *hits_out) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (width <= 0 || height <= 0) return fail(SVO_ERR_ARG, "width/height must be positive");
    size_t px = (size_t)width * (size_t)height;
    HIP_TRY(hipSetDevice(ctx->device));
    int rc = ensure_out(ctx, px);
    if (rc) return rc;
    rc = launch(ctx, width, height, stack_mode, nullptr, rgba_out ? ctx->d_out_rgba : nullptr,
                hits_out ? ctx->d_out_hits : nullptr, nullptr, ctx->stream);
    if (rc) return rc;
    if (hits_out)
        HIP_TRY(hipMemcpyAsync(hits_out, ctx->d_out_hits, px * sizeof(svo_hit), hipMemcpyDeviceToHost, ctx->stream));
    if (rgba_out)
        HIP_TRY(hipMemcpyAsync(rgba_out, ctx->d_out_rgba, px * 4 * sizeof(float), hipMemcpyDeviceToHost,
                               ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return SVO_OK;
}

int svo_render_device(svo_ctx *ctx, int width, int height, int stack_mode, const svo_band *band, void *d_rgba,
                      void *d_hits, void *stream) {
    return launch(ctx, width, height, stack_mode, band, d_rgba, d_hits, nullptr,
                  reinterpret_cast<hipStream_t>(stream));
}

int svo_count_fetches(svo_ctx *ctx, int width, int height, int stack_mode, const svo_band *band,
                      void *d_fetches, void *stream) {
    if (!d_fetches) return fail(SVO_ERR_ARG, "d_fetches is null");
    return launch(ctx, width, height, stack_mode, band, nullptr, nullptr,
                  reinterpret_cast<uint32_t *>(d_fetches), reinterpret_cast<hipStream_t>(stream));
}

int svo_set_options(svo_ctx *ctx, uint32_t options) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (options & ~(uint32_t)(SVO_OPT_SHADOW_RAYS | SVO_OPT_KERNEL_TIMING)) return fail(SVO_ERR_ARG, "unknown option bits");
    ctx->options = options;
    return SVO_OK;
}

int svo_kernel_time(svo_ctx *ctx, double *mean_ms, uint64_t *launches) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    HIP_TRY(hipSetDevice(ctx->device));
    double sum = 0.0;
    uint64_t n = 0;
    hipError_t err = hipSuccess;
    for (auto &ev : ctx->timing_events) {
        float ms = 0.0f;
        if (err == hipSuccess) err = hipEventSynchronize(ev.second);
        if (err == hipSuccess) err = hipEventElapsedTime(&ms, ev.first, ev.second);
        if (err == hipSuccess) { sum += ms; ++n; }
        ctx->timing_free.push_back(ev);
    }
    ctx->timing_events.clear();
    if (err != hipSuccess) return fail(SVO_ERR_HIP, std::string("svo_kernel_time: ") + hipGetErrorString(err));
    if (mean_ms) *mean_ms = n ? sum / (double)n : 0.0;
    if (launches) *launches = n;
    return SVO_OK;
}

int svo_get_info(svo_ctx *ctx, size_t *n_nodes, int *max_depth, int *device) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (n_nodes) *n_nodes = ctx->n_nodes;
    if (max_depth) *max_depth = ctx->depth;
    if (device) *device = ctx->device;
    return SVO_OK;
}

int svo_accumulate(svo_ctx *ctx, void *d_accum, const void *d_sample, size_t n_px, uint32_t sample,
                   void *stream) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (n_px == 0) return SVO_OK;
    if (!d_accum || !d_sample) return fail(SVO_ERR_ARG, "null accumulation or sample buffer");
    if (((uintptr_t)d_accum | (uintptr_t)d_sample) & 15u) return fail(SVO_ERR_ARG, "buffers must be 16-byte aligned");
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    hipError_t e = svo::launch_accumulate(reinterpret_cast<float4 *>(d_accum), reinterpret_cast<const float4 *>(d_sample),
                                          n_px, sample, ctx->num_cus, s);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("accumulate launch: ") + hipGetErrorString(e));
    return SVO_OK;
}

int svo_synchronize(svo_ctx *ctx) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return SVO_OK;
}

int svo_destroy(svo_ctx *ctx) {
    if (!ctx) return SVO_OK;
    hipSetDevice(ctx->device);
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    if (ctx->d_nodes) hipFree(ctx->d_nodes);
    if (ctx->d_att) hipFree(ctx->d_att);
    if (ctx->d_stage) hipFree(ctx->d_stage);
    if (ctx->d_out_hits) hipFree(ctx->d_out_hits);
    if (ctx->d_out_rgba) hipFree(ctx->d_out_rgba);
    if (ctx->d_counter) hipFree(ctx->d_counter);
    if (ctx->d_shadow_cost) hipFree(ctx->d_shadow_cost);
    if (ctx->d_shadow_order) hipFree(ctx->d_shadow_order);
    for (auto &ev : ctx->timing_events) { hipEventDestroy(ev.first); hipEventDestroy(ev.second); }
    for (auto &ev : ctx->timing_free) { hipEventDestroy(ev.first); hipEventDestroy(ev.second); }
    if (ctx->d_wave_log) hipFree(ctx->d_wave_log);
    if (ctx->d_tile_cost) hipFree(ctx->d_tile_cost);
    if (ctx->d_tile_order) hipFree(ctx->d_tile_order);
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    delete ctx;
    return SVO_OK;
}

}  // extern "C"
