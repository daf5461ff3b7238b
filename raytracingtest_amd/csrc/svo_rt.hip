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
// Multi-device contexts (svo_create_multi): one node-pool replica per device;
// a frame is split into band_rows-row bands dealt round-robin to the devices;
// the display device (devices[0]) renders its bands straight into the caller's
// frame, every other device into a band-contiguous payload (12-byte compact
// records, or RGBA8 for display-only frames), and one assemble kernel on the
// display device pulls the payloads over xGMI (peer access) and rebuilds the
// frame's rows.  All of it is enqueued on streams; nothing blocks the host.
//
// Numerics: compiled with -ffp-contract=off and correctly rounded f32 div/sqrt
// so every expression rounds exactly as the strict-IEEE oracle (oracle/).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
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
    // beam starts: the splat list of a self-contained tree at offset 0, built from the
    // host arrays at upload (null: none; a pool of several uploads is walked on the device copy)
    std::shared_ptr<const std::vector<uint2>> boxes;
    int boxes_back;      // the config's beam_back it was built with
    std::shared_ptr<const std::vector<uint2>> boxes_held;   // ... and the held view's (beam_back_held)
    int boxes_held_back;
};

// The device copy of a splat list (a context holds two: a moving camera's and a held view's)
struct DevBoxes {
    uint2 *d = nullptr;
    size_t cap = 0;
    uint32_t n = 0;
    uint64_t id = 0;   // made from the list with this id (0: none)
};

enum { STAGE_KERNEL = 0, STAGE_ASSEMBLE = 1, N_STAGES = 2 };

// The tile-order cache key: the exact geometry (and deal) an order was built for.
struct Geo {
    int width = -1, local_rows = -1, rows = -1, rank = -1, count = -1, xcd = -1, n_tiles = -1;
    int seg = 0;    // the order's seg_cap (segmented heavy tiles, svo_kernel.hip render_seg_kernel) ...
    int kpack = 0;  // ... and the K of each cost class (launch_order_strips' seg_kpack)
    uint64_t deal = 0;
    bool operator==(const Geo &o) const {
        return width == o.width && local_rows == o.local_rows && rows == o.rows && rank == o.rank &&
               count == o.count && xcd == o.xcd && n_tiles == o.n_tiles && seg == o.seg && kpack == o.kpack &&
               deal == o.deal;
    }
    bool operator!=(const Geo &o) const { return !(*this == o); }
};

// Cost-ordered dispatch state of the renders on one stream: every launch records each
// 8x8 tile's trip count; the order kernel, enqueued right behind it, turns them into
// the heaviest-first dispatch order of the next launch at the same geometry.  One set
// per stream (up to MAX_SCHED streams), so renders on different streams -- frames in
// flight -- share nothing mutable and run concurrently.
constexpr int MAX_SCHED = 4;
struct Sched {
    hipStream_t stream = nullptr;
    bool used = false;
    bool idle = false;               // nothing enqueued on `stream` since the last svo_synchronize
    unsigned long long last_use = 0;
    hipEvent_t done = nullptr;       // eviction: recorded on this stream when another takes the set over
    // The dispatch order is built OFF the render stream (round 5): after launch n
    // the order kernel runs on `side` (behind an event on the render stream) from the costs launch n
    // wrote, into one of two order buffers, and the first launch to dispatch in it is n + 2 -- so
    // launch n + 1 never waits for it.  Launch n writes its costs into buffer n % 2 (the build
    // after launch n reads them while launch n + 1 writes the other one); a launch waits on the
    // build event of a build it follows by >= 2 launches once, before its kernel, and only if the
    // host has not already seen that build complete (a held view: never).
    uint16_t *cost_buf[2] = {};
    uint16_t *part_buf[2] = {};          // segmented tiles: per tile and part (SEG_KMAX x cap)
    uint32_t *order_buf[2] = {};
    hipStream_t side = nullptr;
    hipEvent_t render_done = nullptr;    // recorded on the render stream behind a launch a build follows
    hipEvent_t build_ev[2] = {};
    long long build_at[2] = {-1, -1};    // the launch after which buffer i's order was built (-1: none)
    bool build_seen[2] = {};             // the render stream already waits for it (or it completed)
    Geo build_key[2];
    int next_buf = 0;
    uint16_t *shadow_cost = nullptr;   // the two-pass shadow form's own costs and order
    uint32_t *shadow_order = nullptr;
    size_t cap = 0;
    size_t order_cap = 0;              // order_buf entries allocated
    float4 *seg_hint = nullptr;        // segmented tiles: per pixel the segment starts (svo_traverse.h)
    size_t hint_cap = 0;
    unsigned long long *tile_start = nullptr;   // beam starts of this stream's launches (svo_traverse.h)
    size_t ts_cap = 0;
    uint32_t ts_gen = 0;               // the generation of the last launch's keys ...
    unsigned long long ts_view = ~0ull; // ... splatted for this view, splat list and frame size
    uint64_t ts_boxes = 0;
    int ts_w = -1, ts_h = -1;
    bool held_splat = false;           // this launch re-splatted a held view finer: its costs are new
    Geo order_key;                   // the newest build's key (width -1: none)
    Geo shadow_key;
    unsigned long long launches = 0, shadow_launches = 0;
    unsigned long long built_view = 0;   // the context's view generation the order was built under
    unsigned long long view_prev = ~0ull;   // the view generation of this stream's last launch ...
    float off_prev[2] = {-1.0f, -1.0f};     // ... and its pixel offset
    unsigned long long built_cost = ~0ull;  // the context's cost generation the order was built under
    unsigned long long last_build = 0;      // the launch count at the last order build
    int built_mode = -1;                 // shadows | stack_mode << 2 of the costs it was built from
    // loop-form choice (see launch): a ring of the last STATS_RING order builds' statistics
    // (host-visible: per XCD max / sum of the tile costs the order kernel saw, 16 words each),
    // each read only once its build has completed (its event); the decision it gives is kept
    // with the geometry, view and render mode it was measured at.  A ring rather than one slot:
    // while the camera moves every launch rebuilds the order, and one slot would be re-recorded
    // before the host ever found it complete.
    static constexpr int STATS_RING = 4;
    uint32_t *stats = nullptr;           // STATS_RING x 16 words
    hipEvent_t stats_ev[STATS_RING] = {};
    bool stats_pending[STATS_RING] = {};
    Geo stats_key[STATS_RING];
    unsigned long long stats_view[STATS_RING] = {};
    int stats_mode[STATS_RING] = {};
    int stats_head = 0;                  // the slot the next build writes
    bool relayout_pending = false;       // a launch ran in an order of another class layout (see launch)
    int lat_cache = 0;                   // the decision of the last completed build ...
    bool lat_short = false;              // ... and whether its heaviest tile's chain was short
    bool lat_thin = false;               // ... and whether its work was thin against that chain (svo_config.seg_table_thin)
    Geo lat_key;                         // ... made at this geometry / view / mode (width -1: none)
    unsigned long long lat_view = 0;
    int lat_mode = -1;
};

struct Peer {                       // one per member of a multi-device context (index 0: the display device)
    void *buf[2] = {nullptr, nullptr};   // band payload, double-buffered across frames
    size_t cap_bytes = 0;
    hipEvent_t rendered[2] = {nullptr, nullptr};
    void *dense = nullptr;               // sparse payload: the band's dense RGB before the pack
    size_t dense_cap = 0;
    float4 *accum = nullptr;             // svo_render_samples: this member's band accumulation (band layout)
    int accum_w = 0, accum_rows = -1;
    uint64_t accum_deal = 0;             // the band deal its rows belong to
    int link = SVO_LINK_SELF;            // how the payload reaches the display device (svo_get_member_link)
    int native_link = SVO_LINK_SELF;     // ... without svo_config.peer_copy (what svo_create_multi found)
    void *local[2] = {nullptr, nullptr}; // SVO_LINK_COPY: the payload's copy on the display device
    size_t local_cap = 0;
};


// Host threads that move svo_render's outputs from the plugin's pinned staging into the
// caller's (pageable) arrays, chunk by chunk, while the DMA of the next chunk runs.
class CopyPool {
  public:
    explicit CopyPool(int n) {
        for (int i = 0; i < n; ++i) th_.emplace_back([this] { run(); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> l(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int size() const { return (int)th_.size(); }
    void submit(void *dst, const void *src, size_t n) {
        {
            std::lock_guard<std::mutex> l(m_);
            q_.push_back(Job{static_cast<char *>(dst), static_cast<const char *>(src), n});
            ++pending_;
        }
        cv_.notify_one();
    }
    void wait() {
        std::unique_lock<std::mutex> l(m_);
        done_.wait(l, [this] { return pending_ == 0; });
    }

  private:
    struct Job { char *dst; const char *src; size_t n; };
    void run() {
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> l(m_);
                cv_.wait(l, [this] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;
                j = q_.front();
                q_.pop_front();
            }
            std::memcpy(j.dst, j.src, j.n);
            {
                std::lock_guard<std::mutex> l(m_);
                if (--pending_ == 0) done_.notify_all();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    std::deque<Job> q_;
    size_t pending_ = 0;
    bool stop_ = false;
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
    bool depth_exact = false;        // see recompute_pool
    // the splat list of the whole pool (beam starts; null: none) and its unique id
    std::shared_ptr<const std::vector<uint2>> pool_boxes;
    uint64_t pool_boxes_id = 0;
    int pool_boxes_back = -1;
    // ... and the finer one a held view re-splats with (beam_back_held; the same list when equal)
    std::shared_ptr<const std::vector<uint2>> pool_boxes_held;
    uint64_t pool_boxes_held_id = 0;
    // diagnostics (the library's only environment switches, read once at svo_create):
    // SVO_DEBUG bit 0 the loop-form / class-table decision trace, bit 1 the order each launch
    // takes; SVO_WAVE_LOG=<file> the per-wave record; SVO_BEAM_DIAG the splat's timing variants
    int debug = 0;
    std::string wave_log_path;
    uint32_t beam_diag = 0;
    // host-path output scratch
    void *d_out_hits = nullptr;
    void *d_shadow_list = nullptr;   // compacted shadow pass: hit masks, offsets, hit list (svo_kernel.hip)
    size_t shadow_list_cap = 0;
    void *d_out_rgba = nullptr;
    size_t out_cap_px = 0;
    // svo_render: pinned staging of the outputs, its per-chunk events, and the host copy threads
    void *h_stage = nullptr;
    size_t h_stage_cap = 0;
    static constexpr int STAGE_CHUNKS = 16;
    hipEvent_t stage_ev[STAGE_CHUNKS] = {};
    std::unique_ptr<CopyPool> copy_pool;
    // svo_render_progressive: the accumulated frame (RGBA32F, zeroed on a size
    // change) and its RGBA8 display words
    float4 *d_accum = nullptr;
    uint32_t *d_accum8 = nullptr;
    int accum_w = 0, accum_h = 0;
    // svo_render_progressive_async: the accumulated frame's RGBA8 words packed into one of
    // PIN_SLOTS device slots and copied on copy_stream into plugin-owned pinned host memory
    // (the D2H of frame k overlaps the render of frame k + 1)
    static constexpr int PIN_SLOTS = 3;
    uint32_t *h_pin[PIN_SLOTS] = {};
    uint32_t *d_pin[PIN_SLOTS] = {};
    hipEvent_t pin_packed[PIN_SLOTS] = {}, pin_copied[PIN_SLOTS] = {};
    bool pin_used[PIN_SLOTS] = {};
    hipStream_t copy_stream = nullptr;
    int pin_w = 0, pin_h = 0, pin_next = 0;
    int pin_format = SVO_PIXELS_RGBA8;   // the slots' pixel format (svo_render_progressive_async)
    int pin_push = 0;                    // svo_config.readback: 0 hipMemcpyAsync (DMA), 1 a kernel writes the
                                         // mapped pinned buffer, 2 the DMA split over two copy streams
    int host_copy_threads = 0;           // svo_config.host_copy_threads (0: half the hardware threads)
    hipStream_t copy_stream2 = nullptr;
    hipEvent_t pin_copied2[PIN_SLOTS] = {};
    unsigned long long pin_frames = 0;   // frames enqueued since the slots were (re)allocated
    int num_cus = 256;
    size_t lds_per_block = 160 * 1024;   // hipDeviceProp.sharedMemPerBlock
    int xcd_remap = 2;               // svo_config.xcd_strips: 2 interleaved column strips (default), 0 raster
    uint32_t options = 0;            // svo_set_options
    // SVO_OPT_KERNEL_TIMING: event pairs around the primary kernel / the assemble kernel
    std::vector<std::pair<hipEvent_t, hipEvent_t>> timing_events[N_STAGES];   // recorded, not yet read
    std::vector<std::pair<hipEvent_t, hipEvent_t>> timing_free;               // reusable
    uint32_t *d_wave_log = nullptr;  // diagnostics: env SVO_WAVE_LOG=<file>
    size_t wave_log_cap = 0;
    // cost-ordered tile dispatch (svo_rt.hip Sched): switches and per-stream state
    int tile_order = 1;              // svo_config.tile_order (0: strip order)
    int prio = 1;                    // svo_config.issue_priority 0: no issue priority by cost class
    int shadow_order_enabled = 1;    // svo_config.shadow_order 0: shadow tiles in plain strip order
    int fetch_all = -1;              // svo_config.fetch_all 0|1 (default: by pool size, see launch)
    int fused_shadows = 1;           // svo_config.shadow_form 1: shadow rays as a second launch
    int shadow_compact = 0;          // svo_config.shadow_form 2: that launch over the compacted hit list
    int lat_mode = -1;               // svo_config.loop_form: 0 never, 1 always, unset: by the last launch's costs (see launch)
    int seg_mode = 1;                // svo_config.segments 0: never trace heavy tiles as segmented rays (see launch)
    int seg_kpack_lat = 0x444;       // svo_config.seg_table_latency: the K of each cost class (nibble c: class c, >= 7/8,
                                     // 3/4, 1/2, 1/4, 1/8 of the max, rest; 0 none, 4 or 8) in a latency-bound launch
    int seg_kpack_issue = 0x4;       // svo_config.seg_table_issue: the same in an issue-bound launch
    int seg_kpack_thin = 0x888;      // svo_config.seg_table_thin: ... and in a latency-bound launch whose summed trips
    float thin_ratio = 0.083f;       // are below svo_config.seg_thin_ratio x slots x its heaviest tile's: C3 8-way bands
                                     // (flyover 0.045, Main.unity 0.079) and the overview frame (0.063) run faster
                                     // with every heavy class in eighths, the flyover 4-way band (0.087) with 444
                                     // (profiles/r05_thin_ab.json)
    int seg_cap = 96;                // svo_config.seg_cap: at most this many segmented tiles per XCD
    int seg_all = 0;                 // svo_config.seg_all 4|8 (tests): every tile segmented with that K
    uint32_t seg_scramble = 0;       // svo_config.seg_scramble (tests): arbitrary segment starts
    uint32_t seg_launches = 0;
    int beam = 1;                    // svo_config.beam: beam starts
    int beam_back = 2;               // svo_config.beam_back: a new view's splat, this many levels above the leaves
    int beam_back_held = 0;          // svo_config.beam_back_held: a held view's (-1: beam_back)
    DevBoxes dev_boxes[2];           // device copies of pool_boxes / pool_boxes_held
    unsigned long long *count_ts = nullptr;   // beam starts of an instrumented launch (SVO_OPT_COUNT_BEAM)
    size_t count_ts_cap = 0;
    uint32_t count_ts_gen = 0;
    float lat_ratio = 0.3f;          // svo_config.lat_ratio: the auto rule's threshold ...
    // the stored segment starts are those of the pixel's ray in the previous launch: of another
    // sub-pixel ray after a jittered launch, of another view while the camera moves.  Such a launch
    // splits its segments evenly from the beam start instead (segments past an earlier segment's
    // record end early; trace_seg): C3 one-sample route 94.6 against 97.9 us (overview 84.3 / 88.8),
    // a slow pan 91.2 / 93.0 us (profiles/r05_stale_starts.txt).  1: the stored starts, 0 (jittered
    // launches only): no segments
    int seg_move = 2;                // svo_config.seg_move: a launch at a new view
    int seg_jitter = 2;              // svo_config.seg_jitter: a jittered launch (the one-sample samples route)
    int spread = 1;                  // svo_config.move_spread 0: a moving camera's order classes tiles by their own costs only
    int relayout = 1;                // svo_config.relayout 0: keep an order built from costs of another class layout
    int seg_min_chain = 160;         // svo_config.seg_min_chain: a latency-bound launch whose heaviest tile costs fewer
                                     // trips takes the latency form, unsegmented, without beam starts
    float seg_ratio = 0.28f;         // svo_config.seg_ratio: ... and the same with beam starts (class table only)
    int move_every = 4;              // svo_config.move_every: while the camera moves every launch, rebuild the
                                     // order only every k-th launch (see launch; 1 = at every new view).
                                     // C3 pan: 118.8 us per frame at 1, 110.7 at 4, 111.9 at 8
    int order_every = 32;            // svo_config.order_every: rebuild the order every k-th launch (and after
                                     // every camera move or change of render mode)
    unsigned long long view_gen = 0; // bumped when svo_set_camera changes the matrices
    unsigned long long cost_gen = 0; // bumped by whatever else changes the tiles' costs: a new pixel
                                     // offset or light, an upload
    Sched sched[MAX_SCHED];
    unsigned long long sched_clock = 0;
    // The one piece of state renders on different streams still share: the host-path /
    // two-pass-shadow scratch outputs.  A render that uses them waits for the previous
    // such render's stream (an event recorded at the switch; no host sync).
    hipStream_t scratch_stream = nullptr;
    bool scratch_valid = false;
    hipEvent_t switch_event = nullptr;
    // multi-device context (svo_create_multi); empty for a single-device one
    std::vector<svo_ctx *> members;
    std::vector<Peer> peers;
    hipEvent_t gathered[2] = {nullptr, nullptr};
    bool gathered_used[2] = {false, false};
    int parity = 0;
    int band_rows = 8;
    int deal_cycle = 0;                  // svo_set_band_deal: weighted deal over the members (0: round-robin)
    int sparse_payload = 0;              // svo_config.sparse_payload: display-only frames travel as sparse parts
    int peer_copy = 0;                   // svo_config.peer_copy: every member's payload copied, not pulled
    uint8_t deal_owner[svo::MAX_CYCLE] = {};
    uint64_t samples_deal = 0;           // the deal of the last svo_render_samples (band accumulations' rows)
    bool samples_deal_set = false;
};

namespace {

bool is_multi(const svo_ctx *ctx) { return !ctx->members.empty(); }

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

// Make stream s wait for the work the previous scratch user enqueued on another stream.
int order_scratch(svo_ctx *ctx, hipStream_t s) {
    if (ctx->scratch_valid && ctx->scratch_stream != s) {
        // the previous stream is alive: a caller keeps its streams until svo_forget_stream /
        // svo_synchronize / svo_destroy (svo_rt.h)
        if (!ctx->switch_event) HIP_TRY(hipEventCreateWithFlags(&ctx->switch_event, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(ctx->switch_event, ctx->scratch_stream));
        HIP_TRY(hipStreamWaitEvent(s, ctx->switch_event, 0));
    }
    ctx->scratch_stream = s;
    ctx->scratch_valid = true;
    return SVO_OK;
}

// Forget every order build of the set (the buffers stay; the caller has synchronised).
void reset_builds(Sched &q) {
    for (int i = 0; i < 2; ++i) {
        q.build_at[i] = -1;
        q.build_seen[i] = false;
        q.build_key[i] = Geo();
    }
    q.order_key = q.shadow_key = Geo();
}

void free_sched(Sched &q) {
    for (int i = 0; i < 2; ++i) {
        if (q.cost_buf[i]) hipFree(q.cost_buf[i]);
        if (q.part_buf[i]) hipFree(q.part_buf[i]);
        if (q.order_buf[i]) hipFree(q.order_buf[i]);
        q.cost_buf[i] = q.part_buf[i] = nullptr;
        q.order_buf[i] = nullptr;
    }
    if (q.shadow_cost) hipFree(q.shadow_cost);
    if (q.shadow_order) hipFree(q.shadow_order);
    q.shadow_cost = nullptr;
    q.shadow_order = nullptr;
    q.cap = 0;
    q.order_cap = 0;
    reset_builds(q);
}

// The scheduling state of stream s: its own set, or a free one, or the least recently
// used one -- taken over only after the stream that used it has finished its renders.
int sched_for(svo_ctx *ctx, hipStream_t s, Sched **out) {
    Sched *pick = nullptr;
    for (Sched &q : ctx->sched)
        if (q.used && q.stream == s) pick = &q;
    if (!pick) {
        for (Sched &q : ctx->sched)
            if (!q.used) { pick = &q; break; }
    }
    if (!pick) {
        pick = &ctx->sched[0];
        for (Sched &q : ctx->sched)
            if (q.last_use < pick->last_use) pick = &q;
        // s takes over the set only after the renders the evicted stream was given: an event
        // recorded on that stream NOW stands behind all of them (host order = stream order).
        // Recorded here, at the rare eviction, not behind every launch: a marker packet
        // between two renders of one stream cost ~2-3 us of GPU time per frame.  The evicted
        // stream is alive: callers keep a stream until svo_forget_stream (svo_rt.h).
        // After svo_synchronize nothing is pending there and the stream may be gone (svo_rt.h):
        // record nothing on it.
        if (!pick->idle) {
            if (!pick->done) HIP_TRY(hipEventCreateWithFlags(&pick->done, hipEventDisableTiming));
            HIP_TRY(hipEventRecord(pick->done, pick->stream));
            HIP_TRY(hipStreamWaitEvent(s, pick->done, 0));
        }
        if (pick->side) HIP_TRY(hipStreamSynchronize(pick->side));   // its order builds (rare: an eviction)
        reset_builds(*pick);   // built for another stream's frames
        pick->launches = pick->shadow_launches = 0;
        pick->view_prev = ~0ull;
        pick->built_cost = ~0ull;
        pick->last_build = 0;
        for (int r = 0; r < Sched::STATS_RING; ++r) pick->stats_pending[r] = false;
        pick->lat_key = Geo();
        pick->lat_mode = -1;
    }
    pick->stream = s;
    pick->used = true;
    pick->idle = false;
    pick->last_use = ++ctx->sched_clock;
    *out = pick;
    return SVO_OK;
}

// Host-side level walk: validates every non-leaf child index and returns the
// number of descriptor levels reachable from the upload's first node.  A
// breadth-first walk with a seen set: exact for a tree; for a DAG it is the
// shallowest depth, so such pools are traversed with the full stack
// (recompute_pool walks the whole pool instead).
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
                           std::to_string(child) + " outside the node-pool capacity (" + std::to_string(pool_n) + ")";
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

// The splat list of a tree: every box a primary ray can first hit a voxel in, at
// a fixed depth ds = depth - back -- the non-leaf nodes at ds and the leaves above it -- as
// (x | y << 16, z | depth << 16), box [1 + i 2^-depth, 1 + (i + 1) 2^-depth]^3 in SVO space.
// Child c of a node (bit c of its masks, NVIDIASVO.compute:83-94 with slot 7 - c) takes the upper
// half on axis k iff bit k of c is set; its node is first + (non-leaf children before it).
std::shared_ptr<const std::vector<uint2>> build_beam_boxes(const uint32_t *lo, const uint32_t *first, size_t n,
                                                           int depth, int back) {
    const int ds = std::min(depth - back, 16);   // 16-bit coordinates
    if (ds < 1 || n == 0) return nullptr;
    auto out = std::make_shared<std::vector<uint2>>();
    struct Item { uint32_t node, x, y, z; };
    std::vector<Item> cur{{0u, 0u, 0u, 0u}}, nxt;
    // a pool whose subtrees are shared (linked sub-SVOs) expands them once per position; past this many
    // boxes the walk stops descending and lists the nodes it reached as boxes of their own (coarser,
    // still a lower bound: every voxel of the pool lies in one of the listed boxes)
    constexpr size_t BUDGET = (size_t)1 << 23;
    for (int d = 0; d < ds && !cur.empty(); ++d) {
        nxt.clear();
        for (const Item &it : cur) {
            const uint32_t m = lo[it.node] & 0xFFu, v = (lo[it.node] >> 8) & 0xFFu;
            uint32_t rank = 0;
            const bool descend = nxt.size() + out->size() < BUDGET;
            for (uint32_t c = 0; c < 8; ++c) {
                const bool inner = (m >> c) & 1u;
                const uint32_t child = inner ? first[it.node] + rank++ : 0u;
                if (!((v >> c) & 1u)) continue;
                const uint32_t x = 2 * it.x + (c & 1u), y = 2 * it.y + ((c >> 1) & 1u), z = 2 * it.z + ((c >> 2) & 1u);
                if (inner && d + 1 < ds && descend) {
                    if (child < n) nxt.push_back({child, x, y, z});
                } else {
                    out->push_back(make_uint2(x | (y << 16), z | ((uint32_t)(d + 1) << 16)));
                }
            }
        }
        cur.swap(nxt);
    }
    if (out->size() >= 0xFFFFFFFFull) return nullptr;
    // Morton order (coordinates at 16 bits): a splat workgroup's boxes then cover a compact patch
    // of the screen (svo_kernel.hip beam_splat_kernel's LDS window)
    auto spread = [](uint64_t v) {
        v &= 0xFFFFull;
        v = (v | (v << 16)) & 0x0000FF0000FFull;
        v = (v | (v << 8)) & 0x00F00F00F00Full;
        v = (v | (v << 4)) & 0x0C30C30C30C3ull;
        v = (v | (v << 2)) & 0x249249249249ull;
        return v;
    };
    auto morton = [&](const uint2 &b) {
        const int sh = 16 - (int)(b.y >> 16);
        return spread((uint64_t)(b.x & 0xFFFFu) << sh) | spread((uint64_t)(b.x >> 16) << sh) << 1 |
               spread((uint64_t)(b.y & 0xFFFFu) << sh) << 2;
    };
    std::vector<std::pair<uint64_t, uint2>> keyed(out->size());
    for (size_t i = 0; i < out->size(); ++i) keyed[i] = {morton((*out)[i]), (*out)[i]};
    std::sort(keyed.begin(), keyed.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
    for (size_t i = 0; i < keyed.size(); ++i) (*out)[i] = keyed[i].second;
    return out;
}

// The splat depth of a held view (svo_config.beam_back_held; -1: a new view's)
int held_back(const svo_ctx *ctx) { return ctx->beam_back_held < 0 ? ctx->beam_back : ctx->beam_back_held; }

int validate_upload(svo_ctx *ctx, const uint32_t *lo, const uint32_t *first, size_t n, size_t base, Upload *out) {
    std::string err;
    int depth = 0;
    bool ext = false, tree = true;
    // links may point past what is uploaded so far (the reference uploads the trunk
    // before the sub-SVO it links to, Clipmap.cs:158,168): any index inside the
    // capacity is legal; the pool is zero-filled at svo_create, so a link into a
    // region not uploaded yet reads empty descriptors
    if (walk_depth(lo, first, n, base, ctx->capacity, &depth, &ext, &tree, &err) != 0) return fail(SVO_ERR_FORMAT, err);
    *out = Upload{base, n, depth, ext, tree, nullptr, -1, nullptr, -1};
    if (base == 0 && tree && !ext && ctx->beam) {   // the common case: the splat lists from the host arrays
        const int hb = held_back(ctx);
        out->boxes = build_beam_boxes(lo, first, n, depth, ctx->beam_back);
        out->boxes_back = ctx->beam_back;
        out->boxes_held = hb == ctx->beam_back ? out->boxes : build_beam_boxes(lo, first, n, depth, hb);
        out->boxes_held_back = hb;
    }
    return SVO_OK;
}

uint64_t next_boxes_id() {
    static std::atomic<uint64_t> next_id{0};
    return ++next_id;
}

// The pool's traversal facts and its splat list, after every upload and beam config change.
//  * One self-contained tree uploaded at offset 0 (the reference's SetSVOBuffer(data)): its own
//    upload walk; the splat list built from its host arrays then.
//  * Anything else -- a trunk whose leaves link to sub-SVOs uploaded elsewhere (Clipmap.cs:153-169
//    via SetSVOBuffer(data, offset), RaytracingMaster.cs:118-135), several uploads, a shared
//    subtree: the pool as the device holds it is walked from the root (node 0) across the uploads.
//    A child index past the uploaded nodes reads as the zero-filled empty descriptor (no
//    children).  If every node is reached once, the pool is one tree: its depth is exact (the
//    stack needs depth - 1 slots and cannot overflow) and its splat list comes from this walk, so
//    a linked pool gets beam starts too.  A DAG or a pool deeper than 22 levels gets the
//    reference's full 22-slot stack (stack[s_max + 1], NVIDIASVO.compute:13) and no beam starts.
int recompute_pool(svo_ctx *ctx) {
    ctx->depth_exact = false;
    ctx->depth = 22;
    std::shared_ptr<const std::vector<uint2>> boxes, held;
    const int hb = held_back(ctx);
    const bool simple = ctx->uploads.size() == 1 && ctx->uploads[0].offset == 0 && !ctx->uploads[0].external &&
                        ctx->uploads[0].tree && ctx->uploads[0].depth <= 22;
    if (simple) {
        ctx->depth_exact = true;
        ctx->depth = ctx->uploads[0].depth;
        if (ctx->beam && ctx->uploads[0].boxes_back == ctx->beam_back && ctx->uploads[0].boxes_held_back == hb) {
            boxes = ctx->uploads[0].boxes;
            held = ctx->uploads[0].boxes_held;
        }
    }
    const bool have = boxes || !ctx->beam;
    if ((!simple || !have) && ctx->n_nodes > 0 && ctx->n_nodes < 0xFFFFFFFFull) {
        // the device copy of the pool (the host arrays of earlier uploads are gone)
        const size_t n = ctx->n_nodes;
        std::vector<uint2> pool(n);
        HIP_TRY(hipSetDevice(ctx->device));
        HIP_TRY(hipDeviceSynchronize());
        HIP_TRY(hipMemcpy(pool.data(), ctx->d_nodes, n * sizeof(uint2), hipMemcpyDeviceToHost));
        std::vector<uint32_t> lo(n), first(n);
        for (size_t i = 0; i < n; ++i) {
            lo[i] = pool[i].x;
            first[i] = pool[i].y;
        }
        if (!simple) {
            // the longest descriptor path from the root, depth(v) = 1 + the max depth of v's non-leaf
            // children (a child past the uploads reads as an empty descriptor: depth 1): an iterative
            // depth-first walk, each node finished once, so shared subtrees (every trunk leaf linking
            // the same sub-SVO, Clipmap.cs:158-159) cost nothing extra; a cycle has no depth
            std::vector<uint8_t> state(n, 0), dep(n, 0), acc(n, 0);   // state: 0 new, 1 open, 2 done
            struct Frame { uint32_t v; uint32_t slot; };
            std::vector<Frame> st{{0u, 0u}};
            state[0] = 1;
            bool ok = true;
            while (!st.empty() && ok) {
                Frame &f = st.back();
                const uint32_t v = f.v, m = lo[v] & 0xFFu;
                bool pushed = false;
                while (f.slot < 8) {
                    const uint32_t c = f.slot++;
                    if (!((m >> c) & 1u)) continue;
                    const uint64_t child = (uint64_t)first[v] + (uint32_t)__builtin_popcount(m & ((1u << c) - 1u));
                    if (child >= n) { acc[v] = std::max<uint8_t>(acc[v], 1); continue; }
                    if (state[child] == 1) { ok = false; break; }   // a cycle
                    if (state[child] == 2) { acc[v] = std::max(acc[v], dep[child]); continue; }
                    state[child] = 1;
                    st.push_back({(uint32_t)child, 0u});
                    pushed = true;
                    break;
                }
                if (!ok || pushed) continue;
                dep[v] = (uint8_t)std::min(1 + (int)acc[v], 23);   // 23: deeper than the stack allows
                state[v] = 2;
                st.pop_back();
                if (!st.empty()) acc[st.back().v] = std::max(acc[st.back().v], dep[v]);
            }
            if (ok && dep[0] <= 22) {
                ctx->depth_exact = true;
                ctx->depth = dep[0];
            }
        }
        if (ctx->depth_exact && ctx->beam) {
            boxes = build_beam_boxes(lo.data(), first.data(), n, ctx->depth, ctx->beam_back);
            held = hb == ctx->beam_back ? boxes : build_beam_boxes(lo.data(), first.data(), n, ctx->depth, hb);
        }
    }
    if (boxes != ctx->pool_boxes) {
        ctx->pool_boxes = boxes;
        ctx->pool_boxes_id = boxes ? next_boxes_id() : 0;
    }
    if (held != ctx->pool_boxes_held) {
        ctx->pool_boxes_held = held;
        ctx->pool_boxes_held_id = !held ? 0 : held == boxes ? ctx->pool_boxes_id : next_boxes_id();
    }
    ctx->pool_boxes_back = ctx->beam_back;
    return SVO_OK;
}

// Commit an upload's metadata -- only after its device copies have completed.
int commit_upload(svo_ctx *ctx, const Upload &u) {
    ctx->uploads.erase(std::remove_if(ctx->uploads.begin(), ctx->uploads.end(),
                                      [&](const Upload &v) { return v.offset == u.offset; }),
                       ctx->uploads.end());
    ctx->uploads.push_back(u);
    ctx->n_nodes = std::max(ctx->n_nodes, u.offset + u.count);
    ++ctx->cost_gen;   // another pool: other costs
    return recompute_pool(ctx);
}

int ensure_out(svo_ctx *ctx, size_t px) {
    if (px <= ctx->out_cap_px) return SVO_OK;
    HIP_TRY(hipDeviceSynchronize());   // an earlier asynchronous launch may still use the old scratch
    if (ctx->d_out_hits) hipFree(ctx->d_out_hits);
    if (ctx->d_out_rgba) hipFree(ctx->d_out_rgba);
    ctx->d_out_hits = ctx->d_out_rgba = nullptr;
    ctx->out_cap_px = 0;
    HIP_TRY(hipMalloc(&ctx->d_out_hits, px * sizeof(svo_hit)));
    HIP_TRY(hipMalloc(&ctx->d_out_rgba, px * 4 * sizeof(float)));
    ctx->out_cap_px = px;
    return SVO_OK;
}

// *fresh = true when the frame was (re)allocated: the caller's sample counter then
// describes a frame that no longer exists, so the next blend must replace it (sample 0)
int ensure_accum(svo_ctx *ctx, int width, int height, bool *fresh) {
    *fresh = false;
    if (ctx->d_accum && ctx->accum_w == width && ctx->accum_h == height) return SVO_OK;
    *fresh = true;
    HIP_TRY(hipDeviceSynchronize());   // an earlier asynchronous launch may still use the old frame
    if (ctx->d_accum) hipFree(ctx->d_accum);
    if (ctx->d_accum8) hipFree(ctx->d_accum8);
    ctx->d_accum = nullptr;
    ctx->d_accum8 = nullptr;
    ctx->accum_w = ctx->accum_h = 0;
    const size_t px = (size_t)width * (size_t)height;
    HIP_TRY(hipMalloc(&ctx->d_accum, px * sizeof(float4)));
    HIP_TRY(hipMalloc(&ctx->d_accum8, px * sizeof(uint32_t)));
    HIP_TRY(hipMemset(ctx->d_accum, 0, px * sizeof(float4)));   // a fresh render target
    ctx->accum_w = width;
    ctx->accum_h = height;
    return SVO_OK;
}

void free_pinned(svo_ctx *ctx) {
    for (int i = 0; i < svo_ctx::PIN_SLOTS; ++i) {
        if (ctx->h_pin[i]) hipHostFree(ctx->h_pin[i]);
        if (ctx->d_pin[i]) hipFree(ctx->d_pin[i]);
        if (ctx->pin_packed[i]) hipEventDestroy(ctx->pin_packed[i]);
        if (ctx->pin_copied[i]) hipEventDestroy(ctx->pin_copied[i]);
        if (ctx->pin_copied2[i]) hipEventDestroy(ctx->pin_copied2[i]);
        ctx->pin_copied2[i] = nullptr;
        ctx->h_pin[i] = nullptr;
        ctx->d_pin[i] = nullptr;
        ctx->pin_packed[i] = ctx->pin_copied[i] = nullptr;
        ctx->pin_used[i] = false;
    }
    ctx->pin_w = ctx->pin_h = 0;
    ctx->pin_next = 0;
    ctx->pin_frames = 0;
}

// The pinned readback slots for a width x height frame (reallocated on a size change: the
// previous frames' pointers die with them).
int ensure_pinned(svo_ctx *ctx, int width, int height) {
    if (ctx->h_pin[0] && ctx->pin_w == width && ctx->pin_h == height) return SVO_OK;
    if (ctx->copy_stream) HIP_TRY(hipStreamSynchronize(ctx->copy_stream));
    if (ctx->copy_stream2) HIP_TRY(hipStreamSynchronize(ctx->copy_stream2));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    free_pinned(ctx);
    if (!ctx->copy_stream) HIP_TRY(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
    if (ctx->pin_push == 2 && !ctx->copy_stream2)
        HIP_TRY(hipStreamCreateWithFlags(&ctx->copy_stream2, hipStreamNonBlocking));
    // 16-byte multiple (the push kernel moves 16 B per lane); the frame is the first W * H words
    const size_t bytes = ((size_t)width * (size_t)height * sizeof(uint32_t) + 15) & ~(size_t)15;
    const unsigned host_flags = ctx->pin_push == 1 ? (hipHostMallocMapped | hipHostMallocCoherent) : hipHostMallocDefault;
    for (int i = 0; i < svo_ctx::PIN_SLOTS; ++i) {
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_pin[i]), bytes, host_flags));
        HIP_TRY(hipMalloc(&ctx->d_pin[i], bytes));
        HIP_TRY(hipEventCreateWithFlags(&ctx->pin_packed[i], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&ctx->pin_copied[i], hipEventDisableTiming));
        if (ctx->pin_push == 2) HIP_TRY(hipEventCreateWithFlags(&ctx->pin_copied2[i], hipEventDisableTiming));
    }
    ctx->pin_w = width;
    ctx->pin_h = height;
    return SVO_OK;
}

// A validated svo_band, the owner table copied (the caller's pointer is not kept).
struct Deal {
    int rows = 1, rank = 0, count = 1, cycle = 0;
    uint8_t owner[svo::MAX_CYCLE] = {};
    int owner_of(int band) const { return cycle ? owner[band % cycle] : band % count; }
    uint64_t key() const {   // identifies the deal (tile-order cache key)
        uint64_t h = 1469598103934665603ull;
        for (int i = 0; i < cycle; ++i) h = (h ^ owner[i]) * 1099511628211ull;
        return h ^ (uint64_t)cycle;
    }
};

int band_rows_local(int height, const Deal &d) {
    // rows y whose band y / rows belongs to this rank
    int rows = 0;
    if (d.cycle == 0) {
        for (int y0 = d.rank * d.rows; y0 < height; y0 += d.rows * d.count) rows += std::min(d.rows, height - y0);
        return rows;
    }
    for (int b = 0; b * d.rows < height; ++b)
        if (d.owner[b % d.cycle] == d.rank) rows += std::min(d.rows, height - b * d.rows);
    return rows;
}

int check_band(const svo_band *band, int height, Deal *out) {
    Deal d;
    if (band) {
        d.rows = band->band_rows;
        d.rank = band->band_rank;
        d.count = band->band_count;
        d.cycle = band->cycle;
    }
    if (d.rows <= 0 || d.count <= 0 || d.rank < 0 || d.rank >= d.count) return fail(SVO_ERR_ARG, "invalid svo_band");
    if (d.cycle < 0 || d.cycle > svo::MAX_CYCLE) return fail(SVO_ERR_ARG, "svo_band.cycle must be in [0, 256]");
    if (d.cycle > 0) {
        if (!band->owner) return fail(SVO_ERR_ARG, "svo_band.owner is null");
        for (int i = 0; i < d.cycle; ++i) {
            if (band->owner[i] >= d.count) return fail(SVO_ERR_ARG, "svo_band.owner entry out of range");
            d.owner[i] = band->owner[i];
        }
    }
    if (d.count == 1) {
        d.rows = height > 0 ? height : 1;
        d.cycle = 0;
    }
    *out = d;
    return SVO_OK;
}

int take_events(svo_ctx *ctx, int stage, hipEvent_t *ev0, hipEvent_t *ev1) {
    *ev0 = *ev1 = nullptr;
    if (!(ctx->options & SVO_OPT_KERNEL_TIMING)) return SVO_OK;
    if (ctx->timing_free.empty()) {
        HIP_TRY(hipEventCreate(ev0));
        if (hipEventCreate(ev1) != hipSuccess) {
            hipEventDestroy(*ev0);
            *ev0 = nullptr;
            return fail(SVO_ERR_HIP, "hipEventCreate");
        }
    } else {
        *ev0 = ctx->timing_free.back().first;
        *ev1 = ctx->timing_free.back().second;
        ctx->timing_free.pop_back();
    }
    ctx->timing_events[stage].emplace_back(*ev0, *ev1);
    return SVO_OK;
}

svo::Outputs outputs_of(const svo_frame *f) {
    svo::Outputs o{};
    if (!f) return o;
    o.hits = reinterpret_cast<svo::Hit *>(f->hits);
    o.rgba = reinterpret_cast<float4 *>(f->rgba);
    o.rgba8 = f->rgba8;
    o.compact = reinterpret_cast<uint32_t *>(f->compact);
    o.position = reinterpret_cast<float4 *>(f->position);
    o.voxel = reinterpret_cast<unsigned long long *>(f->voxel);
    o.rgb8 = f->rgb8;
    o.hitmask = reinterpret_cast<unsigned long long *>(f->hitmask);
    o.frame_layout = f->layout == SVO_LAYOUT_FRAME ? 1 : 0;
    return o;
}

// svo_render_samples' arguments (launch's optional last parameter)
struct SampleArgs {
    int n;
    const float *offsets;   // 2 n floats
    uint32_t first;
    float4 *accum;
    uint32_t *rgba8;
    uint8_t *rgb8;
    int layout;
};

// The splat's view of a camera (svo_traverse.h BeamParams): origin, the inverse of the pixel ->
// direction map and the frustum's side planes, in double from the render's own formulas
// (svo_kernel.hip camera_ray).  False for a camera the splat cannot bound (non-finite, singular,
// or a field of view so wide that the projection's clipping margin no longer holds).
bool beam_camera(const svo::Camera &c, int width, int height, svo::BeamParams *bp) {
    double A[3], B[3], C[3];
    for (int r = 0; r < 3; ++r) {   // dir = C3 (IP (u, v, 0, 1)).xyz, u = 2 fx / W - 1, v = 2 fy / H - 1
        A[r] = B[r] = C[r] = 0.0;
        for (int k = 0; k < 3; ++k) {
            A[r] += (double)c.c2w[k * 4 + r] * c.inv_proj[0 * 4 + k];
            B[r] += (double)c.c2w[k * 4 + r] * c.inv_proj[1 * 4 + k];
            C[r] += (double)c.c2w[k * 4 + r] * c.inv_proj[3 * 4 + k];
        }
    }
    double M[3][3];
    for (int r = 0; r < 3; ++r) {
        M[r][0] = 2.0 * A[r] / width;
        M[r][1] = 2.0 * B[r] / height;
        M[r][2] = C[r] - A[r] - B[r];
    }
    const double det = M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) -
                       M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) +
                       M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
    if (!std::isfinite(det) || det == 0.0) return false;
    double inv[3][3];
    for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 3; ++k) {
            const int r1 = (k + 1) % 3, r2 = (k + 2) % 3, c1 = (r + 1) % 3, c2 = (r + 2) % 3;
            inv[r][k] = (M[r1][c1] * M[r2][c2] - M[r1][c2] * M[r2][c1]) / det;   // adjugate / det
        }
    auto dir = [&](double fx, double fy, double d[3]) {
        for (int r = 0; r < 3; ++r) d[r] = M[r][0] * fx + M[r][1] * fy + M[r][2];
    };
    auto len = [](const double d[3]) { return std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]); };
    double D[4][3], mid[3];
    dir(-1.0, -1.0, D[0]);
    dir(width + 1.0, -1.0, D[1]);
    dir(width + 1.0, height + 1.0, D[2]);
    dir(-1.0, height + 1.0, D[3]);
    dir(0.5 * width, 0.5 * height, mid);
    double lmin = len(mid), lmax = len(mid);
    for (int j = 0; j < 4; ++j) {
        lmin = std::min(lmin, len(D[j]));
        lmax = std::max(lmax, len(D[j]));
    }
    if (!(lmin > 0.0) || lmax > 30.0 * lmin) return false;
    for (int j = 0; j < 4; ++j) {
        const double *a = D[j], *b = D[(j + 1) % 4];
        double n[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
        const double sgn = n[0] * mid[0] + n[1] * mid[1] + n[2] * mid[2] < 0.0 ? -1.0 : 1.0;
        const double l = len(n);
        if (!(l > 0.0) || !std::isfinite(l)) return false;
        for (int k = 0; k < 3; ++k) bp->plane[j][k] = (float)(sgn * n[k] / l);
    }
    for (int r = 0; r < 3; ++r) {
        double a = 0.0;
        for (int k = 0; k < 3; ++k) {
            bp->minv[3 * r + k] = (float)inv[r][k];
            if (!std::isfinite(bp->minv[3 * r + k])) return false;
            a += std::fabs(inv[r][k]);
        }
        bp->minv_abs[r] = (float)(a * (1.0 + 1e-6));
    }
    for (int k = 0; k < 3; ++k) {   // mul4(c2w, (0, 0, 0, 1)) then to_svo, in f32 (both steps exact or one rounding)
        const float w = c.c2w[12 + k];
        if (!std::isfinite(w)) return false;
        for (int j = 0; j < 3; ++j)
            if (!std::isfinite(c.c2w[4 * j + k])) return false;
        bp->org[k] = w * (1.0f / 32.0f) + 1.5f;
    }
    return true;
}

int launch(svo_ctx *ctx, int width, int height, int stack_mode, const svo_band *band, svo::Outputs out,
           hipStream_t stream, const SampleArgs *sa = nullptr) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (width <= 0 || height <= 0) return fail(SVO_ERR_ARG, "width/height must be positive");
    if ((size_t)width * (size_t)height > ((size_t)1 << 31)) return fail(SVO_ERR_ARG, "frame larger than 2^31 pixels");
    if (stack_mode != SVO_STACK_HLSL && stack_mode != SVO_STACK_EXACT)
        return fail(SVO_ERR_ARG, "unknown stack mode");
    if (ctx->n_nodes == 0) return fail(SVO_ERR_STATE, "no node pool uploaded (svo_set_buffer)");
    if (!ctx->cam_set) return fail(SVO_ERR_STATE, "camera not set (svo_set_camera)");
    Deal b;
    int rc = check_band(band, height, &b);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(ctx->device));
    svo::LaunchParams p;
    std::memset(&p, 0, sizeof p);
    bool jittered = false;   // per-launch pixel offsets: the tiles' costs drift without a new view
    p.nodes = ctx->d_nodes;
    p.att = ctx->d_att;
    p.n_nodes = (uint32_t)std::min<size_t>(ctx->n_nodes, 0xFFFFFFFFu);
    p.cam = ctx->cam;
    p.width = width;
    p.height = height;
    p.band_rows = b.rows;
    p.band_rank = b.rank;
    p.band_count = b.count;
    p.band_cycle = b.cycle;
    for (int i = 0; i < b.cycle; ++i)
        if (b.owner[i] == b.rank) p.band_pos[p.band_cnt++] = (uint8_t)i;
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
    p.out = out;
    if (b.count == 1) p.out.frame_layout = 0;   // the whole frame: both layouts coincide
    p.xcd_remap = ctx->xcd_remap;
    if (p.xcd_remap == 2 && ((width + 7) / 8) % (8 * svo::STRIP_K) != 0) p.xcd_remap = 0;
    p.shadows = (ctx->options & SVO_OPT_SHADOW_RAYS) ? (ctx->shadow_compact ? 3 : ctx->fused_shadows ? 2 : 1) : 0;
    if (sa && sa->n == 1) {
        // one sample: the one-sample launch itself with AddShader's blend in its store epilogue (the
        // samples kernel's S waves per tile, barrier and blend loop cost S = 1 ~13 %)
        std::memset(&p.out, 0, sizeof p.out);
        p.out.accum = sa->accum;
        p.out.acc_a = 1.0f / ((float)sa->first + 1.0f);   // launch_accumulate's a and b, _Sample = first
        p.out.acc_b = 1.0f - p.out.acc_a;
        p.out.rgba8 = sa->rgba8;
        p.out.rgb8 = sa->rgb8;
        p.out.frame_layout = sa->layout == SVO_LAYOUT_FRAME && b.count > 1 ? 1 : 0;
        p.cam.px_off[0] = sa->offsets[0];   // this sample's _PixelOffset
        p.cam.px_off[1] = sa->offsets[1];
        p.shadows = 0;
        jittered = true;
        sa = nullptr;
    }
    if (sa) {   // samples in flight: primary rays only, the blend replaces every other output
        // S stack regions of max(slots, 2) x 64 x 8 bytes in one workgroup (svo_kernel.hip)
        const size_t lds = (size_t)std::max(p.slots, 2) * svo::TILE * sizeof(uint2) * (size_t)sa->n;
        if (lds > ctx->lds_per_block)
            return fail(SVO_ERR_ARG, "svo_render_samples: " + std::to_string(sa->n) + " samples of a depth-" +
                                         std::to_string(ctx->depth) + " pool need " + std::to_string(lds) +
                                         " bytes of LDS per workgroup, the device allows " +
                                         std::to_string(ctx->lds_per_block) + ": use fewer samples per launch");
        p.samples = sa->n;
        for (int k = 0; k < sa->n; ++k) {
            p.sample_off[k][0] = sa->offsets[2 * k];
            p.sample_off[k][1] = sa->offsets[2 * k + 1];
            // launch_accumulate's a and b (host float arithmetic), _Sample = first + k
            p.blend_a[k] = 1.0f / ((float)(sa->first + (uint32_t)k) + 1.0f);
            p.blend_b[k] = 1.0f - p.blend_a[k];
        }
        p.accum = sa->accum;
        p.accum8 = sa->rgba8;
        p.accum_rgb8 = sa->rgb8;
        std::memset(&p.out, 0, sizeof p.out);
        p.out.rgba = sa->accum;   // only tells `record` to shade; the samples kernel stores the blend itself
        p.out.frame_layout = sa->layout == SVO_LAYOUT_FRAME && b.count > 1 ? 1 : 0;
        p.shadows = 0;
    }
    if (p.shadows == 3 && out.hitmask) p.shadows = 1;   // the caller's masks are not a list scratch
    if (p.local_rows == 0) return SVO_OK;
    const bool instr = out.fetches || out.starts;   // instrumented: svo_count_fetches / svo_beam_starts
    if (instr) p.shadows = 0;
    hipStream_t s = stream ? stream : ctx->stream;
    if ((p.shadows == 1 || p.shadows == 3) && !p.out.hits && !p.out.compact) {   // the second pass reads the records
        int rc2 = ensure_out(ctx, (size_t)(p.out.frame_layout ? height : p.local_rows) * (size_t)width);
        if (rc2) return rc2;
        rc2 = order_scratch(ctx, s);
        if (rc2) return rc2;
        p.out.hits = reinterpret_cast<svo::Hit *>(ctx->d_out_hits);
    }
    if (p.shadows == 3) {   // the compacted pass's masks + hit list (shared scratch, ordered like d_out_hits)
        const size_t need = svo::shadow_list_bytes(width, p.local_rows);
        if (ctx->shadow_list_cap < need) {
            HIP_TRY(hipDeviceSynchronize());   // an earlier launch may still read the old list
            if (ctx->d_shadow_list) hipFree(ctx->d_shadow_list);
            ctx->d_shadow_list = nullptr;
            ctx->shadow_list_cap = 0;
            HIP_TRY(hipMalloc(&ctx->d_shadow_list, need));
            ctx->shadow_list_cap = need;
        }
        rc = order_scratch(ctx, s);
        if (rc) return rc;
        p.out.hitmask = reinterpret_cast<unsigned long long *>(ctx->d_shadow_list);
    }
    p.prio = ctx->prio;
    const bool ordered = ctx->tile_order && !instr;
    const int n_tiles = ((width + 7) / 8) * ((p.local_rows + 7) / 8);
    Geo key;        // the geometry (seg 0): the key of the costs and of the loop-form decision
    Geo okey;       // the order's key: key + the seg_cap its order was built with
    int seg_cap = 0;
    Sched *q = nullptr;
    if (ordered) {
        rc = sched_for(ctx, s, &q);
        if (rc) return rc;
        // a new _PixelOffset at the same view (the reference's frame loop draws one every frame,
        // RaytracingMaster.cs:35): the stored segment starts belong to another sub-pixel ray
        if (!p.samples && q->view_prev == ctx->view_gen &&
            (p.cam.px_off[0] != q->off_prev[0] || p.cam.px_off[1] != q->off_prev[1]))
            jittered = true;
        // field by field (a hash of overlapping shifted fields could match another geometry
        // and reuse a permutation of a different tile count)
        key.width = width;
        key.local_rows = p.local_rows;
        key.rows = b.rows;
        key.rank = b.rank;
        key.count = b.count;
        key.xcd = p.xcd_remap;
        key.n_tiles = n_tiles;
        key.deal = b.key();
        // segmented heavy tiles: primary rays of a tree pool in XCD-strip order
        seg_cap = (ctx->seg_mode || ctx->seg_all) && p.xcd_remap == 2 && !p.guard && p.shadows == 0 && !p.samples
                      ? (ctx->seg_all ? (n_tiles + 7) / 8 : ctx->seg_cap) : 0;
        const size_t order_need = svo::order_strips_entries(n_tiles, seg_cap);
        if (!q->side) {
            HIP_TRY(hipStreamCreateWithFlags(&q->side, hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&q->render_done, hipEventDisableTiming));
            for (int i = 0; i < 2; ++i) HIP_TRY(hipEventCreateWithFlags(&q->build_ev[i], hipEventDisableTiming));
        }
        if (q->cap < (size_t)n_tiles || q->order_cap < order_need) {
            HIP_TRY(hipStreamSynchronize(s));   // a pending launch on this stream may still use the old buffers
            HIP_TRY(hipStreamSynchronize(q->side));   // ... or an order build
            free_sched(*q);
            const size_t cap = svo::order_cost_capacity(n_tiles);
            for (int i = 0; i < 2; ++i) {
                HIP_TRY(hipMalloc(&q->cost_buf[i], cap * sizeof(uint16_t)));
                HIP_TRY(hipMemset(q->cost_buf[i], 0, cap * sizeof(uint16_t)));
                HIP_TRY(hipMalloc(&q->part_buf[i], svo::SEG_KMAX * cap * sizeof(uint16_t)));
                HIP_TRY(hipMemset(q->part_buf[i], 0, svo::SEG_KMAX * cap * sizeof(uint16_t)));
                HIP_TRY(hipMalloc(&q->order_buf[i], order_need * sizeof(uint32_t)));
            }
            HIP_TRY(hipMalloc(&q->shadow_cost, cap * sizeof(uint16_t)));
            HIP_TRY(hipMemset(q->shadow_cost, 0, cap * sizeof(uint16_t)));
            HIP_TRY(hipMalloc(&q->shadow_order, ((size_t)n_tiles + 36) * sizeof(uint32_t)));
            q->cap = (size_t)n_tiles;
            q->order_cap = order_need;
        }
        if (seg_cap) {
            const size_t px = (size_t)width * (size_t)p.local_rows;
            if (q->hint_cap < px) {
                HIP_TRY(hipStreamSynchronize(s));
                if (q->seg_hint) hipFree(q->seg_hint);
                q->seg_hint = nullptr;
                q->hint_cap = 0;
                HIP_TRY(hipMalloc(&q->seg_hint, 2 * px * sizeof(float4)));
                HIP_TRY(hipMemset(q->seg_hint, 0xFF, 2 * px * sizeof(float4)));   // NaN: no starts yet
                q->hint_cap = px;
            }
        }
        if (!q->stats) {
            const size_t words = 16 * Sched::STATS_RING;
            HIP_TRY(hipHostMalloc(&q->stats, words * sizeof(uint32_t), hipHostMallocCoherent | hipHostMallocMapped));
            std::memset(q->stats, 0, words * sizeof(uint32_t));
            for (int r = 0; r < Sched::STATS_RING; ++r)
                HIP_TRY(hipEventCreateWithFlags(&q->stats_ev[r], hipEventDisableTiming));
        }
        p.tile_cost = q->cost_buf[q->launches & 1];   // this launch's costs (see Sched)
        p.part_cost = q->part_buf[q->launches & 1];
        if (p.shadows == 1 && ctx->shadow_order_enabled) {
            p.shadow_cost = q->shadow_cost;
            p.shadow_order = q->shadow_key == key ? q->shadow_order : nullptr;
        }
    }
    // Loop form.  A launch whose total work is small against its heaviest wave -- a strong
    // split's per-GPU band, a sky-heavy pose, a lone tile row -- is bound by that wave's serial
    // chain, and the latency form (svo_kernel.hip trace_lat: the node kept in the stack entry,
    // the next node loaded mid-trip, half the occupancy) runs it faster; a launch that fills
    // the chip's wave slots many times over is bound by issue, and the lean loop's full
    // occupancy wins.  Measured: latency form faster when the wave trips T
    // (sum over tiles) and heaviest tile M satisfy T < 0.3 * slots * M, slots = the lean
    // loop's resident waves on the chip.  T and M come from the order kernel of the last
    // COMPLETED order build at this geometry (stats_ev; the host may be many launches ahead
    // of the GPU).  Decisions of an earlier view are kept while the camera moves (one launch
    // per view: the last frame's costs); once a build for the current view is in flight --
    // the second launch after a move -- the host waits for it (once per view), so a jump to
    // a different pose is never rendered with another pose's choice.
    // The costs (and so the decision) are keyed on the render mode too: a shadowed launch's
    // tile costs include its shadow trips.  The wait can block the host for up to a frame,
    // once per new view (svo_rt.h, svo_render_device).
    // The same statistics decide whether the heaviest tiles are traced as segmented rays
    // (segments on: exactly when the launch is latency-bound, i.e. its heaviest chain and not
    // its issued work bounds it -- a strong split's band).
    const int mode_now = p.shadows | (stack_mode << 2);
    // whether this launch's primary rays get beam starts (the test of the beam block below, less the
    // per-launch camera checks)
    const bool beam_planned = ctx->beam && q && !p.guard && !instr && ctx->depth_exact && ctx->pool_boxes &&
                              !ctx->pool_boxes->empty();
    p.lat = 0;
    bool latency_bound = false;
    const bool have_order = q && [&] { Geo g = q->order_key; g.seg = g.kpack = 0; return g == key; }();
    if (!p.guard && p.shadows == 0 && !instr && !p.samples && (ctx->lat_mode != 0 || seg_cap)) {
        if (ctx->lat_mode == 1) {
            latency_bound = true;
        } else if (q && q->stats && have_order) {
            // the newest pending build first: wait for it if it is this view's and this view has
            // no decision yet (once per view), else take the newest build that has completed
            // (stream order: then every older one has too) and drop the older ones
            const bool decided = q->lat_key == key && q->lat_view == ctx->view_gen && q->lat_mode == mode_now;
            for (int i = 1; i <= Sched::STATS_RING; ++i) {
                const int r = (q->stats_head + Sched::STATS_RING - i) % Sched::STATS_RING;
                if (!q->stats_pending[r]) continue;
                const bool wait = i == 1 && !decided && q->stats_key[r] == key && q->stats_view[r] == ctx->view_gen &&
                                  q->stats_mode[r] == mode_now;
                const hipError_t st = wait ? hipEventSynchronize(q->stats_ev[r]) : hipEventQuery(q->stats_ev[r]);
                if (st == hipErrorNotReady) continue;
                if (st != hipSuccess) return fail(SVO_ERR_HIP, std::string("order build event: ") + hipGetErrorString(st));
                for (int j = i; j <= Sched::STATS_RING; ++j)   // r and every older build (newer ones stay pending)
                    q->stats_pending[(q->stats_head + Sched::STATS_RING - j) % Sched::STATS_RING] = false;
                if (q->stats_key[r] == key && q->stats_mode[r] == mode_now) {
                    const volatile uint32_t *st16 = q->stats + 16 * r;
                    uint32_t m = 0;
                    uint64_t t = 0;
                    for (int x = 0; x < 8; ++x) {
                        m = std::max(m, (uint32_t)st16[2 * x]);
                        t += st16[2 * x + 1];
                    }
                    const size_t lds = (size_t)p.slots * svo::TILE * sizeof(uint2);
                    const double slots = (double)ctx->num_cus * (double)std::min<size_t>(32, (160 * 1024) / lds);
                    // with beam starts the rule picks only the class table (the loop stays lean); measured
                    // boundary 0.28: C3 bands at N = 2 (flyover 0.18, terrain-facing 0.23, Main.unity 0.27)
                    // run faster with the latency table, the flyover frame (0.30, 0.30-0.33 panning),
                    // terrain-facing (0.45) and Main.unity (0.49) with the issue table
                    const double ratio = beam_planned ? ctx->seg_ratio : ctx->lat_ratio;
                    // hysteresis of 15 % around it once this geometry and mode have a decision: costs
                    // measured under one class table (or with jittered rays) move T a little, and a
                    // flip near the boundary costs more than either table (the next launches find no
                    // order built for the other table's class layout)
                    const bool prior = q->lat_key == q->stats_key[r] && q->lat_mode == q->stats_mode[r];
                    const double bound = !prior ? ratio : q->lat_cache ? ratio * 1.15 : ratio / 1.15;
                    q->lat_cache = m > 0 && (double)t < bound * slots * (double)m ? 1 : 0;
                    q->lat_short = m < (uint32_t)ctx->seg_min_chain;
                    // far fewer summed trips than resident slots x the heaviest chain (a band of an 8-way
                    // split): the chain alone bounds the launch and eight segments shorten it most.  No
                    // hysteresis: the second build at a new geometry reads costs of the fallback order's
                    // layout (C3 Main.unity 8-way band: 0.118 once, 0.079 from then on), and a sticky
                    // decision would keep that transient (0.0417 ms against 0.0378 with eighths)
                    q->lat_thin = q->lat_cache && (double)t < ctx->thin_ratio * slots * (double)m;
                    q->lat_key = q->stats_key[r];
                    q->lat_view = q->stats_view[r];
                    q->lat_mode = q->stats_mode[r];
                    if (ctx->debug & 1)   // diagnostics (SVO_DEBUG bit 0): the decision and its inputs
                        std::fprintf(stderr, "svo lat: view %llu T %llu M %u slots %.0f ratio %.6f bound %.6f thin %.6f "
                                     "beam %d -> %s%s\n", q->lat_view, (unsigned long long)t, m, slots,
                                     m ? (double)t / (slots * (double)m) : 0.0, bound, (double)ctx->thin_ratio,
                                     beam_planned ? 1 : 0, q->lat_cache ? "latency" : "lean", q->lat_thin ? " thin" : "");
                }
                break;
            }
            latency_bound = q->lat_key == key && q->lat_mode == mode_now && q->lat_cache;
        }
    }
    int used_kpack = 0;   // the class layout of the order this launch dispatches in
    if (q) {   // the order this launch dispatches in: with segmented heavy tiles if so decided
        okey = key;
        // a latency-bound launch whose heaviest chain is short (C1, C2: 76 and 111 trips) runs faster in
        // the latency form without segments or beam starts (C2 0.041 against 0.047 ms, C1 0.025 / 0.031)
        const bool short_chains = latency_bound && !ctx->seg_all && q->lat_short;
        okey.kpack = ctx->seg_all ? ctx->seg_all * 0x111111 : short_chains || (jittered && ctx->seg_jitter == 0) ? 0
                   : latency_bound ? (q->lat_thin ? ctx->seg_kpack_thin : ctx->seg_kpack_lat) : ctx->seg_kpack_issue;
        okey.seg = seg_cap && okey.kpack ? seg_cap : 0;
        if (!okey.seg) okey.kpack = 0;
        // the newest build it follows by >= 2 launches (Sched): a build that launch n - 2 was
        // followed by read the cost buffer this launch writes, so it is waited for whatever its key
        const long long n = (long long)q->launches;
        int use = -1;
        for (int i = 0; i < 2; ++i) {
            if (q->build_at[i] < 0 || q->build_at[i] > n - 2) continue;
            if (!q->build_seen[i]) {
                const hipError_t st = hipEventQuery(q->build_ev[i]);
                if (st == hipErrorNotReady) HIP_TRY(hipStreamWaitEvent(s, q->build_ev[i], 0));
                else if (st != hipSuccess) return fail(SVO_ERR_HIP, std::string("order build: ") + hipGetErrorString(st));
                q->build_seen[i] = true;
            }
            if (q->build_key[i] == okey && (use < 0 || q->build_at[i] > q->build_at[use])) use = i;
        }
        if (use < 0) {   // none for this class table yet: the newest at this geometry, with its own table
            for (int i = 0; i < 2; ++i) {
                if (q->build_at[i] < 0 || q->build_at[i] > n - 2) continue;
                Geo g = q->build_key[i];
                if (g.seg && !okey.seg) continue;   // part entries only where this launch segments
                g.seg = g.kpack = 0;
                if (g == key && (use < 0 || q->build_at[i] > q->build_at[use])) use = i;
            }
        }
        p.tile_order = use >= 0 ? q->order_buf[use] : nullptr;
        if (ctx->debug & 2)   // diagnostics (SVO_DEBUG bit 1): the order and class table each launch takes
            std::fprintf(stderr, "svo order: launch %lld view %llu latency %d kpack %x use %d built_at %lld/%lld keys %d/%d\n",
                         n, ctx->view_gen, (int)latency_bound, okey.kpack, use, q->build_at[0], q->build_at[1],
                         (int)(q->build_key[0] == okey), (int)(q->build_key[1] == okey));
        const Geo &bk = use >= 0 ? q->build_key[use] : okey;   // the class layout the order was built with
        used_kpack = bk.kpack;
        if (p.tile_order && bk.seg) {   // the order lists part entries: the segmented kernel
            p.seg = bk.seg;
            p.seg_kmax = svo::seg_kmax_of(bk.kpack);
            const bool even = (jittered && ctx->seg_jitter == 2) || (q->view_prev != ctx->view_gen && ctx->seg_move == 2);
            p.seg_hint = even ? nullptr : q->seg_hint;
            if (ctx->seg_scramble) p.seg_scramble = ctx->seg_scramble * 0x9E3779B9u + ++ctx->seg_launches;
        }
    }
    // with segmented tiles the whole tiles keep the lean loop: the latency form's doubled LDS halves
    // the resident waves of the quarters too (C3 flyover bands, profiles/r05b_seg_ab.json: N = 2
    // 0.0804 ms with it against 0.0629 without, N = 4 0.0500 / 0.0457, N = 8 0.0388 / 0.0395)
    p.lat = latency_bound && ctx->lat_mode != 0 && (!p.seg || ctx->lat_mode == 1) ? 1 : 0;
    const char *log_path = ctx->wave_log_path.empty() ? nullptr : ctx->wave_log_path.c_str();
    // one record per workgroup: the tile kernel's grid, or the segmented kernel's (its part entries)
    const size_t n_wave = p.seg ? (size_t)svo::order_strips_grid(n_tiles, p.seg, p.seg_kmax) : (size_t)n_tiles;
    if (log_path && !instr) {
        if (ctx->wave_log_cap < n_wave) {
            HIP_TRY(hipDeviceSynchronize());
            if (ctx->d_wave_log) hipFree(ctx->d_wave_log);
            ctx->d_wave_log = nullptr;
            ctx->wave_log_cap = 0;
            HIP_TRY(hipMalloc(&ctx->d_wave_log, n_wave * 4 * svo::WAVE_LOG_WORDS));
            ctx->wave_log_cap = n_wave;
        }
        HIP_TRY(hipMemsetAsync(ctx->d_wave_log, 0, n_wave * 4 * svo::WAVE_LOG_WORDS, s));
        p.wave_log = ctx->d_wave_log;
    }
    // Beam starts: a tree pool's primary rays start at a per-tile lower bound of
    // their hit t, splatted from the pool's boxes right before the render, on its stream.  The
    // bounds are a function of the camera matrices, the pool and the frame size only (pixel offsets
    // in [0, 1] are covered), so a launch at the view of this stream's previous one reuses them --
    // a held view (the reference's accumulating camera) splats once; a moving camera every frame.
    // an instrumented launch with the beam: SVO_OPT_COUNT_BEAM's fetch count, or svo_beam_starts
    const bool count_beam = (p.out.fetches && (ctx->options & SVO_OPT_COUNT_BEAM)) || p.out.starts;
    if (ctx->beam && (q || count_beam) && !p.guard && (!instr || count_beam) && ctx->depth_exact && !p.lat) {
        auto in01 = [](float v) { return v >= 0.0f && v <= 1.0f; };
        bool offs = in01(p.cam.px_off[0]) && in01(p.cam.px_off[1]);
        if (p.samples) {
            offs = true;
            for (int k = 0; k < p.samples; ++k) offs = offs && in01(p.sample_off[k][0]) && in01(p.sample_off[k][1]);
        }
        svo::BeamParams bp;
        std::memset(&bp, 0, sizeof bp);
        const int tx = (width + 7) / 8, ty = (height + 7) / 8, sx = (width + 63) / 64, sy = (height + 63) / 64;
        const size_t need = (size_t)tx * ty + (size_t)sx * sy + 1;
        // the stream's own buffer; an instrumented launch (no scheduling state) the shared scratch
        unsigned long long *&buf = q ? q->tile_start : ctx->count_ts;
        size_t &cap = q ? q->ts_cap : ctx->count_ts_cap;
        uint32_t &gen = q ? q->ts_gen : ctx->count_ts_gen;
        // A new view splats the moving camera's list; the view's next launch on this stream (a held
        // view: the reference's accumulating camera, the drop-in's jittered frames) re-splats once with
        // the finer held list and every later one reuses that.  An instrumented launch (the fetch count
        // of the walk the render runs, svo_beam_starts) takes the held list.
        const bool same_view = q && q->ts_view == ctx->view_gen && q->ts_w == width && q->ts_h == height &&
                               cap >= need && gen != 0;
        const int li = !q || same_view ? 1 : 0;
        const std::shared_ptr<const std::vector<uint2>> &boxes = li ? ctx->pool_boxes_held : ctx->pool_boxes;
        const uint64_t bid = li ? ctx->pool_boxes_held_id : ctx->pool_boxes_id;
        DevBoxes &db = ctx->dev_boxes[li];
        if (boxes && !boxes->empty() && offs && beam_camera(p.cam, width, height, &bp)) {
            if (db.id != bid) {   // the device copy of this splat list
                const size_t nb = boxes->size();
                HIP_TRY(hipDeviceSynchronize());   // launches on any stream may still read the old one
                if (db.cap < nb) {
                    if (db.d) hipFree(db.d);
                    db.d = nullptr;
                    db.cap = 0;
                    HIP_TRY(hipMalloc(&db.d, nb * sizeof(uint2)));
                    db.cap = nb;
                }
                HIP_TRY(hipMemcpy(db.d, boxes->data(), nb * sizeof(uint2), hipMemcpyHostToDevice));
                db.n = (uint32_t)nb;
                db.id = bid;
            }
            if (!q) {
                rc = order_scratch(ctx, s);
                if (rc) return rc;
            }
            const bool reuse = same_view && q->ts_boxes == bid;
            if (!reuse && (cap < need || gen == 0xFFFFFFFEu)) {   // (re)filled with all-ones keys: generation 0, stale
                HIP_TRY(hipDeviceSynchronize());   // a pending launch may still read the old buffer
                if (cap < need) {
                    if (buf) hipFree(buf);
                    buf = nullptr;
                    cap = 0;
                    HIP_TRY(hipMalloc(&buf, need * sizeof(unsigned long long)));
                    cap = need;
                }
                HIP_TRY(hipMemset(buf, 0xFF, cap * sizeof(unsigned long long)));
                gen = 0;
            }
            if (!reuse) ++gen;
            bp.boxes = db.d;
            bp.n_boxes = db.n;
            bp.tile_start = buf;
            bp.gen = gen;
            bp.diag = ctx->beam_diag;   // timing diagnostics only
            bp.tiles_x = tx;
            bp.tiles_y = ty;
            bp.super_x = sx;
            bp.super_y = sy;
            bp.super_off = tx * ty;
            bp.global_off = tx * ty + sx * sy;
            bp.width = width;
            bp.height = height;
            if (!reuse) {
                hipError_t eb = svo::launch_beam_splat(bp, s);
                if (eb != hipSuccess) return fail(SVO_ERR_HIP, std::string("beam splat launch: ") + hipGetErrorString(eb));
                if (q) {
                    q->held_splat = li == 1;
                    q->ts_view = ctx->view_gen;
                    q->ts_boxes = bid;
                    q->ts_w = width;
                    q->ts_h = height;
                }
            }
            p.tile_start = buf;
            p.ts_gen = gen;
            p.ts_tiles_x = tx;
            p.ts_super_x = sx;
            p.ts_super_off = bp.super_off;
            p.ts_global_off = bp.global_off;
        }
    }
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    if (!instr) {
        rc = take_events(ctx, STAGE_KERNEL, &ev0, &ev1);
        if (rc) return rc;
    }
    hipError_t e = svo::launch_render(p, stack_mode, s, ev0, ev1);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("render launch: ") + hipGetErrorString(e));
    // refresh: a new geometry, every order_every-th launch while costs can drift, a change of
    // render mode, and a camera move -- right after the first launch at a view the camera then
    // holds (that launch still uses the old order, a permutation of the same tiles, placement
    // only, and records fresh costs), but while the camera moves every launch only every
    // move_every-th launch: each build is an order kernel plus an event on the render stream, and
    // the last few frames' costs order a slowly moving view almost as well as its own
    bool refresh = false;
    bool moving_build = false;   // the build follows a launch at a new view (a moving camera)
    if (q && p.tile_cost) {
        const unsigned long long n = q->launches++;   // (p.tile_cost is cost_buf[n % 2])
        const bool moving = q->view_prev != ctx->view_gen;   // a new view since this stream's last launch
        q->view_prev = ctx->view_gen;
        q->off_prev[0] = p.cam.px_off[0];
        q->off_prev[1] = p.cam.px_off[1];
        // the periodic rebuild only when costs can have changed without a new view (a jittered
        // pixel offset, a new light or pool, per-launch sample offsets): a held view with nothing
        // else changed records the same costs every launch, so its order stays exact
        const bool drift = q->built_cost != ctx->cost_gen || p.samples != 0 || jittered;
        // a launch dispatched in an order of another class layout (the first at a new class table)
        // recorded its costs under that layout: the next build at this table comes from a launch in
        // its own layout (C3 N = 2 band: 0.059 ms with the first build kept, 0.050 with its own)
        const bool relayout = ctx->relayout && p.tile_order && (p.seg != okey.seg || (okey.seg && p.seg_kmax != svo::seg_kmax_of(okey.kpack))
                                               || used_kpack != okey.kpack);
        if (relayout) q->relayout_pending = true;
        const bool own_layout = !relayout && q->relayout_pending;
        // (a held view's finer re-splat shortens its rays: the order is rebuilt from that launch's costs)
        refresh = q->order_key != okey || (n % ctx->order_every == 0 && drift) || q->built_mode != mode_now || own_layout ||
                  q->held_splat ||
                  (q->built_view != ctx->view_gen && (!moving || n - q->last_build >= (unsigned long long)ctx->move_every));
        q->held_splat = false;
        if (own_layout) q->relayout_pending = false;
        if (refresh) q->last_build = n;
        moving_build = moving;
    }
    if (refresh) {   // the launch after next at this geometry dispatches the heaviest tiles first
        const int r = q->stats_head;
        uint32_t *st16 = q->stats ? q->stats + 16 * r : nullptr;
        const int bi = q->next_buf;
        q->next_buf ^= 1;
        // on the side stream, behind this launch (its costs; and every launch that read buffer bi)
        HIP_TRY(hipEventRecord(q->render_done, s));
        HIP_TRY(hipStreamWaitEvent(q->side, q->render_done, 0));
        e = p.xcd_remap == 2 ? svo::launch_order_strips(p.tile_cost, q->order_buf[bi], n_tiles, (width + 7) / 8, q->side,
                                                        st16, okey.seg, p.part_cost, okey.kpack,
                                                        moving_build && ctx->spread ? 1 : 0)
                             : svo::launch_order_tiles(p.tile_cost, q->order_buf[bi], n_tiles, q->side, st16);
        if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("tile order launch: ") + hipGetErrorString(e));
        HIP_TRY(hipEventRecord(q->build_ev[bi], q->side));
        q->build_at[bi] = (long long)q->launches - 1;   // launches was incremented above
        q->build_seen[bi] = false;
        q->build_key[bi] = okey;
        q->order_key = okey;
        q->built_view = ctx->view_gen;
        q->built_cost = ctx->cost_gen;
        q->built_mode = mode_now;
        if (st16) {   // slot r: a build still pending there (ring full) is simply superseded
            HIP_TRY(hipEventRecord(q->stats_ev[r], q->side));
            q->stats_pending[r] = true;
            q->stats_key[r] = key;
            q->stats_view[r] = ctx->view_gen;
            q->stats_mode[r] = mode_now;
            q->stats_head = (r + 1) % Sched::STATS_RING;
        }
    }
    if (q && p.shadow_cost && (q->shadow_key != key || q->shadow_launches++ % ctx->order_every == 0)) {
        e = p.xcd_remap == 2 ? svo::launch_order_strips(q->shadow_cost, q->shadow_order, n_tiles, (width + 7) / 8, s)
                             : svo::launch_order_tiles(q->shadow_cost, q->shadow_order, n_tiles, s);
        if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("shadow order launch: ") + hipGetErrorString(e));
        q->shadow_key = key;
    }
    if (p.wave_log) {   // blocking dump of the last launch's per-wave record
        HIP_TRY(hipStreamSynchronize(s));
        std::vector<uint32_t> h(n_wave * svo::WAVE_LOG_WORDS);
        HIP_TRY(hipMemcpy(h.data(), ctx->d_wave_log, h.size() * 4, hipMemcpyDeviceToHost));
        if (FILE *f = std::fopen(log_path, "wb")) {
            std::fwrite(h.data(), 4 * svo::WAVE_LOG_WORDS, n_wave, f);
            std::fclose(f);
        }
    }
    return SVO_OK;
}

// Enqueue the assemble kernel on this context's device (svo_assemble_frame, and
// the gather of a multi-device frame).
int assemble(svo_ctx *ctx, int width, int height, const Deal &deal, int n_parts, const void *const *parts,
             int part_format, int skip_part, const svo::Outputs &out, hipStream_t s) {
    svo::AssembleParams a;
    std::memset(&a, 0, sizeof a);
    a.att = ctx->d_att;
    a.n_nodes = (uint32_t)std::min<size_t>(ctx->n_nodes, 0xFFFFFFFFu);
    a.cam = ctx->cam;
    a.width = width;
    a.height = height;
    a.band_rows = deal.rows;
    a.n_parts = n_parts;
    a.cycle = deal.cycle;
    for (int i = 0; i < deal.cycle; ++i) {
        const int m = deal.owner[i];
        a.owner[i] = (uint8_t)m;
        a.idx[i] = (uint8_t)a.cnt[m]++;
    }
    a.part_format = part_format;
    a.skip_part = skip_part;
    for (int i = 0; i < n_parts; ++i) a.parts[i] = parts[i];
    a.out = out;
    a.out.frame_layout = 1;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int rc = take_events(ctx, STAGE_ASSEMBLE, &ev0, &ev1);
    if (rc) return rc;
    if (ev0) HIP_TRY(hipEventRecord(ev0, s));
    if (part_format == SVO_PART_SPARSE_RGB8) {   // the parts' tile counts (their offsets travel in them)
        const int tiles_x = (width + 7) / 8;
        for (int m = 0; m < n_parts; ++m) {
            Deal dm = deal;
            dm.rank = m;
            a.n_tiles[m] = (uint32_t)(tiles_x * ((band_rows_local(height, dm) + 7) / 8));
        }
    }
    hipError_t e = svo::launch_assemble(a, s);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("assemble launch: ") + hipGetErrorString(e));
    if (ev1) HIP_TRY(hipEventRecord(ev1, s));
    return SVO_OK;
}

int check_assemble_args(svo_ctx *ctx, int width, int height, int n_parts, int part_format, int skip_part,
                        const svo::Outputs &o) {
    if (width <= 0 || height <= 0) return fail(SVO_ERR_ARG, "width/height must be positive");
    if (n_parts < 1 || n_parts > svo::MAX_PARTS) return fail(SVO_ERR_ARG, "n_parts must be in [1, 64]");
    if (skip_part < -1 || skip_part >= n_parts) return fail(SVO_ERR_ARG, "skip_part out of range");
    if (o.position || o.voxel || o.fetches) return fail(SVO_ERR_ARG, "position / voxel outputs are not assembled");
    if (o.rgb8 || o.hitmask) return fail(SVO_ERR_ARG, "the assembled frame is RGBA8 (rgb8 / hitmask are band payloads)");
    if (part_format == SVO_PART_RGBA8 || part_format == SVO_PART_RGB8 || part_format == SVO_PART_SPARSE_RGB8) {
        if (!o.rgba8 || o.hits || o.rgba || o.compact)
            return fail(SVO_ERR_ARG, "RGBA8 / RGB8 / sparse parts rebuild only an RGBA8 frame");
        if (part_format == SVO_PART_SPARSE_RGB8 && !ctx->cam_set)
            return fail(SVO_ERR_STATE, "camera not set (svo_set_camera): sparse parts need it for the sky");
    } else if (part_format == SVO_PART_COMPACT) {
        if ((o.hits || o.rgba || o.rgba8) && ctx->n_nodes == 0)
            return fail(SVO_ERR_STATE, "no node pool uploaded: compact parts need the SVO replica");
        if ((o.rgba || o.rgba8) && !ctx->cam_set) return fail(SVO_ERR_STATE, "camera not set (svo_set_camera)");
    } else {
        return fail(SVO_ERR_ARG, "unknown part format");
    }
    return SVO_OK;
}

// ------------------------------------------------------ multi-device frame
// sa (svo_render_samples): every member traces S samples of its bands and blends them into its
// own band accumulation (the display member into the caller's frame-layout accum); the members'
// payloads are the blended bands' 3-byte RGB, assembled into the caller's rgba8 frame.
int multi_render(svo_ctx *ctx, int width, int height, int stack_mode, const svo_frame *frame, hipStream_t stream,
                 const SampleArgs *sa = nullptr) {
    const int n = (int)ctx->members.size();
    svo::Outputs out = outputs_of(frame);
    out.frame_layout = 1;
    if (out.position || out.voxel) return fail(SVO_ERR_ARG, "position / voxel outputs are not gathered across devices");
    if (out.rgb8 || out.hitmask) return fail(SVO_ERR_ARG, "a multi-device frame is assembled as rgba8, not rgb8 / hitmask");
    if (!out.hits && !out.rgba && !out.rgba8 && !out.compact) return fail(SVO_ERR_ARG, "no output requested");
    // display-only frames travel as 3-byte RGB (the RGBA8 word without its constant alpha), or
    // (SVO_SPARSE_PAYLOAD=1) as sparse parts: tile hit masks + offsets + the hits' RGB, pulled by the
    // assemble kernel with no host round trip (the offsets travel in the part)
    const int fmt = sa ? SVO_PART_RGB8
                    : (out.hits || out.rgba || out.compact) ? SVO_PART_COMPACT
                    : ctx->sparse_payload ? SVO_PART_SPARSE_RGB8 : SVO_PART_RGB8;
    const size_t elem = fmt == SVO_PART_COMPACT ? 12 : 3;
    // the band accumulations hold the rows of the deal they were blended under: a continued
    // accumulation (first sample > 0) under another deal would blend into other members' rows
    uint64_t dkey = 1469598103934665603ull ^ (uint64_t)n ^ ((uint64_t)ctx->band_rows << 16);
    for (int i = 0; i < ctx->deal_cycle; ++i) dkey = (dkey ^ ctx->deal_owner[i]) * 1099511628211ull;
    dkey ^= (uint64_t)ctx->deal_cycle << 40;
    if (sa) {
        if (sa->first > 0 && ctx->samples_deal_set && ctx->samples_deal != dkey)
            return fail(SVO_ERR_STATE, "the band deal changed since the last svo_render_samples: restart the "
                                       "accumulation at first_sample 0");
        ctx->samples_deal = dkey;
        ctx->samples_deal_set = true;
    }
    const int k = ctx->parity;
    ctx->parity ^= 1;
    svo_ctx *m0 = ctx->members[0];
    hipStream_t s0 = stream ? stream : m0->stream;
    // the display device renders its own bands straight into the caller's frame
    svo_band b0{ctx->band_rows, 0, n, ctx->deal_cycle, ctx->deal_cycle ? ctx->deal_owner : nullptr};
    int rc = launch(m0, width, height, stack_mode, &b0, out, s0, sa);
    if (rc) return rc;
    std::vector<const void *> parts(n, nullptr);
    for (int i = 1; i < n; ++i) {
        svo_ctx *m = ctx->members[i];
        Peer &pr = ctx->peers[i];
        svo_band bi{ctx->band_rows, i, n, ctx->deal_cycle, ctx->deal_cycle ? ctx->deal_owner : nullptr};
        Deal di;
        rc = check_band(&bi, height, &di);
        if (rc) return rc;
        const int rows_i = band_rows_local(height, di);
        const int tiles_i = ((width + 7) / 8) * ((rows_i + 7) / 8);
        const size_t bytes = fmt == SVO_PART_SPARSE_RGB8 ? SVO_SPARSE_PART_BYTES(tiles_i, (size_t)rows_i * width)
                                                         : (size_t)rows_i * (size_t)width * elem;
        HIP_TRY(hipSetDevice(m->device));
        if (pr.cap_bytes < bytes) {
            // the assembles of earlier frames read the old payloads, possibly on another caller
            // stream than this call's: wait for the last assemble of each payload slot
            HIP_TRY(hipSetDevice(m0->device));
            for (int j = 0; j < 2; ++j)
                if (ctx->gathered_used[j]) HIP_TRY(hipEventSynchronize(ctx->gathered[j]));
            HIP_TRY(hipSetDevice(m->device));
            HIP_TRY(hipStreamSynchronize(m->stream));
            for (int j = 0; j < 2; ++j) {
                if (pr.buf[j]) hipFree(pr.buf[j]);
                pr.buf[j] = nullptr;
            }
            pr.cap_bytes = 0;
            for (int j = 0; j < 2; ++j) HIP_TRY(hipMalloc(&pr.buf[j], std::max<size_t>(bytes, 16)));
            pr.cap_bytes = bytes;
        }
        if (fmt == SVO_PART_SPARSE_RGB8 && pr.dense_cap < (size_t)rows_i * width * 3) {
            HIP_TRY(hipStreamSynchronize(m->stream));   // an earlier pack may still read the old scratch
            if (pr.dense) hipFree(pr.dense);
            pr.dense = nullptr;
            pr.dense_cap = 0;
            HIP_TRY(hipMalloc(&pr.dense, std::max<size_t>((size_t)rows_i * width * 3, 16)));
            pr.dense_cap = (size_t)rows_i * width * 3;
        }
        if (sa && (pr.accum_w != width || pr.accum_rows != rows_i || pr.accum_deal != dkey)) {   // this member's band accumulation
            HIP_TRY(hipStreamSynchronize(m->stream));
            if (pr.accum) hipFree(pr.accum);
            pr.accum = nullptr;
            pr.accum_w = 0;
            pr.accum_rows = -1;
            const size_t abytes = std::max<size_t>((size_t)rows_i * (size_t)width * sizeof(float4), 16);
            HIP_TRY(hipMalloc(&pr.accum, abytes));
            HIP_TRY(hipMemsetAsync(pr.accum, 0, abytes, m->stream));   // a fresh render target
            pr.accum_w = width;
            pr.accum_rows = rows_i;
            pr.accum_deal = dkey;
        }
        if (ctx->gathered_used[k]) HIP_TRY(hipStreamWaitEvent(m->stream, ctx->gathered[k], 0));   // payload k is free
        svo::Outputs oi{};
        if (fmt == SVO_PART_COMPACT) {
            oi.compact = reinterpret_cast<uint32_t *>(pr.buf[k]);
        } else if (fmt == SVO_PART_SPARSE_RGB8) {
            oi.rgb8 = reinterpret_cast<uint8_t *>(pr.dense);
            oi.hitmask = reinterpret_cast<unsigned long long *>(pr.buf[k]);
        } else {
            oi.rgb8 = reinterpret_cast<uint8_t *>(pr.buf[k]);
        }
        SampleArgs sai{};
        if (sa) {
            sai = *sa;
            sai.accum = pr.accum;
            sai.rgba8 = nullptr;
            sai.rgb8 = reinterpret_cast<uint8_t *>(pr.buf[k]);
            sai.layout = SVO_LAYOUT_BAND;
        }
        rc = launch(m, width, height, stack_mode, &bi, oi, m->stream, sa ? &sai : nullptr);
        if (rc) return rc;
        if (fmt == SVO_PART_SPARSE_RGB8) {
            hipError_t e = svo::launch_pack_hits(reinterpret_cast<const uint8_t *>(pr.dense), width, rows_i, pr.buf[k],
                                                 m->stream);
            if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("pack hits launch: ") + hipGetErrorString(e));
        }
        parts[i] = pr.buf[k];
        if (pr.link == SVO_LINK_COPY) {
            // no peer access to this member: its stream copies the payload into a buffer on the
            // display device (the whole capacity for a sparse part, whose size only the device
            // knows).  local[k] is reused only after frame k's assemble: the member's stream
            // waited for gathered[k] above, before this frame's render
            if (pr.local_cap < bytes) {
                HIP_TRY(hipSetDevice(m0->device));
                for (int j = 0; j < 2; ++j)
                    if (ctx->gathered_used[j]) HIP_TRY(hipEventSynchronize(ctx->gathered[j]));
                for (int j = 0; j < 2; ++j) {
                    if (pr.local[j]) hipFree(pr.local[j]);
                    pr.local[j] = nullptr;
                }
                pr.local_cap = 0;
                for (int j = 0; j < 2; ++j) HIP_TRY(hipMalloc(&pr.local[j], std::max<size_t>(bytes, 16)));
                pr.local_cap = bytes;
                HIP_TRY(hipSetDevice(m->device));
            }
            HIP_TRY(hipMemcpyPeerAsync(pr.local[k], m0->device, pr.buf[k], m->device, bytes, m->stream));
            parts[i] = pr.local[k];
        }
        HIP_TRY(hipEventRecord(pr.rendered[k], m->stream));
    }
    HIP_TRY(hipSetDevice(m0->device));
    for (int i = 1; i < n; ++i) HIP_TRY(hipStreamWaitEvent(s0, ctx->peers[i].rendered[k], 0));
    Deal deal;
    rc = check_band(&b0, height, &deal);
    if (rc) return rc;
    rc = assemble(m0, width, height, deal, n, parts.data(), fmt, 0, out, s0);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(ctx->gathered[k], s0));
    ctx->gathered_used[k] = true;
    return SVO_OK;
}

// Multi-device upload: the region [offset, offset + n) was validated and uploaded on
// the display member; copy its nodes and attachments to every other member's pool
// device to device (xGMI / SDMA, no second host validation walk or PCIe copy) and
// commit the same upload record there.
int replicate_upload(svo_ctx *g, size_t offset, size_t n) {
    svo_ctx *m0 = g->members[0];
    if (n == 0) return SVO_OK;
    const Upload *u0 = nullptr;
    for (const Upload &u : m0->uploads)
        if (u.offset == offset) u0 = &u;
    if (!u0) return fail(SVO_ERR_STATE, "replicate_upload: no upload record on the display member");
    const Upload u = *u0;
    for (size_t i = 1; i < g->members.size(); ++i) {
        svo_ctx *m = g->members[i];
        if (offset + n > m->capacity) return fail(SVO_ERR_CAPACITY, "upload exceeds a member's node-pool capacity");
        HIP_TRY(hipSetDevice(m->device));
        HIP_TRY(hipDeviceSynchronize());   // renders on the member may still read its pool
        HIP_TRY(hipSetDevice(m0->device));
        HIP_TRY(hipMemcpyPeerAsync(m->d_nodes + offset, m->device, m0->d_nodes + offset, m0->device,
                                   n * sizeof(uint2), m0->stream));
        HIP_TRY(hipMemcpyPeerAsync(m->d_att + offset, m->device, m0->d_att + offset, m0->device,
                                   n * sizeof(uint2), m0->stream));
    }
    HIP_TRY(hipSetDevice(m0->device));
    HIP_TRY(hipStreamSynchronize(m0->stream));
    for (size_t i = 1; i < g->members.size(); ++i) {
        const int rc = commit_upload(g->members[i], u);
        if (rc) return rc;
    }
    return SVO_OK;
}

int destroy_single(svo_ctx *ctx) {
    hipSetDevice(ctx->device);
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    hipDeviceSynchronize();   // renders on caller streams may still use the context's buffers
    if (ctx->d_nodes) hipFree(ctx->d_nodes);
    if (ctx->d_att) hipFree(ctx->d_att);
    if (ctx->d_stage) hipFree(ctx->d_stage);
    if (ctx->d_shadow_list) hipFree(ctx->d_shadow_list);
    if (ctx->d_out_hits) hipFree(ctx->d_out_hits);
    if (ctx->d_out_rgba) hipFree(ctx->d_out_rgba);
    if (ctx->d_accum) hipFree(ctx->d_accum);
    if (ctx->d_accum8) hipFree(ctx->d_accum8);
    if (ctx->copy_stream) hipStreamSynchronize(ctx->copy_stream);
    if (ctx->copy_stream2) hipStreamSynchronize(ctx->copy_stream2);
    free_pinned(ctx);
    if (ctx->copy_stream) hipStreamDestroy(ctx->copy_stream);
    if (ctx->copy_stream2) hipStreamDestroy(ctx->copy_stream2);
    ctx->copy_pool.reset();
    if (ctx->h_stage) hipHostFree(ctx->h_stage);
    for (int i = 0; i < svo_ctx::STAGE_CHUNKS; ++i)
        if (ctx->stage_ev[i]) hipEventDestroy(ctx->stage_ev[i]);
    for (Sched &q : ctx->sched) {
        free_sched(q);
        if (q.seg_hint) hipFree(q.seg_hint);
        if (q.tile_start) hipFree(q.tile_start);
        if (q.done) hipEventDestroy(q.done);
        for (int r = 0; r < Sched::STATS_RING; ++r)
            if (q.stats_ev[r]) hipEventDestroy(q.stats_ev[r]);
        if (q.side) {
            hipStreamSynchronize(q.side);
            hipStreamDestroy(q.side);
        }
        if (q.render_done) hipEventDestroy(q.render_done);
        for (int i = 0; i < 2; ++i)
            if (q.build_ev[i]) hipEventDestroy(q.build_ev[i]);
        if (q.stats) hipHostFree(q.stats);
    }
    for (auto &v : ctx->timing_events)
        for (auto &ev : v) { hipEventDestroy(ev.first); hipEventDestroy(ev.second); }
    for (auto &ev : ctx->timing_free) { hipEventDestroy(ev.first); hipEventDestroy(ev.second); }
    if (ctx->switch_event) hipEventDestroy(ctx->switch_event);
    if (ctx->d_wave_log) hipFree(ctx->d_wave_log);
    for (DevBoxes &db : ctx->dev_boxes)
        if (db.d) hipFree(db.d);
    if (ctx->count_ts) hipFree(ctx->count_ts);
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    delete ctx;
    return SVO_OK;
}

// ------------------------------------------------------------------ svo_config
void config_of(const svo_ctx *c, svo_config *o) {
    svo_config k;
    std::memset(&k, 0, sizeof k);
    k.size = sizeof(svo_config);
    k.version = SVO_CONFIG_VERSION;
    k.tile_order = c->tile_order;
    k.xcd_strips = c->xcd_remap == 2 ? 1 : 0;
    k.issue_priority = c->prio;
    k.order_every = c->order_every;
    k.move_every = c->move_every;
    k.move_spread = c->spread;
    k.relayout = c->relayout;
    k.fetch_all = c->fetch_all;
    k.loop_form = c->lat_mode;
    k.lat_ratio = c->lat_ratio;
    k.segments = c->seg_mode;
    k.seg_table_latency = (uint32_t)c->seg_kpack_lat;
    k.seg_table_issue = (uint32_t)c->seg_kpack_issue;
    k.seg_table_thin = (uint32_t)c->seg_kpack_thin;
    k.seg_ratio = c->seg_ratio;
    k.seg_thin_ratio = c->thin_ratio;
    k.seg_cap = c->seg_cap;
    k.seg_min_chain = c->seg_min_chain;
    k.seg_move = c->seg_move;
    k.seg_jitter = c->seg_jitter;
    k.seg_all = c->seg_all;
    k.seg_scramble = c->seg_scramble;
    k.beam = c->beam;
    k.beam_back = c->beam_back;
    k.beam_back_held = c->beam_back_held;
    k.shadow_form = c->shadow_compact ? 2 : c->fused_shadows ? 0 : 1;
    k.shadow_order = c->shadow_order_enabled;
    k.readback = c->pin_push;
    k.host_copy_threads = c->host_copy_threads;
    k.sparse_payload = c->sparse_payload;
    k.peer_copy = c->peer_copy;
    *o = k;
}

int check_config(const svo_config &k) {
    auto bit = [](int32_t v) { return v == 0 || v == 1; };
    auto table = [](uint32_t t) {
        if (t > 0xFFFFFFu) return false;
        for (int c = 0; c < 6; ++c) {
            const uint32_t kc = (t >> (4 * c)) & 15u;
            if (kc != 0 && kc != 4 && kc != 8) return false;
        }
        return true;
    };
    auto ratio = [](float r) { return std::isfinite(r) && r >= 0.0f; };
    const char *bad = !bit(k.tile_order) ? "tile_order" : !bit(k.xcd_strips) ? "xcd_strips"
                    : !bit(k.issue_priority) ? "issue_priority" : k.order_every < 1 ? "order_every"
                    : k.move_every < 1 ? "move_every" : !bit(k.move_spread) ? "move_spread"
                    : !bit(k.relayout) ? "relayout" : k.fetch_all < -1 || k.fetch_all > 1 ? "fetch_all"
                    : k.loop_form < -1 || k.loop_form > 1 ? "loop_form" : !ratio(k.lat_ratio) ? "lat_ratio"
                    : !bit(k.segments) ? "segments" : !table(k.seg_table_latency) ? "seg_table_latency"
                    : !table(k.seg_table_issue) ? "seg_table_issue" : !table(k.seg_table_thin) ? "seg_table_thin"
                    : !ratio(k.seg_ratio) ? "seg_ratio" : !ratio(k.seg_thin_ratio) ? "seg_thin_ratio"
                    : k.seg_cap < 1 ? "seg_cap" : k.seg_min_chain < 0 ? "seg_min_chain"
                    : k.seg_move < 1 || k.seg_move > 2 ? "seg_move" : k.seg_jitter < 0 || k.seg_jitter > 2 ? "seg_jitter"
                    : k.seg_all != 0 && k.seg_all != 4 && k.seg_all != 8 ? "seg_all" : !bit(k.beam) ? "beam"
                    : k.beam_back < 0 || k.beam_back > 22 ? "beam_back" : k.shadow_form < 0 || k.shadow_form > 2 ? "shadow_form"
                    : !bit(k.shadow_order) ? "shadow_order" : k.readback < 0 || k.readback > 2 ? "readback"
                    : k.host_copy_threads < 0 || k.host_copy_threads > 16 ? "host_copy_threads"
                    : !bit(k.sparse_payload) ? "sparse_payload" : !bit(k.peer_copy) ? "peer_copy"
                    : k.beam_back_held < -1 || k.beam_back_held > 22 ? "beam_back_held" : nullptr;
    if (bad) return fail(SVO_ERR_ARG, std::string("svo_config.") + bad + " out of range");
    return SVO_OK;
}

// One device's context takes a validated config.  Nothing here changes a result; what holds state
// built under the old value is rebuilt: the pinned readback slots (their allocation flags follow
// `readback`), the host copy threads, the pool's splat lists (beam, beam_back, beam_back_held); and every stream's
// loop-form / class-table decision is dropped, so the next order build decides under the new rule.
int apply_config(svo_ctx *c, const svo_config &k) {
    c->tile_order = k.tile_order;
    c->xcd_remap = k.xcd_strips ? 2 : 0;
    c->prio = k.issue_priority;
    c->order_every = k.order_every;
    c->move_every = k.move_every;
    c->spread = k.move_spread;
    c->relayout = k.relayout;
    c->fetch_all = k.fetch_all;
    c->lat_mode = k.loop_form;
    c->lat_ratio = k.lat_ratio;
    c->seg_mode = k.segments;
    c->seg_kpack_lat = (int)k.seg_table_latency;
    c->seg_kpack_issue = (int)k.seg_table_issue;
    c->seg_kpack_thin = (int)k.seg_table_thin;
    c->seg_ratio = k.seg_ratio;
    c->thin_ratio = k.seg_thin_ratio;
    c->seg_cap = k.seg_cap;
    c->seg_min_chain = k.seg_min_chain;
    c->seg_move = k.seg_move;
    c->seg_jitter = k.seg_jitter;
    c->seg_all = k.seg_all;
    c->seg_scramble = k.seg_scramble;
    c->shadow_compact = k.shadow_form == 2;
    c->fused_shadows = k.shadow_form == 0;
    c->shadow_order_enabled = k.shadow_order;
    c->sparse_payload = k.sparse_payload;
    c->peer_copy = k.peer_copy;
    if (c->pin_push != k.readback) {
        if (c->h_pin[0]) {
            HIP_TRY(hipSetDevice(c->device));
            HIP_TRY(hipStreamSynchronize(c->stream));
            if (c->copy_stream) HIP_TRY(hipStreamSynchronize(c->copy_stream));
            if (c->copy_stream2) HIP_TRY(hipStreamSynchronize(c->copy_stream2));
            free_pinned(c);
        }
        c->pin_push = k.readback;
    }
    if (c->host_copy_threads != k.host_copy_threads) {
        c->copy_pool.reset();   // idle between calls (svo_render waits for it)
        c->host_copy_threads = k.host_copy_threads;
    }
    const bool boxes = c->beam != k.beam || c->beam_back != k.beam_back || c->beam_back_held != k.beam_back_held;
    c->beam = k.beam;
    c->beam_back = k.beam_back;
    c->beam_back_held = k.beam_back_held;
    if (boxes && c->n_nodes > 0) {
        const int rc = recompute_pool(c);
        if (rc) return rc;
    }
    for (Sched &q : c->sched) {
        q.lat_key = Geo();
        q.lat_mode = -1;
    }
    return SVO_OK;
}

}  // namespace

extern "C" {

int svo_get_config(svo_ctx *ctx, svo_config *cfg) {
    if (!cfg) return fail(SVO_ERR_ARG, "cfg is null");
    if (cfg->size < 2 * sizeof(uint32_t)) return fail(SVO_ERR_ARG, "svo_config.size must hold at least size and version");
    static const svo_ctx defaults;
    svo_config k;
    config_of(ctx ? ctx : &defaults, &k);
    const size_t n = std::min<size_t>(cfg->size, sizeof k);
    k.size = (uint32_t)n;
    std::memcpy(cfg, &k, n);
    return SVO_OK;
}

int svo_set_config(svo_ctx *ctx, const svo_config *cfg) {
    if (!ctx || !cfg) return fail(SVO_ERR_ARG, "null argument");
    if (cfg->size < 2 * sizeof(uint32_t)) return fail(SVO_ERR_ARG, "svo_config.size must hold at least size and version");
    if (cfg->size > sizeof(svo_config))
        return fail(SVO_ERR_ARG, "svo_config.size " + std::to_string(cfg->size) + " is larger than this library's (" +
                                     std::to_string(sizeof(svo_config)) + "): a newer ABI");
    svo_config k;
    config_of(ctx, &k);   // fields past the caller's size keep the context's values
    std::memcpy(&k, cfg, cfg->size);
    k.size = sizeof k;
    k.version = SVO_CONFIG_VERSION;
    int rc = check_config(k);
    if (rc) return rc;
    if (is_multi(ctx)) {
        for (svo_ctx *m : ctx->members) {
            rc = apply_config(m, k);
            if (rc) return rc;
        }
        if (k.peer_copy != ctx->peer_copy) {   // the members' payload routes: frames in flight first
            for (svo_ctx *m : ctx->members) {
                HIP_TRY(hipSetDevice(m->device));
                HIP_TRY(hipDeviceSynchronize());
            }
            HIP_TRY(hipSetDevice(ctx->members[0]->device));
            for (size_t i = 1; i < ctx->peers.size(); ++i)
                ctx->peers[i].link = k.peer_copy ? SVO_LINK_COPY : ctx->peers[i].native_link;
        }
    }
    return apply_config(ctx, k);
}

int svo_beam_starts(svo_ctx *ctx, int width, int height, const svo_band *band, float *d_starts, void *stream) {
    if (!d_starts) return fail(SVO_ERR_ARG, "d_starts is null");
    if (ctx && is_multi(ctx)) return fail(SVO_ERR_ARG, "beam starts of a member context (svo_get_member)");
    svo::Outputs o{};
    o.starts = d_starts;
    return launch(ctx, width, height, SVO_STACK_HLSL, band, o, reinterpret_cast<hipStream_t>(stream));
}

int svo_abi_version(void) { return 10; }

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
    // zero-filled pool: descriptors never uploaded read as empty (0), like the
    // fresh ComputeBuffers of RaytracingMaster.InitializeSVOBuffer
    if (e == hipSuccess) e = hipMemsetAsync(ctx->d_nodes, 0, capacity_nodes * sizeof(uint2), ctx->stream);
    if (e == hipSuccess) e = hipMemsetAsync(ctx->d_att, 0, capacity_nodes * sizeof(uint2), ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&ctx->num_cus, hipDeviceAttributeMultiprocessorCount, device);
    int lds_block = 0;
    if (e == hipSuccess) e = hipDeviceGetAttribute(&lds_block, hipDeviceAttributeMaxSharedMemoryPerBlock, device);
    if (e == hipSuccess && lds_block > 0) ctx->lds_per_block = (size_t)lds_block;
    // diagnostics only (svo_rt.h): traces and timing aids, never a policy
    if (const char *k = std::getenv("SVO_DEBUG")) ctx->debug = std::atoi(k);
    if (const char *k = std::getenv("SVO_WAVE_LOG")) ctx->wave_log_path = k;
    if (const char *k = std::getenv("SVO_BEAM_DIAG")) ctx->beam_diag = (uint32_t)std::atoi(k);
    if (e != hipSuccess) {
        destroy_single(ctx);
        return fail(SVO_ERR_HIP, std::string("svo_create: ") + hipGetErrorString(e));
    }
    *out = ctx;
    return SVO_OK;
}

int svo_create_multi(const int *devices, int num_devices, size_t capacity_nodes, int band_rows, svo_ctx **out) {
    if (!out || !devices) return fail(SVO_ERR_ARG, "null argument");
    *out = nullptr;
    if (num_devices < 1 || num_devices > svo::MAX_PARTS) return fail(SVO_ERR_ARG, "num_devices must be in [1, 64]");
    if (band_rows <= 0) return fail(SVO_ERR_ARG, "band_rows must be positive");
    svo_ctx *g = new (std::nothrow) svo_ctx();
    if (!g) return fail(SVO_ERR_ARG, "out of host memory");
    g->device = devices[0];
    g->capacity = capacity_nodes;
    g->band_rows = band_rows;
    g->peers.resize(num_devices);
    auto bail = [&](int rc) {
        svo_destroy(g);
        return rc;
    };
    for (int i = 0; i < num_devices; ++i) {
        svo_ctx *m = nullptr;
        int rc = svo_create(devices[i], capacity_nodes, &m);
        if (rc) return bail(rc);
        g->members.push_back(m);
    }
    // the display device reads every other device's payload over xGMI (peer access);
    // a member it cannot map gets the copy fallback (SVO_LINK_COPY, multi_render).
    // svo_config.peer_copy forces the copy for every member but the display device itself
    // (the one-GPU test of that path: a repeated device index)
    for (int i = 1; i < num_devices; ++i) {
        Peer &pr = g->peers[i];
        if (devices[i] == devices[0]) {
            pr.native_link = pr.link = SVO_LINK_SELF;
            continue;
        }
        int ok = 0;
        hipError_t e = hipDeviceCanAccessPeer(&ok, devices[0], devices[i]);
        if (e != hipSuccess || !ok) {
            (void)hipGetLastError();
            pr.native_link = pr.link = SVO_LINK_COPY;
            continue;
        }
        hipSetDevice(devices[0]);
        e = hipDeviceEnablePeerAccess(devices[i], 0);
        if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) {
            (void)hipGetLastError();
            pr.native_link = pr.link = SVO_LINK_PEER;
        } else {   // reported as possible, refused when enabled: copy instead
            (void)hipGetLastError();
            pr.native_link = pr.link = SVO_LINK_COPY;
        }
    }
    for (int i = 1; i < num_devices; ++i) {
        hipSetDevice(devices[i]);
        for (int j = 0; j < 2; ++j)
            if (hipEventCreateWithFlags(&g->peers[i].rendered[j], hipEventDisableTiming) != hipSuccess)
                return bail(fail(SVO_ERR_HIP, "hipEventCreate"));
    }
    hipSetDevice(devices[0]);
    for (int j = 0; j < 2; ++j)
        if (hipEventCreateWithFlags(&g->gathered[j], hipEventDisableTiming) != hipSuccess)
            return bail(fail(SVO_ERR_HIP, "hipEventCreate"));
    *out = g;
    return SVO_OK;
}

int svo_set_band_deal(svo_ctx *ctx, int cycle, const uint8_t *owner) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (!is_multi(ctx)) return fail(SVO_ERR_ARG, "svo_set_band_deal needs a multi-device context");
    if (cycle < 0 || cycle > svo::MAX_CYCLE) return fail(SVO_ERR_ARG, "cycle must be in [0, 256]");
    if (cycle > 0 && !owner) return fail(SVO_ERR_ARG, "owner is null");
    const int n = (int)ctx->members.size();
    for (int i = 0; i < cycle; ++i)
        if (owner[i] >= n) return fail(SVO_ERR_ARG, "owner entry names no member");
    // payload sizes change: let frames in flight finish with the old deal first
    for (svo_ctx *m : ctx->members) {
        HIP_TRY(hipSetDevice(m->device));
        HIP_TRY(hipDeviceSynchronize());
    }
    ctx->deal_cycle = cycle;
    for (int i = 0; i < cycle; ++i) ctx->deal_owner[i] = owner[i];
    return SVO_OK;
}

int svo_num_devices(svo_ctx *ctx, int *n) {
    if (!ctx || !n) return fail(SVO_ERR_ARG, "null argument");
    *n = is_multi(ctx) ? (int)ctx->members.size() : 1;
    return SVO_OK;
}

int svo_get_member_link(svo_ctx *ctx, int index, int *device, int *link) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    const int n = is_multi(ctx) ? (int)ctx->members.size() : 1;
    if (index < 0 || index >= n) return fail(SVO_ERR_ARG, "member index out of range");
    if (device) *device = is_multi(ctx) ? ctx->members[index]->device : ctx->device;
    if (link) *link = is_multi(ctx) && index > 0 ? ctx->peers[index].link : SVO_LINK_SELF;
    return SVO_OK;
}

int svo_get_member(svo_ctx *ctx, int index, svo_ctx **member) {
    if (!ctx || !member) return fail(SVO_ERR_ARG, "null argument");
    const int n = is_multi(ctx) ? (int)ctx->members.size() : 1;
    if (index < 0 || index >= n) return fail(SVO_ERR_ARG, "member index out of range");
    *member = is_multi(ctx) ? ctx->members[index] : ctx;
    return SVO_OK;
}

int svo_set_buffer(svo_ctx *ctx, const int32_t *desc, size_t n_desc, const uint32_t *att,
                   size_t n_att, size_t dst_offset) {
    if (!ctx || (!desc && n_desc) || (!att && n_att)) return fail(SVO_ERR_ARG, "null argument");
    if (is_multi(ctx)) {   // validated and uploaded once, then replicated device to device
        int rc = svo_set_buffer(ctx->members[0], desc, n_desc, att, n_att, dst_offset);
        if (rc) return rc;
        return replicate_upload(ctx, dst_offset, n_desc);
    }
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
    Upload u;
    int rc = validate_upload(ctx, lo.data(), first.data(), n_desc, dst_offset, &u);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(ctx->device));
    // renders, assembles and accumulations on any stream may still read the pool
    HIP_TRY(hipDeviceSynchronize());
    if (n_desc > ctx->stage_cap) {
        HIP_TRY(hipStreamSynchronize(ctx->stream));
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
    return commit_upload(ctx, u);
}

int svo_set_buffer_v2(svo_ctx *ctx, const uint64_t *nodes, size_t n_nodes, const uint32_t *att,
                      size_t n_att, size_t dst_offset) {
    if (!ctx || (!nodes && n_nodes) || (!att && n_att)) return fail(SVO_ERR_ARG, "null argument");
    if (is_multi(ctx)) {
        int rc = svo_set_buffer_v2(ctx->members[0], nodes, n_nodes, att, n_att, dst_offset);
        if (rc) return rc;
        return replicate_upload(ctx, dst_offset, n_nodes);
    }
    if (dst_offset + n_nodes > ctx->capacity) return fail(SVO_ERR_CAPACITY, "upload exceeds node-pool capacity");
    if (n_att != 2 * n_nodes) return fail(SVO_ERR_ARG, "attachments must hold 2 words per node");
    if (n_nodes == 0) return SVO_OK;
    std::vector<uint32_t> lo(n_nodes), first(n_nodes);
    for (size_t i = 0; i < n_nodes; ++i) {
        lo[i] = (uint32_t)nodes[i];
        first[i] = (uint32_t)(nodes[i] >> 32);
        if (lo[i] > 0xFFFFu) return fail(SVO_ERR_FORMAT, "v2 node low word must only hold the two masks");
    }
    Upload u;
    int rc = validate_upload(ctx, lo.data(), first.data(), n_nodes, dst_offset, &u);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipDeviceSynchronize());   // as in svo_set_buffer
    static_assert(sizeof(uint2) == sizeof(uint64_t), "node layout");
    HIP_TRY(hipMemcpyAsync(ctx->d_nodes + dst_offset, nodes, n_nodes * sizeof(uint64_t), hipMemcpyHostToDevice,
                           ctx->stream));
    HIP_TRY(hipMemcpyAsync(ctx->d_att + dst_offset, att, n_att * sizeof(uint32_t), hipMemcpyHostToDevice,
                           ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return commit_upload(ctx, u);
}

int svo_set_camera(svo_ctx *ctx, const float c2w[16], const float inv_proj[16], float px_off_x,
                   float px_off_y, const float light[4]) {
    if (!ctx || !c2w || !inv_proj || !light) return fail(SVO_ERR_ARG, "null argument");
    for (svo_ctx *m : ctx->members) svo_set_camera(m, c2w, inv_proj, px_off_x, px_off_y, light);
    // a moved camera changes the tiles' costs: the next launch refreshes the dispatch order
    // (a new pixel offset or light alone does not)
    if (!ctx->cam_set || std::memcmp(ctx->cam.c2w, c2w, sizeof(ctx->cam.c2w)) != 0 ||
        std::memcmp(ctx->cam.inv_proj, inv_proj, sizeof(ctx->cam.inv_proj)) != 0)
        ++ctx->view_gen;
    if (!ctx->cam_set || ctx->cam.px_off[0] != px_off_x || ctx->cam.px_off[1] != px_off_y ||
        std::memcmp(ctx->cam.light, light, sizeof(ctx->cam.light)) != 0)
        ++ctx->cost_gen;
    std::memcpy(ctx->cam.c2w, c2w, sizeof(ctx->cam.c2w));
    std::memcpy(ctx->cam.inv_proj, inv_proj, sizeof(ctx->cam.inv_proj));
    ctx->cam.px_off[0] = px_off_x;
    ctx->cam.px_off[1] = px_off_y;
    std::memcpy(ctx->cam.light, light, sizeof(ctx->cam.light));
    ctx->cam_set = true;
    return SVO_OK;
}

int svo_render_frame(svo_ctx *ctx, int width, int height, int stack_mode, const svo_band *band,
                     const svo_frame *frame, void *stream) {
    if (!ctx || !frame) return fail(SVO_ERR_ARG, "null argument");
    if (is_multi(ctx)) {
        if (band && band->band_count != 1) return fail(SVO_ERR_ARG, "a multi-device context splits the frame itself");
        if (width <= 0 || height <= 0) return fail(SVO_ERR_ARG, "width/height must be positive");
        return multi_render(ctx, width, height, stack_mode, frame, reinterpret_cast<hipStream_t>(stream));
    }
    return launch(ctx, width, height, stack_mode, band, outputs_of(frame), reinterpret_cast<hipStream_t>(stream));
}

int svo_render_samples(svo_ctx *ctx, int width, int height, int stack_mode, const svo_band *band, int n_samples,
                       const float *px_offsets, uint32_t first_sample, float *d_accum, uint32_t *d_rgba8,
                       uint8_t *d_rgb8, int layout, void *stream) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (n_samples < 1 || n_samples > svo::MAX_SAMPLES) return fail(SVO_ERR_ARG, "n_samples must be in [1, 8]");
    if (!px_offsets || !d_accum) return fail(SVO_ERR_ARG, "null px_offsets or d_accum");
    if ((uintptr_t)d_accum & 15u) return fail(SVO_ERR_ARG, "d_accum must be 16-byte aligned");
    if (layout != SVO_LAYOUT_BAND && layout != SVO_LAYOUT_FRAME) return fail(SVO_ERR_ARG, "unknown layout");
    SampleArgs sa{n_samples, px_offsets, first_sample, reinterpret_cast<float4 *>(d_accum), d_rgba8, d_rgb8, layout};
    if (is_multi(ctx)) {   // the frame split over the members, each blending its own rows on its own device
        if (band && band->band_count != 1) return fail(SVO_ERR_ARG, "a multi-device context splits the frame itself");
        if (width <= 0 || height <= 0) return fail(SVO_ERR_ARG, "width/height must be positive");
        if (!d_rgba8 || d_rgb8) return fail(SVO_ERR_ARG, "a multi-device context assembles d_rgba8 (d_rgb8 must be NULL)");
        svo_frame f{};
        f.rgba8 = d_rgba8;
        f.layout = SVO_LAYOUT_FRAME;
        sa.layout = SVO_LAYOUT_FRAME;
        return multi_render(ctx, width, height, stack_mode, &f, reinterpret_cast<hipStream_t>(stream), &sa);
    }
    return launch(ctx, width, height, stack_mode, band, svo::Outputs{}, reinterpret_cast<hipStream_t>(stream), &sa);
}

int svo_assemble_frame(svo_ctx *ctx, int width, int height, const svo_band *deal, int n_parts,
                       const void *const *parts, int part_format, int skip_part, const svo_frame *frame,
                       void *stream) {
    if (!ctx || !parts || !frame || !deal) return fail(SVO_ERR_ARG, "null argument");
    svo_ctx *c = is_multi(ctx) ? ctx->members[0] : ctx;
    svo::Outputs o = outputs_of(frame);
    int rc = check_assemble_args(c, width, height, n_parts, part_format, skip_part, o);
    if (rc) return rc;
    if (deal->band_count != n_parts) return fail(SVO_ERR_ARG, "deal band_count must equal n_parts");
    svo_band db = *deal;
    db.band_rank = 0;
    Deal d;
    rc = check_band(&db, height, &d);
    if (rc) return rc;
    for (int i = 0; i < n_parts; ++i)
        if (!parts[i] && i != skip_part) return fail(SVO_ERR_ARG, "null part pointer");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    // no ordering against the context's render streams: the assemble reads only the
    // caller's parts and the (upload-synchronised) attachments and writes only the
    // caller's frame, so a gather stream beside the render stream runs concurrently
    // (ordering the two made the display rank's step 1.3x slower, tools/rank0_cost.py)
    return assemble(c, width, height, d, n_parts, parts, part_format, skip_part, o, s);
}

int svo_render(svo_ctx *ctx, int width, int height, int stack_mode, float *rgba_out, svo_hit *hits_out) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (width <= 0 || height <= 0) return fail(SVO_ERR_ARG, "width/height must be positive");
    size_t px = (size_t)width * (size_t)height;
    svo_ctx *c = is_multi(ctx) ? ctx->members[0] : ctx;
    HIP_TRY(hipSetDevice(c->device));
    int rc = ensure_out(c, px);
    if (rc) return rc;
    rc = order_scratch(c, c->stream);
    if (rc) return rc;
    svo_frame f{};
    f.hits = hits_out ? reinterpret_cast<svo_hit *>(c->d_out_hits) : nullptr;
    f.rgba = rgba_out ? reinterpret_cast<float *>(c->d_out_rgba) : nullptr;
    f.layout = SVO_LAYOUT_FRAME;
    if (is_multi(ctx)) {
        if (!hits_out && !rgba_out) return SVO_OK;
        rc = multi_render(ctx, width, height, stack_mode, &f, c->stream);
    } else {
        rc = launch(c, width, height, stack_mode, nullptr, outputs_of(&f), c->stream);
    }
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    // The outputs reach the caller's pageable arrays through plugin-owned pinned staging: the DMA of
    // chunk i (at the link's rate) runs while host threads copy chunk i - 1 out of the staging
    // (a pageable hipMemcpy stages through the runtime's own small buffer: ~13 GB/s, 6.2 ms for the
    // 83 MB of a 1080p frame, BENCH_r04.json host_path).
    const size_t hb = hits_out ? px * sizeof(svo_hit) : 0, rb = rgba_out ? px * 4 * sizeof(float) : 0;
    if (c->h_stage_cap < hb + rb) {
        if (c->h_stage) hipHostFree(c->h_stage);
        c->h_stage = nullptr;
        c->h_stage_cap = 0;
        HIP_TRY(hipHostMalloc(&c->h_stage, hb + rb, hipHostMallocDefault));
        c->h_stage_cap = hb + rb;
    }
    if (!c->stage_ev[0])
        for (int i = 0; i < svo_ctx::STAGE_CHUNKS; ++i)
            HIP_TRY(hipEventCreateWithFlags(&c->stage_ev[i], hipEventDisableTiming));
    if (!c->copy_pool) {
        const int n = c->host_copy_threads > 0 ? c->host_copy_threads : (int)std::thread::hardware_concurrency() / 2;
        c->copy_pool.reset(new CopyPool(std::max(1, std::min(n, 16))));
    }
    struct Part { char *dst; const char *dev; char *stage; size_t bytes; };
    Part parts[2];
    int np = 0;
    if (hb) parts[np++] = {reinterpret_cast<char *>(hits_out), static_cast<const char *>(c->d_out_hits),
                           static_cast<char *>(c->h_stage), hb};
    if (rb) parts[np++] = {reinterpret_cast<char *>(rgba_out), static_cast<const char *>(c->d_out_rgba),
                           static_cast<char *>(c->h_stage) + hb, rb};
    const size_t total = hb + rb;
    const size_t chunk = ((total + svo_ctx::STAGE_CHUNKS - 1) / svo_ctx::STAGE_CHUNKS + 4095) & ~(size_t)4095;
    // chunk i covers bytes [i chunk, (i + 1) chunk) of the concatenated outputs
    auto for_range = [&](size_t lo, size_t hi, auto fn) {
        size_t base = 0;
        for (int k = 0; k < np; ++k) {
            const size_t a = std::max(lo, base), b = std::min(hi, base + parts[k].bytes);
            if (a < b) fn(parts[k], a - base, b - a);
            base += parts[k].bytes;
        }
    };
    int n_chunks = 0;
    for (size_t lo = 0; lo < total; lo += chunk, ++n_chunks) {
        const size_t hi = std::min(total, lo + chunk);
        hipError_t e = hipSuccess;
        for_range(lo, hi, [&](const Part &q, size_t off, size_t n) {
            if (e == hipSuccess) e = hipMemcpyAsync(q.stage + off, q.dev + off, n, hipMemcpyDeviceToHost, c->stream);
        });
        HIP_TRY(e);
        HIP_TRY(hipEventRecord(c->stage_ev[n_chunks], c->stream));
    }
    CopyPool &pool = *c->copy_pool;
    // every exit waits for the copy threads: none may still write the caller's arrays, or read the
    // staging, once this call has returned (an error included)
    struct WaitPool {
        CopyPool &p;
        ~WaitPool() { p.wait(); }
    } wait_pool{pool};
    for (int i = 0; i < n_chunks; ++i) {
        HIP_TRY(hipEventSynchronize(c->stage_ev[i]));
        const size_t lo = (size_t)i * chunk, hi = std::min(total, lo + chunk);
        for_range(lo, hi, [&](const Part &q, size_t off, size_t n) {
            const size_t per = ((n + pool.size() - 1) / pool.size() + 63) & ~(size_t)63;
            for (size_t o = 0; o < n; o += per) pool.submit(q.dst + off + o, q.stage + off + o, std::min(per, n - o));
        });
    }
    return SVO_OK;
}

int svo_render_progressive(svo_ctx *ctx, int width, int height, int stack_mode, uint32_t sample,
                           uint32_t *rgba8_out, float *rgba_out) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (!rgba8_out && !rgba_out) return fail(SVO_ERR_ARG, "no output requested");
    if (width <= 0 || height <= 0) return fail(SVO_ERR_ARG, "width/height must be positive");
    const size_t px = (size_t)width * (size_t)height;
    svo_ctx *c = is_multi(ctx) ? ctx->members[0] : ctx;
    HIP_TRY(hipSetDevice(c->device));
    int rc = ensure_out(c, px);
    if (rc) return rc;
    bool fresh = false;
    rc = ensure_accum(c, width, height, &fresh);
    if (rc) return rc;
    if (fresh) sample = 0;   // a resized target: this sample replaces the (zeroed) frame
    rc = order_scratch(c, c->stream);
    if (rc) return rc;
    svo_frame f{};
    f.rgba = reinterpret_cast<float *>(c->d_out_rgba);   // this sample's Result
    f.layout = SVO_LAYOUT_FRAME;
    rc = is_multi(ctx) ? multi_render(ctx, width, height, stack_mode, &f, c->stream)
                       : launch(c, width, height, stack_mode, nullptr, outputs_of(&f), c->stream);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    hipError_t e = svo::launch_accumulate(c->d_accum, reinterpret_cast<const float4 *>(c->d_out_rgba), px, sample,
                                          c->num_cus, c->stream);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("accumulate launch: ") + hipGetErrorString(e));
    if (rgba8_out) {
        e = svo::launch_pack_rgba8(c->d_accum, c->d_accum8, px, c->num_cus, c->stream);
        if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("pack launch: ") + hipGetErrorString(e));
        HIP_TRY(hipMemcpyAsync(rgba8_out, c->d_accum8, px * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    }
    if (rgba_out)
        HIP_TRY(hipMemcpyAsync(rgba_out, c->d_accum, px * sizeof(float4), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SVO_OK;
}

int svo_render_progressive_async(svo_ctx *ctx, int width, int height, int stack_mode, uint32_t sample,
                                 int pixel_format, const void **frame_out) {
    if (!ctx || !frame_out) return fail(SVO_ERR_ARG, "null argument");
    *frame_out = nullptr;
    if (width <= 0 || height <= 0) return fail(SVO_ERR_ARG, "width/height must be positive");
    if (pixel_format != SVO_PIXELS_RGBA8 && pixel_format != SVO_PIXELS_RGB8)
        return fail(SVO_ERR_ARG, "unknown pixel format");
    const size_t px = (size_t)width * (size_t)height;
    svo_ctx *c = is_multi(ctx) ? ctx->members[0] : ctx;
    HIP_TRY(hipSetDevice(c->device));
    int rc = ensure_out(c, px);
    if (rc) return rc;
    bool fresh = false;
    rc = ensure_accum(c, width, height, &fresh);
    if (rc) return rc;
    if (fresh) sample = 0;   // as svo_render_progressive: a resized target restarts the accumulation
    if (c->pin_format != pixel_format) {   // the slots' previous frames are in another format
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (c->copy_stream) HIP_TRY(hipStreamSynchronize(c->copy_stream));
        if (c->copy_stream2) HIP_TRY(hipStreamSynchronize(c->copy_stream2));
        free_pinned(c);
        c->pin_format = pixel_format;
    }
    rc = ensure_pinned(c, width, height);
    if (rc) return rc;
    rc = order_scratch(c, c->stream);
    if (rc) return rc;
    svo_frame f{};
    f.rgba = reinterpret_cast<float *>(c->d_out_rgba);   // this sample's Result
    f.layout = SVO_LAYOUT_FRAME;
    rc = is_multi(ctx) ? multi_render(ctx, width, height, stack_mode, &f, c->stream)
                       : launch(c, width, height, stack_mode, nullptr, outputs_of(&f), c->stream);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    hipError_t e = svo::launch_accumulate(c->d_accum, reinterpret_cast<const float4 *>(c->d_out_rgba), px, sample,
                                          c->num_cus, c->stream);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("accumulate launch: ") + hipGetErrorString(e));
    const int k = c->pin_next;
    // slot k's previous copy (PIN_SLOTS frames ago) must have read d_pin[k] before the pack overwrites it
    if (c->pin_used[k]) HIP_TRY(hipStreamWaitEvent(c->stream, c->pin_copied[k], 0));
    e = pixel_format == SVO_PIXELS_RGB8
            ? svo::launch_pack_rgb8(c->d_accum, reinterpret_cast<uint8_t *>(c->d_pin[k]), px, c->num_cus, c->stream)
            : svo::launch_pack_rgba8(c->d_accum, c->d_pin[k], px, c->num_cus, c->stream);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("pack launch: ") + hipGetErrorString(e));
    HIP_TRY(hipEventRecord(c->pin_packed[k], c->stream));
    HIP_TRY(hipStreamWaitEvent(c->copy_stream, c->pin_packed[k], 0));
    const size_t fbytes = px * (pixel_format == SVO_PIXELS_RGB8 ? 3 : 4);
    if (c->pin_push == 1) {   // a kernel writes the mapped pinned buffer over PCIe
        void *dst = nullptr;
        HIP_TRY(hipHostGetDevicePointer(&dst, c->h_pin[k], 0));
        e = svo::launch_push_host(c->d_pin[k], dst, (fbytes + 15) & ~(size_t)15, c->num_cus, c->copy_stream);
        if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("push launch: ") + hipGetErrorString(e));
        HIP_TRY(hipEventRecord(c->pin_copied[k], c->copy_stream));
    } else if (c->pin_push == 2) {   // two DMA copies of half the frame each, on two copy streams
        const size_t half = (fbytes / 2) & ~(size_t)4095;
        HIP_TRY(hipStreamWaitEvent(c->copy_stream2, c->pin_packed[k], 0));
        HIP_TRY(hipMemcpyAsync(c->h_pin[k], c->d_pin[k], half, hipMemcpyDeviceToHost, c->copy_stream));
        HIP_TRY(hipMemcpyAsync(reinterpret_cast<uint8_t *>(c->h_pin[k]) + half,
                               reinterpret_cast<uint8_t *>(c->d_pin[k]) + half, fbytes - half, hipMemcpyDeviceToHost,
                               c->copy_stream2));
        HIP_TRY(hipEventRecord(c->pin_copied2[k], c->copy_stream2));
        HIP_TRY(hipStreamWaitEvent(c->copy_stream, c->pin_copied2[k], 0));
        HIP_TRY(hipEventRecord(c->pin_copied[k], c->copy_stream));
    } else {
        HIP_TRY(hipMemcpyAsync(c->h_pin[k], c->d_pin[k], fbytes, hipMemcpyDeviceToHost, c->copy_stream));
        HIP_TRY(hipEventRecord(c->pin_copied[k], c->copy_stream));
    }
    c->pin_used[k] = true;
    c->pin_next = (k + 1) % svo_ctx::PIN_SLOTS;
    ++c->pin_frames;
    if (c->pin_frames >= 2) {   // the previous call's frame: wait for its copy only
        const int prev = (k + svo_ctx::PIN_SLOTS - 1) % svo_ctx::PIN_SLOTS;
        HIP_TRY(hipEventSynchronize(c->pin_copied[prev]));
        *frame_out = c->h_pin[prev];
    }
    return SVO_OK;
}

int svo_progressive_last(svo_ctx *ctx, const void **frame_out) {
    if (!ctx || !frame_out) return fail(SVO_ERR_ARG, "null argument");
    *frame_out = nullptr;
    svo_ctx *c = is_multi(ctx) ? ctx->members[0] : ctx;
    if (c->pin_frames == 0) return SVO_OK;
    HIP_TRY(hipSetDevice(c->device));
    const int last = (c->pin_next + svo_ctx::PIN_SLOTS - 1) % svo_ctx::PIN_SLOTS;
    HIP_TRY(hipEventSynchronize(c->pin_copied[last]));
    *frame_out = c->h_pin[last];
    return SVO_OK;
}

int svo_render_device(svo_ctx *ctx, int width, int height, int stack_mode, const svo_band *band, void *d_rgba,
                      void *d_hits, void *stream) {
    svo_frame f{};
    f.hits = reinterpret_cast<svo_hit *>(d_hits);
    f.rgba = reinterpret_cast<float *>(d_rgba);
    f.layout = SVO_LAYOUT_BAND;
    if (ctx && is_multi(ctx)) {
        f.layout = SVO_LAYOUT_FRAME;
        if (!d_rgba && !d_hits) return SVO_OK;
    }
    return svo_render_frame(ctx, width, height, stack_mode, band, &f, stream);
}

int svo_pack_hits(svo_ctx *ctx, int width, int height, const svo_band *band, const void *d_rgb8, void *d_part,
                  void *stream) {
    if (!ctx || !d_rgb8 || !d_part) return fail(SVO_ERR_ARG, "null argument");
    if (width <= 0 || height <= 0) return fail(SVO_ERR_ARG, "width/height must be positive");
    svo_ctx *c = is_multi(ctx) ? ctx->members[0] : ctx;
    Deal d;
    int rc = check_band(band, height, &d);
    if (rc) return rc;
    const int rows = band_rows_local(height, d);
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    hipError_t e = svo::launch_pack_hits(reinterpret_cast<const uint8_t *>(d_rgb8), width, rows, d_part, s);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("pack hits launch: ") + hipGetErrorString(e));
    return SVO_OK;
}

int svo_count_fetches(svo_ctx *ctx, int width, int height, int stack_mode, const svo_band *band,
                      void *d_fetches, void *stream) {
    if (!d_fetches) return fail(SVO_ERR_ARG, "d_fetches is null");
    if (ctx && is_multi(ctx)) return fail(SVO_ERR_ARG, "count fetches on a member context (svo_get_member)");
    svo::Outputs o{};
    o.fetches = reinterpret_cast<uint32_t *>(d_fetches);
    return launch(ctx, width, height, stack_mode, band, o, reinterpret_cast<hipStream_t>(stream));
}

int svo_set_options(svo_ctx *ctx, uint32_t options) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (options & ~(uint32_t)(SVO_OPT_SHADOW_RAYS | SVO_OPT_KERNEL_TIMING | SVO_OPT_COUNT_BEAM)) return fail(SVO_ERR_ARG, "unknown option bits");
    for (svo_ctx *m : ctx->members) m->options = options;
    ctx->options = options;
    return SVO_OK;
}

int svo_stage_time(svo_ctx *ctx, int stage, double *mean_ms, uint64_t *launches) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (stage < 0 || stage >= N_STAGES) return fail(SVO_ERR_ARG, "unknown stage");
    if (is_multi(ctx)) {
        // every member records its own launches (svo_set_options sets the option on all):
        // drain them all, so none accumulates events, and report the slowest member
        double worst = 0.0;
        uint64_t worst_n = 0;
        for (svo_ctx *m : ctx->members) {
            double ms = 0.0;
            uint64_t n = 0;
            int rc = svo_stage_time(m, stage, &ms, &n);
            if (rc) return rc;
            if (n && (worst_n == 0 || ms > worst)) { worst = ms; worst_n = n; }
        }
        if (mean_ms) *mean_ms = worst;
        if (launches) *launches = worst_n;
        return SVO_OK;
    }
    svo_ctx *c = ctx;
    HIP_TRY(hipSetDevice(c->device));
    double sum = 0.0;
    uint64_t n = 0;
    hipError_t err = hipSuccess;
    for (auto &ev : c->timing_events[stage]) {
        float ms = 0.0f;
        if (err == hipSuccess) err = hipEventSynchronize(ev.second);
        if (err == hipSuccess) err = hipEventElapsedTime(&ms, ev.first, ev.second);
        if (err == hipSuccess) { sum += ms; ++n; }
        c->timing_free.push_back(ev);
    }
    c->timing_events[stage].clear();
    if (err != hipSuccess) return fail(SVO_ERR_HIP, std::string("svo_stage_time: ") + hipGetErrorString(err));
    if (mean_ms) *mean_ms = n ? sum / (double)n : 0.0;
    if (launches) *launches = n;
    return SVO_OK;
}

int svo_kernel_time(svo_ctx *ctx, double *mean_ms, uint64_t *launches) {
    return svo_stage_time(ctx, STAGE_KERNEL, mean_ms, launches);
}

int svo_stage_times(svo_ctx *ctx, int stage, float *ms_out, size_t cap, size_t *launches) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (stage < 0 || stage >= N_STAGES) return fail(SVO_ERR_ARG, "unknown stage");
    if (cap && !ms_out) return fail(SVO_ERR_ARG, "ms_out is null");
    svo_ctx *c = is_multi(ctx) ? ctx->members[0] : ctx;
    if (is_multi(ctx))   // the other members' records are dropped, so none accumulates
        for (size_t i = 1; i < ctx->members.size(); ++i) {
            int rc = svo_stage_time(ctx->members[i], stage, nullptr, nullptr);
            if (rc) return rc;
        }
    HIP_TRY(hipSetDevice(c->device));
    size_t n = 0;
    hipError_t err = hipSuccess;
    for (auto &ev : c->timing_events[stage]) {
        float ms = 0.0f;
        if (err == hipSuccess) err = hipEventSynchronize(ev.second);
        if (err == hipSuccess) err = hipEventElapsedTime(&ms, ev.first, ev.second);
        if (err == hipSuccess) {
            if (n < cap) ms_out[n] = ms;
            ++n;
        }
        c->timing_free.push_back(ev);
    }
    c->timing_events[stage].clear();
    if (err != hipSuccess) return fail(SVO_ERR_HIP, std::string("svo_stage_times: ") + hipGetErrorString(err));
    if (launches) *launches = n;
    return SVO_OK;
}

int svo_get_info(svo_ctx *ctx, size_t *n_nodes, int *max_depth, int *device) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    svo_ctx *c = is_multi(ctx) ? ctx->members[0] : ctx;
    if (n_nodes) *n_nodes = c->n_nodes;
    if (max_depth) *max_depth = c->depth;
    if (device) *device = c->device;
    return SVO_OK;
}

int svo_accumulate(svo_ctx *ctx, void *d_accum, const void *d_sample, size_t n_px, uint32_t sample,
                   void *stream) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (n_px == 0) return SVO_OK;
    if (!d_accum || !d_sample) return fail(SVO_ERR_ARG, "null accumulation or sample buffer");
    if (((uintptr_t)d_accum | (uintptr_t)d_sample) & 15u) return fail(SVO_ERR_ARG, "buffers must be 16-byte aligned");
    svo_ctx *c = is_multi(ctx) ? ctx->members[0] : ctx;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    // caller buffers only: the caller orders them against its renders (no context state)
    hipError_t e = svo::launch_accumulate(reinterpret_cast<float4 *>(d_accum), reinterpret_cast<const float4 *>(d_sample),
                                          n_px, sample, c->num_cus, s);
    if (e != hipSuccess) return fail(SVO_ERR_HIP, std::string("accumulate launch: ") + hipGetErrorString(e));
    return SVO_OK;
}

int svo_forget_stream(svo_ctx *ctx, void *stream) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (!stream) return SVO_OK;   // the context's own stream lives as long as the context
    for (svo_ctx *m : ctx->members) {
        int rc = svo_forget_stream(m, stream);
        if (rc) return rc;
    }
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    bool known = ctx->scratch_valid && ctx->scratch_stream == s;
    for (Sched &q : ctx->sched) known = known || (q.used && q.stream == s);
    if (!known) return SVO_OK;
    HIP_TRY(hipStreamSynchronize(s));
    for (Sched &q : ctx->sched) {
        if (!q.used || q.stream != s) continue;
        // the set's buffers stay allocated for the next stream; only the stream is forgotten
        if (q.side) HIP_TRY(hipStreamSynchronize(q.side));
        q.used = false;
        q.stream = nullptr;
        reset_builds(q);
        q.launches = q.shadow_launches = 0;
        q.view_prev = ~0ull;
        q.built_cost = ~0ull;
        q.last_build = 0;
        for (int r = 0; r < Sched::STATS_RING; ++r) q.stats_pending[r] = false;
        q.lat_key = Geo();
        q.lat_mode = -1;
    }
    if (ctx->scratch_valid && ctx->scratch_stream == s) {
        ctx->scratch_valid = false;
        ctx->scratch_stream = nullptr;
    }
    return SVO_OK;
}

int svo_synchronize(svo_ctx *ctx) {
    if (!ctx) return fail(SVO_ERR_ARG, "null context");
    if (is_multi(ctx)) {
        for (svo_ctx *m : ctx->members) {
            int rc = svo_synchronize(m);
            if (rc) return rc;
        }
        return SVO_OK;
    }
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipDeviceSynchronize());   // the context's stream and every caller stream it rendered on
    // nothing is pending on any stream now, and a caller may destroy its streams (svo_rt.h): the
    // context records no event on a stream it saw before this point (an eviction of its
    // dispatch-order set skips the hand-over event; the host-path scratch needs no ordering)
    for (Sched &q : ctx->sched) q.idle = true;
    ctx->scratch_valid = false;
    ctx->scratch_stream = nullptr;
    return SVO_OK;
}

int svo_destroy(svo_ctx *ctx) {
    if (!ctx) return SVO_OK;
    if (!is_multi(ctx) && ctx->peers.empty()) return destroy_single(ctx);
    for (svo_ctx *m : ctx->members) {   // drain every device first: payloads and events are shared
        hipSetDevice(m->device);
        hipDeviceSynchronize();
    }
    for (size_t i = 1; i < ctx->peers.size(); ++i) {
        Peer &pr = ctx->peers[i];
        if (i < ctx->members.size()) hipSetDevice(ctx->members[i]->device);
        for (int j = 0; j < 2; ++j) {
            if (pr.buf[j]) hipFree(pr.buf[j]);
            if (pr.rendered[j]) hipEventDestroy(pr.rendered[j]);
        }
        if (pr.dense) hipFree(pr.dense);
        if (pr.accum) hipFree(pr.accum);
    }
    if (!ctx->members.empty()) hipSetDevice(ctx->members[0]->device);
    for (size_t i = 1; i < ctx->peers.size(); ++i)
        for (int j = 0; j < 2; ++j)
            if (ctx->peers[i].local[j]) hipFree(ctx->peers[i].local[j]);
    for (int j = 0; j < 2; ++j)
        if (ctx->gathered[j]) hipEventDestroy(ctx->gathered[j]);
    for (svo_ctx *m : ctx->members) destroy_single(m);
    delete ctx;
    return SVO_OK;
}

}  // extern "C"
