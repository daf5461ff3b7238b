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
 *  - one context is driven from one host thread at a time; its asynchronous
 *    entry points take any hipStream_t, and renders on different streams run
 *    concurrently (per-stream dispatch-order state).
 *  - a caller stream handed to a context may be destroyed after
 *    svo_forget_stream(ctx, stream), svo_synchronize(ctx) or svo_destroy(ctx):
 *    until one of them, the context may record an event on it (when a fifth
 *    stream takes its dispatch-order state over, or another stream takes the
 *    host-path scratch).  After svo_synchronize no work is pending anywhere, so
 *    the context records nothing on a stream it saw before that call.
 *  - policy (dispatch order, loop form, segmented rays, beam starts, shadow and
 *    readback forms) is one svo_config per context, svo_set_config; no
 *    environment variable changes what the library computes or how (four
 *    diagnostic switches only add traces and timing aids: INTEGRATION.md).
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

/* Compact per-pixel record, 12 bytes = the first 12 bytes of svo_hit: what moves
 * between devices when a frame is split.  The display device rebuilds the normal
 * and the Result colour from it with its own SVO replica and camera (the normal
 * is a function of `parent` alone, NVIDIASVO.compute:177-182). */
typedef struct svo_hit_compact {
    uint32_t parent;
    uint32_t meta;       /* hit_idx | hit_scale << 8 | flags << 16 (svo_hit bytes 4..7) */
    float    t;
} svo_hit_compact;

/* Row split of one frame across ranks/GPUs: rows are grouped in bands of
 * `band_rows`; round-robin (cycle 0) band b belongs to rank b % band_count;
 * a weighted deal (0 < cycle <= 256) gives band b to rank owner[b % cycle]
 * (owner: `cycle` entries, each < band_count), e.g. fewer bands to the display
 * rank, which also assembles the frame.  A rank's output holds only its own rows,
 * in increasing y.  {1, 0, 1} (or NULL) = whole frame. */
typedef struct svo_band {
    int band_rows;
    int band_rank;
    int band_count;
    int cycle;                /* 0: round-robin */
    const uint8_t *owner;     /* cycle > 0: owner[b % cycle] = rank of band b */
} svo_band;

/* Every per-pixel output of one render (device pointers on the context's
 * device, each nullable).  layout SVO_LAYOUT_BAND: buffers hold only the rows of
 * the render's band, in increasing y (the whole frame without a band);
 * SVO_LAYOUT_FRAME: full-frame buffers, this band's rows written in place. */
enum { SVO_LAYOUT_BAND = 0, SVO_LAYOUT_FRAME = 1 };
typedef struct svo_frame {
    svo_hit *hits;             /* 24-byte hit records */
    float *rgba;               /* RGBA32F Result (RaytraceCompute.compute:167) */
    uint32_t *rgba8;           /* display RGBA8: R | G << 8 | B << 16 | 255 << 24, each
                                  channel (uint)(saturate(c) * 255 + 0.5) */
    svo_hit_compact *compact;  /* 12-byte records */
    float *position;           /* float4 per pixel: bestHit.position (NVIDIASVO.compute:165-174),
                                  w = 0; misses 0 (CreateRayHit, RaytraceCompute.compute:33-41) */
    uint64_t *voxel;           /* voxel key x | y << 21 | z << 42 of the hit leaf (integer voxel
                                  coordinates at the leaf scale, un-mirrored; unique for depth <= 21);
                                  misses all ones */
    uint8_t *rgb8;             /* display RGB, 3 bytes per pixel (R, G, B): the RGBA8 word without
                                  its constant alpha -- the dense band payload of a split frame */
    uint64_t *hitmask;         /* one word per 8x8 tile of the render's rows (band-local tiles, row-major,
                                  ceil(W/8) per tile row): bit (y%8)*8 + x%8 set = that pixel hit a
                                  voxel (the wave's ballot) -- the head of a sparse band payload */
    int layout;
} svo_frame;

/* Render policy of a context (ABI 10) -- the plugin's counterpart of RaytracingMaster's
 * Inspector fields (RaytracingMaster.cs:16-18): every switch that chooses HOW a frame is
 * traced.  None changes a result: every combination renders bit-identical frames (the GPU
 * suite runs the oracle comparison under each); they move only time.  Versioned by size: a
 * caller sets `size` = sizeof(svo_config) as it was compiled, svo_set_config reads the fields
 * that fit in it and keeps the context's values of any later ones, svo_get_config writes at
 * most `size` bytes.  svo_get_config(NULL, cfg) gives the defaults below.  Hex tables: one
 * nibble per cost class (lowest = heaviest: >= 7/8, 3/4, 1/2, 1/4, 1/8 of the heaviest tile,
 * rest), each 0 (whole tiles), 4 or 8 (t-segments per ray). */
#define SVO_CONFIG_VERSION 2
typedef struct svo_config {
    uint32_t size;               /* sizeof(svo_config) as compiled by the caller */
    uint32_t version;            /* SVO_CONFIG_VERSION (written by svo_get_config) */
    /* dispatch order */
    int32_t  tile_order;         /* 1: heaviest cost class first, from earlier launches' tile costs; 0: strip order */
    int32_t  xcd_strips;         /* 1: tile columns dealt to the 8 XCDs in interleaved strips; 0: raster */
    int32_t  issue_priority;     /* 1: s_setprio 3/2/1 by cost class */
    int32_t  order_every;        /* >= 1: rebuild the order every k-th launch while costs drift (32) */
    int32_t  move_every;         /* >= 1: while the camera moves, rebuild every k-th launch (4) */
    int32_t  move_spread;        /* 1: a moving camera's order classes a tile by its 3x3 neighbourhood (1) */
    int32_t  relayout;           /* 1: rebuild once in a new class table's own layout (1) */
    int32_t  fetch_all;          /* -1: by pool size (< 2^24 nodes: 1); 0: fetch on a changed node; 1: every trip */
    /* loop form */
    int32_t  loop_form;          /* -1: by the last order build's statistics; 0: lean; 1: latency form */
    float    lat_ratio;          /* latency-bound when summed trips < ratio x resident waves x heaviest (0.3) */
    /* segmented rays */
    int32_t  segments;           /* 1: heavy tiles traced as t-segments by the class tables; 0: never */
    uint32_t seg_table_latency;  /* class table of a latency-bound launch (0x444) */
    uint32_t seg_table_issue;    /* ... of an issue-bound launch (0x4) */
    uint32_t seg_table_thin;     /* ... of a latency-bound launch below seg_thin_ratio (0x888) */
    float    seg_ratio;          /* the latency-bound boundary with beam starts (0.28) */
    float    seg_thin_ratio;     /* the thin boundary (0.083) */
    int32_t  seg_cap;            /* >= 1: segmented tiles per XCD at most (96) */
    int32_t  seg_min_chain;      /* a latency-bound launch whose heaviest tile has fewer trips: no segments (160) */
    int32_t  seg_move;           /* starts after a camera move: 1 the stored ones, 2 even split (2) */
    int32_t  seg_jitter;         /* ... in a jittered launch: 0 no segments, 1 stored, 2 even split (2) */
    int32_t  seg_all;            /* tests: 0 off, 4 or 8 = every tile segmented with that K */
    uint32_t seg_scramble;       /* tests: != 0 replaces every start by a hash (unordered, NaN, +-inf) */
    /* beam starts */
    int32_t  beam;               /* 1: primary rays start at their tile's splatted lower bound of the hit t */
    int32_t  beam_back;          /* >= 0: splat the boxes this many levels above the leaves (2) */
    /* shadow rays (SVO_OPT_SHADOW_RAYS) */
    int32_t  shadow_form;        /* 0: fused into the primary launch; 1: second pass over tiles; 2: over the
                                    compacted hit list */
    int32_t  shadow_order;       /* 1: the two-pass form's tiles in their own cost order */
    /* host paths */
    int32_t  readback;           /* svo_render_progressive_async copy: 0 one DMA, 1 kernel push, 2 two DMAs */
    int32_t  host_copy_threads;  /* svo_render's host copy threads (0: half the hardware threads, <= 16) */
    /* multi-device contexts (svo_create_multi) */
    int32_t  sparse_payload;     /* 1: display-only frames travel as sparse hit payloads */
    int32_t  peer_copy;          /* 1: every member's payload copied instead of pulled over xGMI (tests) */
    /* version 2 */
    int32_t  beam_back_held;     /* a held view (the second launch at a view on a stream and later) re-splats
                                    once with boxes this many levels above the leaves (0); -1: beam_back */
} svo_config;
int svo_get_config(svo_ctx *ctx, svo_config *cfg);
int svo_set_config(svo_ctx *ctx, const svo_config *cfg);

/* ~ RaytracingMaster.InitializeSVOBuffer (RaytracingMaster.cs:111-116):
 * allocate a node pool of `capacity_nodes` descriptors (+2 attachment words
 * each) on HIP device `device`. */
int svo_create(int device, size_t capacity_nodes, svo_ctx **out);

/* Multi-device context (north star: the image sharded into screen bands over
 * the GPUs of one node, the SVO replicated per GPU, the bands gathered to the
 * display GPU over xGMI).  devices[0] is the display device; the same index may
 * repeat (one GPU then renders several members' bands: the test form).  Every
 * other entry point accepts the result: uploads and camera go to every device;
 * svo_render / svo_render_device / svo_render_frame render the whole frame in
 * `band_rows`-row bands dealt round-robin over the devices and leave it on
 * devices[0] (outputs are devices[0] pointers, frame layout).  The reference
 * dispatches one grid over the whole frame (RaytracingMaster.cs:66-68).
 * Payload transport per member (svo_get_member_link): the display device pulls a
 * member's payload over xGMI when hipDeviceCanAccessPeer allows it; when it does
 * not (or svo_config.peer_copy forces it), the member's stream copies the payload
 * into a buffer on the display device (hipMemcpyPeerAsync) and the assemble
 * reads that copy -- creation no longer fails for lack of peer access. */
int svo_create_multi(const int *devices, int num_devices, size_t capacity_nodes, int band_rows, svo_ctx **out);
int svo_num_devices(svo_ctx *ctx, int *num_devices);
/* How member `index`'s band payload reaches the display device: SVO_LINK_SELF
 * (the display device itself, or the same device index), SVO_LINK_PEER (pulled
 * over xGMI with peer access), SVO_LINK_COPY (copied by hipMemcpyPeerAsync).
 * *device = the member's HIP device.  Single-device contexts: index 0, SELF. */
enum { SVO_LINK_SELF = 0, SVO_LINK_PEER = 1, SVO_LINK_COPY = 2 };
int svo_get_member_link(svo_ctx *ctx, int index, int *device, int *link);
/* Weighted band deal for a multi-device context (svo_band.cycle / owner): band b
 * goes to member owner[b % cycle]; e.g. fewer bands for devices[0], which also
 * assembles the frame.  cycle 0 = round-robin (the default). */
int svo_set_band_deal(svo_ctx *ctx, int cycle, const uint8_t *owner);
/* The per-device context `index` of a multi-device context (the context itself
 * for index 0 of a single-device one): owned by the group, not destroyed alone. */
int svo_get_member(svo_ctx *ctx, int index, svo_ctx **member);

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
 * (NULL = the context's own stream).  Asynchronous: returns after enqueue --
 * with one exception: the automatic loop-form choice (svo_config.loop_form -1,
 * the default) waits, once per new static view (the second render after a camera move),
 * for the dispatch-order build of the first one, i.e. for up to one frame of
 * already-enqueued work on that stream.  A caller whose stream waits on something
 * the host signals only after this call returns must set loop_form 0 or 1.  The same
 * holds for svo_render_frame and the renders of svo_render. */
int svo_render_device(svo_ctx *ctx, int width, int height, int stack_mode,
                      const svo_band *band, void *d_rgba, void *d_hits, void *stream);

/* General render: every output of svo_frame, for the rows of `band` (NULL = the
 * whole frame; a multi-device context requires NULL).  Asynchronous. */
int svo_render_frame(svo_ctx *ctx, int width, int height, int stack_mode, const svo_band *band,
                     const svo_frame *frame, void *stream);

/* Samples in flight -- the reference's progressive frame loop (_PixelOffset = (Random.value,
 * Random.value) per frame, RaytracingMaster.cs:35; the AddShader blend with _Sample =
 * _currentSample, then _currentSample++, :70-73, AddShader.shader:44-47), several frames'
 * samples in ONE launch: trace n_samples (1..8) jittered samples of the frame (or of `band`'s
 * rows) -- sample k with _PixelOffset (px_offsets[2k], px_offsets[2k + 1]), the context's
 * camera otherwise -- and blend them in order into d_accum (RGBA32F, band or frame layout as
 * `layout`), sample k with _Sample = first_sample + k.  The blend is svo_accumulate's
 * arithmetic: d_accum ends bit-identical to n_samples single-sample renders each followed by
 * svo_accumulate.  d_rgba8 / d_rgb8 (nullable): the blended pixels' display RGBA8 words /
 * 3-byte RGB (a split frame's band payload).  Primary rays only.  Asynchronous.  One launch
 * holds n_samples waves per 8x8 tile, so a small band's heaviest wave no longer drains alone
 * (DESIGN.md 6.1).  A multi-device context (band NULL, frame layout) splits the frame over
 * its devices: each member blends its own rows into a band accumulation it keeps on its own
 * device (zeroed when the frame size changes), the display device into d_accum's rows of its
 * bands; the members' blended rows travel as 3-byte RGB and d_rgba8 (required; d_rgb8 must be
 * NULL) receives the whole frame's display words. */
int svo_render_samples(svo_ctx *ctx, int width, int height, int stack_mode, const svo_band *band, int n_samples,
                       const float *px_offsets, uint32_t first_sample, float *d_accum, uint32_t *d_rgba8,
                       uint8_t *d_rgb8, int layout, void *stream);

/* Rebuild a split frame on this context's device from its band parts: part m
 * holds the rows of rank m of the deal `deal` (band_count == n_parts; band_rank
 * ignored; round-robin: bands b with b % n_parts == m), band layout, as
 * svo_hit_compact records (SVO_PART_COMPACT: frame
 * outputs hits / rgba / rgba8 / compact, the normal and colour rebuilt from this
 * context's SVO replica and camera), RGBA8 words (SVO_PART_RGBA8) or 3-byte RGB
 * (SVO_PART_RGB8; rows of 3 * width bytes) or sparse hit RGB (SVO_PART_SPARSE_RGB8:
 * svo_pack_hits' layout, read as is -- no scan here; miss pixels get the sky computed
 * here) -- the last three
 * rebuild the frame output rgba8 only.  Part pointers must be readable from this device (its own memory,
 * or a peer's with peer access).  skip_part (or -1): a part already rendered in
 * place.  `frame` must use the frame layout.  This is the display-side half of
 * the one-process-per-GPU split (parts received over RCCL); multi-device
 * contexts use it internally.  Asynchronous. */
enum { SVO_PART_COMPACT = 0, SVO_PART_RGBA8 = 1, SVO_PART_RGB8 = 2, SVO_PART_SPARSE_RGB8 = 3 };
int svo_assemble_frame(svo_ctx *ctx, int width, int height, const svo_band *deal, int n_parts,
                       const void *const *parts, int part_format, int skip_part, const svo_frame *frame,
                       void *stream);

/* Sparse band payload (wave ballot + prefix sum).  Part layout, n_tiles = ceil(W/8) *
 * ceil(rows/8) of the band:
 *   bytes [0, 8 n)             uint64 hit mask per tile (svo_frame.hitmask, written by the render)
 *   bytes [8 n, 12 n + 4)      uint32 hits before each tile, then the band's hit count
 *   bytes [12 n + 4, + 3 count) the 3-byte RGB of every hit pixel, tile by tile in lane order
 * `d_part` holds the masks on entry; this writes the offsets (an exclusive scan of the
 * masks' popcounts) and packs the hits' RGB from `d_rgb8` (the band's dense
 * svo_frame.rgb8).  Allocate SVO_SPARSE_PART_BYTES(n_tiles, band pixels) (its tail
 * beyond the RGB is the scan's scratch, never sent); the part to send is
 * SVO_SPARSE_HEAD_BYTES(n_tiles) + 3 * count bytes, count = the uint32 at byte 12 n.
 * Misses cost nothing -- the display device computes their sky.  Asynchronous. */
#define SVO_SPARSE_HEAD_BYTES(n_tiles) (12u * (size_t)(n_tiles) + 4u)
#define SVO_SPARSE_PART_BYTES(n_tiles, n_px)                                                          \
    (((SVO_SPARSE_HEAD_BYTES(n_tiles) + 3u * (size_t)(n_px) + 3u) & ~(size_t)3) + 4u * (size_t)(n_tiles) + \
     4u * (((size_t)(n_tiles) + 1023u) / 1024u))
int svo_pack_hits(svo_ctx *ctx, int width, int height, const svo_band *band, const void *d_rgb8, void *d_part,
                  void *stream);

/* Instrumented trace: per-ray descriptor-fetch counts (device uint32 array,
 * NVIDIASVO.compute:60-62 executions), used for the algorithmic-bytes figure
 * of the roofline.  Same arguments as svo_render_device plus d_fetches.
 * By default the reference's own walk from the cube entry; with the option
 * SVO_OPT_COUNT_BEAM the walk the render actually runs, from the beam start
 * (DESIGN.md 3.1d). */
int svo_count_fetches(svo_ctx *ctx, int width, int height, int stack_mode,
                      const svo_band *band, void *d_fetches, void *stream);

/* Diagnostics (ABI 10): the start of every primary ray's walk under the current camera -- the
 * beam start of DESIGN.md 3.1d, in SVO-space t (the loop's t_min; the hit record's t is 2048 x
 * that), one float per pixel of `band`'s rows (band layout), -inf where the ray starts at its cube
 * entry.  A record is exact iff no hit lies before its start, so start <= the oracle's hit t on
 * every hit ray is the bound's conservativeness (tests/test_gpu_beam.py).  Asynchronous. */
int svo_beam_starts(svo_ctx *ctx, int width, int height, const svo_band *band, float *d_starts, void *stream);

/* Render options (bit set).  SVO_OPT_SHADOW_RAYS: after the primary pass,
 * trace one shadow ray per hit toward -_DirectionalLight (SURVEY.md 8(d) C3;
 * the reference's shadow test is commented out at RaytraceCompute.compute:105-112):
 * origin = world hit point + 0.001 * normal; an occluded pixel gets hit flag
 * bit 3 and a black Result. */
enum { SVO_OPT_SHADOW_RAYS = 1, SVO_OPT_KERNEL_TIMING = 2, SVO_OPT_COUNT_BEAM = 4 };
int svo_set_options(svo_ctx *ctx, uint32_t options);

/* SVO_OPT_KERNEL_TIMING: every render launch brackets its primary-ray kernel
 * (only that kernel: not the shadow pass, not the dispatch-order kernel) with
 * HIP events on the launch stream.  svo_kernel_time waits for the recorded
 * launches and returns their mean kernel duration in ms and their number, then
 * forgets them.  Measurement only (bench.py's roofline); no reference
 * counterpart. */
int svo_kernel_time(svo_ctx *ctx, double *mean_ms, uint64_t *launches);
/* The same for a stage: SVO_STAGE_KERNEL (= svo_kernel_time) or SVO_STAGE_ASSEMBLE
 * (the assemble kernel of svo_assemble_frame / a multi-device frame).  On a
 * multi-device context every member's recorded launches of the stage are drained
 * and the slowest member's mean is returned (launches: that member's count);
 * svo_get_member gives one device's own figure. */
enum { SVO_STAGE_KERNEL = 0, SVO_STAGE_ASSEMBLE = 1 };
int svo_stage_time(svo_ctx *ctx, int stage, double *mean_ms, uint64_t *launches);
/* Every recorded launch's duration of a stage, in launch order (the first `cap`
 * into ms_out; *launches = how many were recorded), then forgets them like
 * svo_stage_time.  A multi-device context returns devices[0]'s launches and drops
 * the other members' records.  For hosts that watch frame-to-frame variation
 * (a moving camera renders every frame at a new view). */
int svo_stage_times(svo_ctx *ctx, int stage, float *ms_out, size_t cap, size_t *launches);

/* ~ Graphics.Blit(Result, destination, AddMaterial) with _Sample = `sample`
 * (RaytracingMaster.cs:70-73, AddShader.shader:10,44-47): progressive
 * accumulation dst = src * a + dst * (1 - a), a = 1 / (sample + 1), on all four
 * channels (source alpha = a).  d_accum and d_sample are device buffers of
 * n_px RGBA32F pixels (16-byte aligned) on the context's device; `stream` as in
 * svo_render_device.  The caller keeps `sample` (_currentSample): 0 after a
 * camera change (RaytracingMaster.cs:44-47), +1 per frame. */
int svo_accumulate(svo_ctx *ctx, void *d_accum, const void *d_sample, size_t n_px, uint32_t sample,
                   void *stream);

/* ~ RaytracingMaster.OnRenderImage end to end (RaytracingMaster.cs:55-74 with
 * AddShader.shader:44-47): render one sample of the frame at the current camera,
 * blend it into the context's device-resident accumulation frame with
 * _Sample = `sample` (svo_accumulate's blend; the frame is reallocated whenever
 * its size changes, and the first sample after that is blended as sample 0 --
 * it replaces the frame -- whatever `sample` says), and copy the accumulated frame to the host as display RGBA8
 * words (4 B/px, R in the low byte = Unity TextureFormat.RGBA32; each colour
 * channel (uint)(saturate(c) * 255 + 0.5), alpha 255) and/or RGBA32F (16 B/px); either output may be
 * NULL, not both.  Only the accumulated frame crosses PCIe: 8.3 MB per 1080p
 * frame as RGBA8 against 83 MB for svo_render's RGBA32F + hit records.  A
 * multi-device context renders the sample split over its devices and
 * accumulates on devices[0].  Blocking. */
int svo_render_progressive(svo_ctx *ctx, int width, int height, int stack_mode, uint32_t sample,
                           uint32_t *rgba8_out, float *rgba_out);

/* svo_render_progressive for a host that displays every frame (Unity:
 * Texture2D.LoadRawTextureData(IntPtr, int) on the returned pointer, then Apply):
 * enqueue one sample -- render, blend with _Sample = `sample`, pack the accumulated
 * frame to display pixels -- and their copy into plugin-owned pinned host memory on a
 * copy stream, then return in *frame_out the PREVIOUS call's frame (NULL on the first
 * call after creation, a size change or a pixel-format change), waiting only for that
 * frame's copy.  So the D2H of frame k overlaps the render of frame k + 1, and the host
 * never waits for the frame it just asked for.  pixel_format: SVO_PIXELS_RGBA8 (4 B/px,
 * the words of svo_render_progressive's rgba8_out = TextureFormat.RGBA32) or
 * SVO_PIXELS_RGB8 (3 B/px, the same words without their constant alpha =
 * TextureFormat.RGB24: a quarter fewer bytes over PCIe).  A returned pointer (W * H
 * pixels) stays valid until the call after next; the plugin owns it.
 * svo_progressive_last returns the most recent frame, waiting for its copy (the end of a
 * sequence).  The blocking svo_render_progressive stays available. */
enum { SVO_PIXELS_RGBA8 = 0, SVO_PIXELS_RGB8 = 1 };
int svo_render_progressive_async(svo_ctx *ctx, int width, int height, int stack_mode, uint32_t sample,
                                 int pixel_format, const void **frame_out);
int svo_progressive_last(svo_ctx *ctx, const void **frame_out);

/* Information about the uploaded pool. */
int svo_get_info(svo_ctx *ctx, size_t *n_nodes, int *max_depth, int *device);

/* Block until all work of the context has finished: its own stream and every
 * caller stream it rendered, assembled or accumulated on (a device-wide
 * synchronise of each of its devices). */
int svo_synchronize(svo_ctx *ctx);

/* Let go of a caller stream before the caller destroys it: waits for the work the
 * context enqueued on it and frees the stream's dispatch-order state (a multi-device
 * context: every member).  A stream never passed in is not an error.  (ABI 9) */
int svo_forget_stream(svo_ctx *ctx, void *stream);

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
