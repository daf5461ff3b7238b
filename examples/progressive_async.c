/*
 * progressive_async.c -- the Unity host's per-frame loop (RaytracingMaster.OnRenderImage,
 * RaytracingMaster.cs:55-74) from plain C through svo_render_progressive_async: each frame
 * sets a new _PixelOffset (:35), enqueues one sample and gets back the PREVIOUS frame's
 * display words in plugin-owned pinned memory -- what the C# shim hands to
 * Texture2D.LoadRawTextureData(IntPtr, int).  Writes every displayed frame, in order, so a
 * test can compare them with the oracle's accumulation; prints the host time per frame.
 *
 *   progressive_async POOL CAM OFFS W H N OUT [rgb]
 *     POOL: uint32 n_desc, uint32 n_att, int32 desc[n_desc] (NaiveCreator.cs:184-187 words),
 *           uint32 att[n_att]
 *     CAM:  36 floats: c2w[16], inv_proj[16] (Unity column-major), light[4]
 *     OFFS: 2 N floats: _PixelOffset of frame k
 *     OUT:  N frames of W * H uint32 display words (frame k = the accumulation of samples 0..k),
 *           or with `rgb` W * H 3-byte pixels (SVO_PIXELS_RGB8 = TextureFormat.RGB24)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "svo_rt.h"

static void check(int rc, const char *what) {
    if (rc != SVO_OK) {
        fprintf(stderr, "%s failed (%d): %s\n", what, rc, svo_last_error());
        exit(1);
    }
}

static void *slurp(const char *path, size_t *size) {
    FILE *f = fopen(path, "rb");
    if (!f) { perror(path); exit(1); }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    void *buf = malloc((size_t)n);
    if (!buf || fread(buf, 1, (size_t)n, f) != (size_t)n) { fprintf(stderr, "read %s\n", path); exit(1); }
    fclose(f);
    *size = (size_t)n;
    return buf;
}

static double now_ms(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

int main(int argc, char **argv) {
    if (argc != 8 && argc != 9) {
        fprintf(stderr, "usage: %s POOL CAM OFFS W H N OUT [rgb]\n", argv[0]);
        return 2;
    }
    size_t pool_size, cam_size, offs_size;
    uint32_t *pool = slurp(argv[1], &pool_size);
    float *cam = slurp(argv[2], &cam_size);
    float *offs = slurp(argv[3], &offs_size);
    const int w = atoi(argv[4]), h = atoi(argv[5]), n = atoi(argv[6]);
    const uint32_t n_desc = pool[0], n_att = pool[1];
    if (cam_size != 36 * sizeof(float) || offs_size < 2 * (size_t)n * sizeof(float) ||
        pool_size != (2 + (size_t)n_desc + n_att) * 4) {
        fprintf(stderr, "bad input sizes\n");
        return 2;
    }
    const int32_t *desc = (const int32_t *)(pool + 2);
    const uint32_t *att = pool + 2 + n_desc;
    FILE *out = fopen(argv[7], "wb");
    if (!out) { perror(argv[7]); return 1; }

    svo_ctx *ctx = NULL;
    check(svo_create(0, n_desc, &ctx), "svo_create");
    check(svo_set_buffer(ctx, desc, n_desc, att, n_att, 0), "svo_set_buffer");
    const int fmt = argc == 9 && strcmp(argv[8], "rgb") == 0 ? SVO_PIXELS_RGB8 : SVO_PIXELS_RGBA8;
    const size_t frame_bytes = (size_t)w * h * (fmt == SVO_PIXELS_RGB8 ? 3 : 4);
    double t0 = 0.0;
    int written = 0;
    for (int k = 0; k < n; ++k) {
        if (k == 1) t0 = now_ms();   /* frame 0 allocates the accumulation and the pinned slots */
        check(svo_set_camera(ctx, cam, cam + 16, offs[2 * k], offs[2 * k + 1], cam + 32), "svo_set_camera");
        const void *frame = NULL;
        check(svo_render_progressive_async(ctx, w, h, SVO_STACK_HLSL, (uint32_t)k, fmt, &frame),
              "svo_render_progressive_async");
        if ((k == 0) != (frame == NULL)) { fprintf(stderr, "frame %d: unexpected pointer\n", k); return 1; }
        if (frame) {   /* the previous frame (k - 1): consume it as LoadRawTextureData would */
            fwrite(frame, 1, frame_bytes, out);
            ++written;
        }
    }
    const double ms = n > 1 ? (now_ms() - t0) / (n - 1) : 0.0;
    const void *last = NULL;
    check(svo_progressive_last(ctx, &last), "svo_progressive_last");
    if (!last) { fprintf(stderr, "no last frame\n"); return 1; }
    fwrite(last, 1, frame_bytes, out);
    ++written;
    fclose(out);
    check(svo_destroy(ctx), "svo_destroy");
    printf("{\"frames\": %d, \"ms_per_frame\": %.4f, \"width\": %d, \"height\": %d}\n", written, ms, w, h);
    free(pool);
    free(cam);
    free(offs);
    return 0;
}
