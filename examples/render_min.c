/*
 * render_min.c -- the plugin driven from plain C, no Python or torch: what a
 * native host (the Unity P/Invoke shim) does through
 * include/svo_rt.h.
 *
 * Scene: a one-level SVO (the root's 8 children are all solid leaves), i.e. the
 * whole [-16, 16]^3 world cube; camera at (0, 0, -40) looking down +z with a
 * 60-degree vertical field of view (Unity's GL perspective and camera-to-world
 * = TRS * diag(1, 1, -1, 1), column-major like Matrix4x4).  The centre ray hits
 * the cube face z = -16 after ~24 world units, so bestHit.distance ~ 24 * 64 =
 * 1536 (NVIDIASVO.compute:163,171), in a leaf of the root (hit scale 22) with
 * the root's normal (0, 0, -1) (attachment normal code 0xC000,
 * AttachmentLookup.compute:37-61).
 *
 *   gcc -O2 -Iinclude examples/render_min.c -Lraytracingtest_amd -lsvo_rt \
 *       -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/raytracingtest_amd -o render_min
 *   ./render_min [out.ppm]     exit status 0 = the checks passed
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "svo_rt.h"

#define W 64
#define H 64

static int check(int rc, const char *what) {
    if (rc != SVO_OK) {
        fprintf(stderr, "%s failed (%d): %s\n", what, rc, svo_last_error());
        exit(1);
    }
    return rc;
}

int main(int argc, char **argv) {
    /* descriptor: ptr16 << 16 | valid8 << 8 | nonleaf8 (NaiveCreator.cs:184-187) */
    const int32_t desc[1] = { 0x0000FF00 };
    /* attachment pair: colours A|B (565, R in the low bits), choices | normal16 << 16 */
    const uint32_t att[2] = { 0x001Fu | (0xF800u << 16), 0x0000u | (0xC000u << 16) };

    const float fov = 60.0f * 3.14159265358979f / 180.0f, n = 0.3f, f = 1000.0f, aspect = (float)W / H;
    const float cot = 1.0f / tanf(fov * 0.5f);
    float inv_proj[16] = { 0 };   /* inverse of the GL perspective, column-major m[col * 4 + row] */
    inv_proj[0 * 4 + 0] = aspect / cot;
    inv_proj[1 * 4 + 1] = 1.0f / cot;
    inv_proj[3 * 4 + 2] = -1.0f;
    inv_proj[2 * 4 + 3] = (n - f) / (2.0f * f * n);
    inv_proj[3 * 4 + 3] = (f + n) / (2.0f * f * n);
    float c2w[16] = { 0 };        /* translate (0, 0, -40), scale (1, 1, -1) */
    c2w[0 * 4 + 0] = 1.0f;
    c2w[1 * 4 + 1] = 1.0f;
    c2w[2 * 4 + 2] = -1.0f;
    c2w[3 * 4 + 2] = -40.0f;
    c2w[3 * 4 + 3] = 1.0f;
    const float light[4] = { 0.0f, 0.0f, 1.0f, 1.0f };   /* shining along +z: faces -z lit */

    printf("svo_rt ABI %d\n", svo_abi_version());
    svo_ctx *ctx = NULL;
    check(svo_create(0, 1024, &ctx), "svo_create");
    check(svo_set_buffer(ctx, desc, 1, att, 2, 0), "svo_set_buffer");
    check(svo_set_camera(ctx, c2w, inv_proj, 0.5f, 0.5f, light), "svo_set_camera");
    float *rgba = (float *)malloc(sizeof(float) * 4 * W * H);
    svo_hit *hits = (svo_hit *)malloc(sizeof(svo_hit) * W * H);
    check(svo_render(ctx, W, H, SVO_STACK_HLSL, rgba, hits), "svo_render");

    int n_hit = 0;
    for (int i = 0; i < W * H; ++i) n_hit += hits[i].flags & 1;
    const svo_hit c = hits[(H / 2) * W + W / 2];
    printf("hits %d of %d; centre: parent %u idx %u scale %u t %.3f n (%.3f %.3f %.3f) rgb (%.3f %.3f %.3f)\n",
           n_hit, W * H, c.parent, c.hit_idx, c.hit_scale, c.t, c.nx, c.ny, c.nz, rgba[((H / 2) * W + W / 2) * 4],
           rgba[((H / 2) * W + W / 2) * 4 + 1], rgba[((H / 2) * W + W / 2) * 4 + 2]);
    /* the centre ray is slightly off-axis (pixel centre): 24 / d.z world units, x 64 */
    int ok = (c.flags & 1) && c.parent == 0 && c.hit_scale == 22 && c.t > 1536.0f && c.t < 1536.5f &&
             c.nx == 0.0f && c.ny == 0.0f && c.nz == -1.0f;
    /* the cube face spans ~2 * atan(16/24) = 67 degrees > the 60-degree view: every ray hits */
    ok = ok && n_hit == W * H;

    /* OnRenderImage end to end (svo_render_progressive): two samples at the same pixel
     * offset accumulate to the sample itself, so the display words are the packed Result */
    uint32_t *rgba8 = (uint32_t *)malloc(sizeof(uint32_t) * W * H);
    for (uint32_t sample = 0; sample < 2; ++sample)
        check(svo_render_progressive(ctx, W, H, SVO_STACK_HLSL, sample, rgba8, NULL), "svo_render_progressive");
    int bad8 = 0;
    for (int i = 0; i < W * H; ++i) {
        uint32_t want = 255u << 24;
        for (int k = 0; k < 3; ++k) {
            float v = fminf(fmaxf(rgba[i * 4 + k], 0.0f), 1.0f) * 255.0f;
            want |= (uint32_t)(v + 0.5f) << (8 * k);
        }
        bad8 += rgba8[i] != want;
    }
    printf("progressive: %d display words differ\n", bad8);
    ok = ok && bad8 == 0;

    /* the same frame split over a two-member multi-device context (device 0 twice:
     * the bands of member 1 travel as a payload and are assembled on member 0) */
    const int devs[2] = { 0, 0 };
    svo_ctx *multi = NULL;
    check(svo_create_multi(devs, 2, 1024, 8, &multi), "svo_create_multi");
    check(svo_set_buffer(multi, desc, 1, att, 2, 0), "svo_set_buffer (multi)");
    check(svo_set_camera(multi, c2w, inv_proj, 0.5f, 0.5f, light), "svo_set_camera (multi)");
    svo_hit *hits2 = (svo_hit *)malloc(sizeof(svo_hit) * W * H);
    check(svo_render(multi, W, H, SVO_STACK_HLSL, NULL, hits2), "svo_render (multi)");
    const int same = memcmp(hits, hits2, sizeof(svo_hit) * W * H) == 0;
    printf("multi-device frame %s the single-device frame\n", same ? "equals" : "DIFFERS FROM");
    ok = ok && same;
    check(svo_destroy(multi), "svo_destroy (multi)");
    free(hits2);
    free(rgba8);

    if (argc > 1) {   /* the Result texture as a PPM */
        FILE *fp = fopen(argv[1], "wb");
        if (fp) {
            fprintf(fp, "P6\n%d %d\n255\n", W, H);
            for (int y = H - 1; y >= 0; --y)
                for (int x = 0; x < W; ++x)
                    for (int k = 0; k < 3; ++k) {
                        float v = rgba[(y * W + x) * 4 + k];
                        fputc((int)(fminf(fmaxf(v, 0.0f), 1.0f) * 255.0f + 0.5f), fp);
                    }
            fclose(fp);
        }
    }
    free(rgba);
    free(hits);
    check(svo_destroy(ctx), "svo_destroy");
    printf(ok ? "render_min: ok\n" : "render_min: CHECK FAILED\n");
    return ok ? 0 : 2;
}
