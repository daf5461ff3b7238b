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
