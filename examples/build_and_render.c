/*
 * build_and_render.c -- the reference's key-R path from a plain C host:
 * RaytracingMaster.Update -> SetSVOBuffer() (RaytracingMaster.cs:50-52,90-109),
 * i.e. NaiveCreator.Create(SampleFunctions.functions[sampleType], maxLevel) and
 * the upload, then one Render.  What the Unity shim (unity/RaytracingMasterNative.cs)
 * does through the same two C-ABIs:
 *   svob_build_sampler  (include/svo_build.h)  the native NaiveCreator
 *   svo_set_buffer_v2   (include/svo_rt.h)     wide child pointers: every BASELINE
 *                                              config from C2 up overflows the
 *                                              reference's 16-bit relative pointer
 *   svo_get_info        stack mode by pool size: EXACT above 2^24 nodes (the HLSL
 *                       float2 stack rounds parent indices there)
 *   svo_render          RGBA32F Result + 24-byte hit records into host buffers
 *
 *   gcc -O2 -Iinclude examples/build_and_render.c -Lraytracingtest_amd -lsvo_rt -lsvo_build \
 *       -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/raytracingtest_amd -o build_and_render
 *   ./build_and_render <sampler> <max_level> <camera.bin> <width> <height> <hits.bin> [rgba.bin]
 *
 * camera.bin: 36 little-endian float32 -- camera-to-world[16] and inverse
 * projection[16] (column-major, Unity Matrix4x4 order) and the light[4].  The
 * pixel offset is (0.5, 0.5).  Exit status 0 = built, uploaded and rendered.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "svo_build.h"
#include "svo_rt.h"

static void die(const char *what, int rc, const char *msg) {
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, msg);
    exit(1);
}

static void write_all(const char *path, const void *p, size_t n) {
    FILE *f = fopen(path, "wb");
    if (!f || fwrite(p, 1, n, f) != n) {
        fprintf(stderr, "cannot write %s\n", path);
        exit(1);
    }
    fclose(f);
}

int main(int argc, char **argv) {
    if (argc < 7) {
        fprintf(stderr, "usage: %s sampler max_level camera.bin width height hits.bin [rgba.bin]\n", argv[0]);
        return 2;
    }
    const int sampler = atoi(argv[1]), max_level = atoi(argv[2]);
    const int width = atoi(argv[4]), height = atoi(argv[5]);
    float cam[36];
    FILE *cf = fopen(argv[3], "rb");
    if (!cf || fread(cam, sizeof(float), 36, cf) != 36) {
        fprintf(stderr, "cannot read 36 floats from %s\n", argv[3]);
        return 2;
    }
    fclose(cf);

    /* NaiveCreator.Create(sampler, maxLevel) on GPU 0 */
    svob_result svo;
    int rc = svob_build_sampler(0, sampler, max_level, &svo);
    if (rc) die("svob_build_sampler", rc, svob_last_error());

    /* InitializeSVOBuffer + SetSVOBuffer: the V2 upload takes any pool the builder makes */
    svo_ctx *ctx = NULL;
    rc = svo_create(0, svo.n_nodes, &ctx);
    if (rc) die("svo_create", rc, svo_last_error());
    rc = svo_set_buffer_v2(ctx, svo.nodes, svo.n_nodes, svo.attachments, 2 * svo.n_nodes, 0);
    if (rc) die("svo_set_buffer_v2", rc, svo_last_error());
    size_t n_nodes = 0;
    int depth = 0, device = 0;
    rc = svo_get_info(ctx, &n_nodes, &depth, &device);
    if (rc) die("svo_get_info", rc, svo_last_error());
    const int stack_mode = n_nodes > ((size_t)1 << 24) ? SVO_STACK_EXACT : SVO_STACK_HLSL;

    rc = svo_set_camera(ctx, cam, cam + 16, 0.5f, 0.5f, cam + 32);
    if (rc) die("svo_set_camera", rc, svo_last_error());
    const size_t px = (size_t)width * (size_t)height;
    svo_hit *hits = (svo_hit *)malloc(px * sizeof(svo_hit));
    float *rgba = (float *)malloc(px * 4 * sizeof(float));
    if (!hits || !rgba) return 3;
    rc = svo_render(ctx, width, height, stack_mode, rgba, hits);
    if (rc) die("svo_render", rc, svo_last_error());

    size_t n_hit = 0;
    for (size_t i = 0; i < px; ++i) n_hit += hits[i].flags & 1u;
    printf("built sampler %d maxLevel %d: %zu nodes (%zu surface voxels), depth %d, v1 pointers %s; "
           "stack mode %s; %zu of %zu rays hit\n",
           sampler, max_level, n_nodes, svo.n_leaves, depth, svo.v1_ok ? "fit" : "overflow",
           stack_mode == SVO_STACK_EXACT ? "exact" : "hlsl", n_hit, px);
    write_all(argv[6], hits, px * sizeof(svo_hit));
    if (argc > 7) write_all(argv[7], rgba, px * 4 * sizeof(float));
    free(hits);
    free(rgba);
    svob_free(&svo);
    rc = svo_destroy(ctx);
    if (rc) die("svo_destroy", rc, svo_last_error());
    return 0;
}
