/*
 * bench_native.c -- the metric's frame timed from a plain C host, no Python and no torch
 * anywhere in the process: what a native engine that keeps its frame in HBM measures
 * through the two C-ABIs (include/svo_build.h, include/svo_rt.h).
 *
 *   svob_build_sampler -> svo_create -> svo_set_buffer_v2 -> svo_set_camera, then K x
 *   svo_render_device (24-byte hit records + RGBA32F Result into hipMalloc'ed buffers, on a
 *   stream of the host's own) between two stream synchronizes, as bench.py's timed region;
 *   SVO_OPT_KERNEL_TIMING + svo_kernel_time for the render kernel's own mean duration.
 *
 *   gcc -O2 -D__HIP_PLATFORM_AMD__ -Iinclude -I/opt/rocm/include examples/bench_native.c \
 *       -Lraytracingtest_amd -lsvo_rt -lsvo_build -L/opt/rocm/lib -lamdhip64 \
 *       -Wl,-rpath,$PWD/raytracingtest_amd -o bench_native
 *   ./bench_native <sampler> <max_level> <camera.bin> <width> <height> [steps] [warmup]
 *
 * camera.bin: as build_and_render.c (camera-to-world[16], inverse projection[16], column-
 * major, then light[4]; float32).  Prints one JSON line.
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "svo_build.h"
#include "svo_rt.h"

static void die(const char *what, int rc, const char *msg) {
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, msg);
    exit(1);
}

static void hip_check(hipError_t e, const char *what) {
    if (e != hipSuccess) {
        fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
        exit(1);
    }
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int main(int argc, char **argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: %s sampler max_level camera.bin width height [steps] [warmup]\n", argv[0]);
        return 2;
    }
    const int sampler = atoi(argv[1]), max_level = atoi(argv[2]);
    const int width = atoi(argv[4]), height = atoi(argv[5]);
    const int steps = argc > 6 ? atoi(argv[6]) : 1000, warmup = argc > 7 ? atoi(argv[7]) : 50;
    if (width <= 0 || height <= 0 || steps <= 0 || warmup < 0) {
        fprintf(stderr, "bad frame size or step count\n");
        return 2;
    }
    float cam[36];
    FILE *cf = fopen(argv[3], "rb");
    if (!cf || fread(cam, sizeof(float), 36, cf) != 36) {
        fprintf(stderr, "cannot read 36 floats from %s\n", argv[3]);
        return 2;
    }
    fclose(cf);

    svob_result svo;
    int rc = svob_build_sampler(0, sampler, max_level, &svo);
    if (rc) die("svob_build_sampler", rc, svob_last_error());
    svo_ctx *ctx = NULL;
    rc = svo_create(0, svo.n_nodes, &ctx);
    if (rc) die("svo_create", rc, svo_last_error());
    rc = svo_set_buffer_v2(ctx, svo.nodes, svo.n_nodes, svo.attachments, 2 * svo.n_nodes, 0);
    if (rc) die("svo_set_buffer_v2", rc, svo_last_error());
    const int stack_mode = svo.n_nodes > ((size_t)1 << 24) ? SVO_STACK_EXACT : SVO_STACK_HLSL;
    rc = svo_set_camera(ctx, cam, cam + 16, 0.5f, 0.5f, cam + 32);
    if (rc) die("svo_set_camera", rc, svo_last_error());

    const size_t px = (size_t)width * (size_t)height;
    void *d_hits = NULL, *d_rgba = NULL;
    hip_check(hipMalloc(&d_hits, px * sizeof(svo_hit)), "hipMalloc hits");
    hip_check(hipMalloc(&d_rgba, px * 4 * sizeof(float)), "hipMalloc rgba");
    hipStream_t s;
    hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");

    for (int i = 0; i < warmup; ++i) {
        rc = svo_render_device(ctx, width, height, stack_mode, NULL, d_rgba, d_hits, (void *)s);
        if (rc) die("svo_render_device", rc, svo_last_error());
    }
    hip_check(hipStreamSynchronize(s), "warmup");
    const double t0 = now_s();
    for (int i = 0; i < steps; ++i) {
        rc = svo_render_device(ctx, width, height, stack_mode, NULL, d_rgba, d_hits, (void *)s);
        if (rc) die("svo_render_device", rc, svo_last_error());
    }
    hip_check(hipStreamSynchronize(s), "timed steps");
    const double dt = now_s() - t0;

    /* the render kernel alone (HIP events around it, as bench.py's roofline), K more steps */
    rc = svo_set_options(ctx, SVO_OPT_KERNEL_TIMING);
    if (rc) die("svo_set_options", rc, svo_last_error());
    double kern_ms = 0.0;
    uint64_t n = 0;
    svo_kernel_time(ctx, &kern_ms, &n);   /* forget anything recorded before */
    for (int i = 0; i < steps; ++i) {
        rc = svo_render_device(ctx, width, height, stack_mode, NULL, d_rgba, d_hits, (void *)s);
        if (rc) die("svo_render_device", rc, svo_last_error());
    }
    rc = svo_kernel_time(ctx, &kern_ms, &n);
    if (rc) die("svo_kernel_time", rc, svo_last_error());
    hip_check(hipStreamSynchronize(s), "timed kernels");

    const double ms = dt / steps * 1e3;
    printf("{\"host\": \"C (examples/bench_native.c)\", \"sampler\": %d, \"max_level\": %d, \"nodes\": %zu, "
           "\"frame\": \"%dx%d\", \"stack_mode\": \"%s\", \"steps\": %d, \"warmup\": %d, \"ms_per_step\": %.4f, "
           "\"Mrays_per_s\": %.2f, \"kernel_ms\": %.4f, \"kernel_launches\": %llu}\n",
           sampler, max_level, svo.n_nodes, width, height, stack_mode == SVO_STACK_EXACT ? "exact" : "hlsl",
           steps, warmup, ms, (double)px / (ms * 1e-3) / 1e6, kern_ms, (unsigned long long)n);
    hip_check(hipStreamDestroy(s), "hipStreamDestroy");
    hip_check(hipFree(d_hits), "hipFree");
    hip_check(hipFree(d_rgba), "hipFree");
    svob_free(&svo);
    rc = svo_destroy(ctx);
    if (rc) die("svo_destroy", rc, svo_last_error());
    return 0;
}
