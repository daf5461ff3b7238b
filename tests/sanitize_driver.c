/* TEST INFRASTRUCTURE: drives the CPU oracle (oracle/svo_oracle.c) from a plain C
 * process so that it can run under -fsanitize=address,undefined and
 * -fsanitize=thread (race detection / sanitizers on host code; GPU
 * sanitizers are not available on the pool).  tests/test_sanitizers.py builds it.
 *
 * Input file: u32 n_nodes, i32 width, i32 height, i32 mode, i32 nthreads,
 *             orc_camera (raw), int32 desc[n_nodes], u32 att[2 * n_nodes].
 * Output file: orc_hit[width * height] then float rgba[4 * width * height]. */
#include <stdio.h>
#include <stdlib.h>

#include "svo_oracle.h"

static int rd(FILE *f, void *p, size_t n) { return fread(p, 1, n, f) == n; }

int main(int argc, char **argv) {
    if (argc != 3) { fprintf(stderr, "usage: %s in out\n", argv[0]); return 2; }
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    uint32_t n;
    int32_t w, h, mode, nthreads;
    orc_camera cam;
    if (!rd(f, &n, 4) || !rd(f, &w, 4) || !rd(f, &h, 4) || !rd(f, &mode, 4) || !rd(f, &nthreads, 4) ||
        !rd(f, &cam, sizeof cam)) return 3;
    int32_t *desc = malloc((size_t)n * 4);
    uint32_t *att = malloc((size_t)n * 8);
    if (!desc || !att || !rd(f, desc, (size_t)n * 4) || !rd(f, att, (size_t)n * 8)) return 3;
    fclose(f);
    orc_svo svo = {ORC_FMT_V1, desc, NULL, n, att};
    const size_t px = (size_t)w * (size_t)h;
    orc_hit *hits = malloc(px * sizeof(orc_hit));
    float *rgba = malloc(px * 4 * sizeof(float));
    uint32_t *fetch = malloc(px * sizeof(uint32_t));
    if (!hits || !rgba || !fetch) return 4;
    orc_render(&svo, &cam, w, h, 0, h, mode, nthreads, hits, rgba, fetch);
    FILE *o = fopen(argv[2], "wb");
    if (!o) return 5;
    fwrite(hits, sizeof(orc_hit), px, o);
    fwrite(rgba, sizeof(float), px * 4, o);
    fclose(o);
    free(desc); free(att); free(hits); free(rgba); free(fetch);
    return 0;
}
