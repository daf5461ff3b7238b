// dispatch_rate.hip -- how fast does MI355X start short workgroups?  (diagnostics for
// in the second half of a C3 frame half of the tile waves start while
// resident waves sit at ~6,000 of 8,192, i.e. the wave starts, not free slots, set the pace)
//
// Launches G workgroups of B threads with L bytes of dynamic LDS each; every workgroup
// spins for ~S cycles (s_sleep-free busy loop on s_memtime) and writes one word.  Reports
// the launch time per workgroup and per wave.
//
//   hipcc --offload-arch=gfx950 -O3 tools/dispatch_rate.hip -o build/dispatch_rate && build/dispatch_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void short_wg(unsigned *out, unsigned long long spin) {
    extern __shared__ unsigned lds[];
    lds[threadIdx.x] = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < spin) {
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = lds[blockDim.x - 1] + 1u;
}

static float run(int grid, int block, size_t lds, unsigned long long spin, unsigned *d_out) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(short_wg, dim3(grid), dim3(block), lds, 0, d_out, spin);
    hipEventRecord(a, 0);
    const int reps = 10;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(short_wg, dim3(grid), dim3(block), lds, 0, d_out, spin);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0.0f;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms / reps;
}

int main() {
    unsigned *d_out = nullptr;
    if (hipMalloc(&d_out, 1 << 20) != hipSuccess) return 1;
    struct Case { int grid, block; size_t lds; unsigned long long spin; const char *what; };
    const Case cases[] = {
        {32400, 64, 5120, 0, "C3 tile grid, 1-wave WGs, 5 KB LDS, no work"},
        {32400, 64, 5120, 2000, "  same, ~2000 cycles of work per wave"},
        {32400, 64, 5120, 8000, "  same, ~8000 cycles"},
        {16200, 64, 5120, 0, "half the WGs (2 tiles per wave), no work"},
        {8100, 256, 20480, 0, "4-wave WGs (16x16 tiles), 20 KB LDS, no work"},
        {8100, 256, 20480, 2000, "  same, ~2000 cycles"},
        {32400, 64, 0, 0, "1-wave WGs without LDS, no work"},
    };
    for (const Case &c : cases) {
        const float ms = run(c.grid, c.block, c.lds, c.spin, d_out);
        const int waves = c.grid * (c.block / 64);
        printf("%-48s grid %6d x %3d: %8.2f us  (%.1f WG/us, %.1f waves/us)\n", c.what, c.grid, c.block, ms * 1e3,
               c.grid / (ms * 1e3), waves / (ms * 1e3));
    }
    hipFree(d_out);
    return 0;
}
