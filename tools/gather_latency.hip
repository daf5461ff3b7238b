// gather_latency.hip -- diagnostics: the latency of ONE wave64 gather of 8-byte words (the
// traversal's node fetch, global_load_dwordx2) as a function of how many distinct 128-byte
// lines its 64 lanes touch, for L1-resident and L2-resident footprints.
//
// A dependent chain: every lane of step s loads a word of row r_s -- lane l from line
// (l mod G) of the row's G lines, at 8-byte slot (l / G) mod 16 -- and every word of row r holds
// the next row's index, so step s + 1's addresses depend on step s's data.  Rows are visited
// in a random cycle (no stride for a prefetcher to follow); one warm pass over all rows, then
// the timed pass.  One wave, one workgroup: the lone-wave case of DESIGN.md 5.1.  The loop is
// bounded by `steps`; lane 0 stores the result with an ordinary vector store.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/build/gather_latency tools/gather_latency.hip
//   tools/build/gather_latency
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

constexpr int LINE_WORDS = 16;   // uint2 words per 128-byte line

__global__ __launch_bounds__(64) void chase(const uint2 *__restrict__ buf, int lines_per_row, int rows, int steps,
                                            unsigned long long *out) {
    const int l = threadIdx.x;
    const uint32_t lane_off = (uint32_t)((l % lines_per_row) * LINE_WORDS + (l / lines_per_row) % LINE_WORDS);
    uint32_t r = 0;
    // warm pass: every row once
    for (int s = 0; s < rows; ++s) r = buf[r * (uint32_t)lines_per_row * LINE_WORDS + lane_off].x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < steps; ++s) r = buf[r * (uint32_t)lines_per_row * LINE_WORDS + lane_off].x;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) {
        out[0] = t1 - t0;
        out[1] = r;   // keeps the chain live
    }
}

int main() {
    const int G[] = {1, 2, 4, 8, 16, 32, 64};
    const size_t footprints[] = {16u << 10, 2u << 20};   // L1-resident (vL1D 32 KB), L2-resident (4 MB per XCD)
    std::mt19937 rng(7);
    unsigned long long *d_out;
    if (hipMalloc(&d_out, 16) != hipSuccess) return 1;
    std::printf("footprint  lines/gather  cycles/step (s_memtime)\n");
    for (size_t fp : footprints) {
        for (int g : G) {
            const int rows = (int)(fp / (128u * (size_t)g));
            if (rows < 2) continue;
            std::vector<uint32_t> perm(rows);
            std::iota(perm.begin(), perm.end(), 0u);
            std::shuffle(perm.begin() + 1, perm.end(), rng);   // one cycle through every row, from row 0
            std::vector<uint2> h((size_t)rows * g * LINE_WORDS);
            for (int i = 0; i < rows; ++i) {
                const uint32_t next = perm[(i + 1) % rows];
                for (int w = 0; w < g * LINE_WORDS; ++w) h[(size_t)perm[i] * g * LINE_WORDS + w] = make_uint2(next, 0u);
            }
            uint2 *d;
            if (hipMalloc(&d, h.size() * sizeof(uint2)) != hipSuccess) return 1;
            hipMemcpy(d, h.data(), h.size() * sizeof(uint2), hipMemcpyHostToDevice);
            const int steps = 4 * rows > 4096 ? 4096 : 4 * rows;
            unsigned long long res[2] = {0, 0};
            double best = 1e30;
            for (int rep = 0; rep < 3; ++rep) {
                hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, d, g, rows, steps, d_out);
                if (hipDeviceSynchronize() != hipSuccess) return 2;
                hipMemcpy(res, d_out, 16, hipMemcpyDeviceToHost);
                best = std::min(best, (double)res[0] / steps);
            }
            std::printf("%8zu KB  %12d  %8.1f\n", fp >> 10, g, best);
            hipFree(d);
        }
    }
    hipFree(d_out);
    return 0;
}
