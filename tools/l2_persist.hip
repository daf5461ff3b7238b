// Does a kernel find the node pool's lines in L2 that the previous launch left there?
// (the lone heaviest wave's trip waits ~600 cycles on its node fetch.)
// One wave, lane 0, chases a dependent chain of loads through a 4 MiB array (512-byte steps,
// so the 32 KB vector L1 cannot hold the chain): pass 1 of a launch reads lines the previous
// launch's pass touched; pass 2 of the same launch reads them again (L2-warm for certain).
// A first launch after a host write shows the cold (Infinity Cache / HBM) latency.
//   hipcc --offload-arch=gfx950 -O3 -o l2_persist tools/l2_persist.hip && ./l2_persist
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr int N_WORDS = (4 << 20) / 4;     // 4 MiB of uint32
constexpr int STEP = 512 / 4;              // 512 bytes
constexpr int HOPS = 2048;                 // 1 MiB of the array touched per pass

__global__ void chase(const uint32_t *__restrict__ a, unsigned long long *out, uint32_t start) {
    if (threadIdx.x != 0) return;
    uint32_t i = start;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < HOPS; ++k) i = a[i];
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < HOPS; ++k) i = a[i];
    unsigned long long t2 = __builtin_amdgcn_s_memtime();
    out[0] = t1 - t0;
    out[1] = t2 - t1;
    out[2] = i;   // keeps the chain live
}

int main() {
    std::vector<uint32_t> h(N_WORDS);
    for (int i = 0; i < N_WORDS; ++i) h[i] = (uint32_t)((i + STEP) % N_WORDS);
    uint32_t *d;
    unsigned long long *o;
    CHECK(hipMalloc(&d, N_WORDS * sizeof(uint32_t)));
    CHECK(hipMalloc(&o, 3 * sizeof(unsigned long long)));
    CHECK(hipMemcpy(d, h.data(), N_WORDS * sizeof(uint32_t), hipMemcpyHostToDevice));
    unsigned long long r[3];
    for (int launch = 0; launch < 6; ++launch) {
        hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, d, o, 0u);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost));
        std::printf("launch %d: pass 1 (lines the previous launch read) %.0f cycles/load, "
                    "pass 2 (same launch, L2-warm) %.0f cycles/load\n",
                    launch, (double)r[0] / HOPS, (double)r[1] / HOPS);
    }
    return 0;
}
