// filler.hip -- diagnostics: what slows the heaviest wave inside a full frame?  A filler kernel
// occupies ~7 of the 8 wave slots of every SIMD for a fixed time while a lone tile row renders
// beside it (tools/contention_ab.py), so the row's waves share their SIMD and memory path with
// one kind of load at a time:
//   mode 1: VALU only (four independent v_fma_f32 chains per lane, no memory);
//   mode 2: dependent 8-byte gathers over an L1-resident table (vector L1 / TA traffic);
//   mode 3: dependent 8-byte gathers over a 2 MB table (L2 traffic).
// Every wave exits once `ticks` of the 100 MHz constant clock have passed (s_memrealtime), so the
// grid always drains.  The only store is lane 0's ordinary vector store of a checksum.
//
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/build/libfiller.so tools/filler.hip
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ __launch_bounds__(64) void filler_kernel(int mode, unsigned long long ticks, const uint2 *__restrict__ table,
                                                    uint32_t mask, float *sink) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t lane = threadIdx.x;
    float a0 = (float)lane, a1 = a0 + 1.0f, a2 = a0 + 2.0f, a3 = a0 + 3.0f;
    uint32_t idx = (blockIdx.x * 64u + lane * 7u) & mask;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        if (mode == 1) {
            for (int i = 0; i < 32; ++i) {
                a0 = __builtin_fmaf(a0, 1.0001f, 0.5f);
                a1 = __builtin_fmaf(a1, 0.9999f, 0.25f);
                a2 = __builtin_fmaf(a2, 1.0002f, 0.125f);
                a3 = __builtin_fmaf(a3, 0.9998f, 0.0625f);
            }
        } else {
            for (int i = 0; i < 8; ++i) idx = (table[idx].x + lane * 3u) & mask;
        }
    }
    if (lane == 0) sink[blockIdx.x] = a0 + a1 + a2 + a3 + (float)idx;
}

extern "C" int filler_launch(int mode, int waves, unsigned long long ticks, const void *table, unsigned mask,
                             void *sink, void *stream) {
    hipLaunchKernelGGL(filler_kernel, dim3(waves), dim3(64), 0, (hipStream_t)stream, mode, ticks,
                       (const uint2 *)table, (uint32_t)mask, (float *)sink);
    return (int)hipGetLastError();
}
