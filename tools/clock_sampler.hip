// clock_sampler.hip -- diagnostics: the shader clock over time, beside the renders.
//
// One wave (lane 0 working) samples (s_memrealtime, s_memtime) every `interval`
// ticks of the 100 MHz constant clock, `n` times, into a device buffer of uint64
// pairs; launched on its own stream it runs concurrently with the renders and
// occupies one wave slot of 8,192.  clock = d(memtime) / d(memrealtime) * 100 MHz
// (MI355X_MICROARCH.md "DVFS give-back" item 6).  The loop is bounded by n, so the
// wave always exits.  Stores are ordinary vector stores.
//
//   hipcc --offload-arch=gfx950 -O2 -shared -fPIC -o tools/build/libclock_sampler.so tools/clock_sampler.hip
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ void clock_sampler_kernel(unsigned long long *out, int n, unsigned interval) {
    if (threadIdx.x != 0) return;
    unsigned long long next = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < n; ++i) {
        unsigned long long rt = __builtin_amdgcn_s_memrealtime();
        while (rt < next) {
            __builtin_amdgcn_s_sleep(8);
            rt = __builtin_amdgcn_s_memrealtime();
        }
        const unsigned long long st = __builtin_amdgcn_s_memtime();
        out[2 * i] = rt;
        out[2 * i + 1] = st;
        next = rt + interval;
    }
}

extern "C" int clock_sampler_launch(void *d_out, int n, unsigned interval_ticks, void *stream) {
    hipLaunchKernelGGL(clock_sampler_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                       (unsigned long long *)d_out, n, interval_ticks);
    return (int)hipGetLastError();
}
