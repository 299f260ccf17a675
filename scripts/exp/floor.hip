// Launch / memory-latency floor probes for the step kernel (profiling only).
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void k_empty(int n) {}

// one dependent round trip: every wave loads its 5 robot words + 50 package
// words and writes the robot words back (the step's minimal memory shape)
__global__ __launch_bounds__(256) void k_rt1(const uint32_t* __restrict__ rob, const uint64_t* __restrict__ pkg,
                                             uint32_t* __restrict__ rob_out, int n, int A, int P) {
    const int w = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    if (w >= n) return;
    uint32_t r = lane < A ? rob[(size_t)w * A + lane] : 0u;
    uint64_t p = lane < P ? pkg[(size_t)w * P + lane] : 0ull;
    r += (uint32_t)p;
    if (lane < A) rob_out[(size_t)w * A + lane] = r;
}

// two dependent round trips (second load address from the first's data)
__global__ __launch_bounds__(256) void k_rt2(const uint32_t* __restrict__ rob, const uint64_t* __restrict__ pkg,
                                             const uint8_t* __restrict__ tab, uint32_t* __restrict__ rob_out, int n,
                                             int A, int P) {
    const int w = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    if (w >= n) return;
    uint32_t r = lane < A ? rob[(size_t)w * A + lane] : 0u;
    uint64_t p = lane < P ? pkg[(size_t)w * P + lane] : 0ull;
    r += (uint32_t)p;
    r += tab[r & 255];
    if (lane < A) rob_out[(size_t)w * A + lane] = r;
}

extern "C" {
int exp_empty(int n, hipStream_t s) {
    hipLaunchKernelGGL(k_empty, dim3((n + 3) / 4), dim3(256), 0, s, n);
    return (int)hipGetLastError();
}
int exp_rt1(const void* rob, const void* pkg, void* out, int n, int A, int P, hipStream_t s) {
    hipLaunchKernelGGL(k_rt1, dim3((n + 3) / 4), dim3(256), 0, s, (const uint32_t*)rob, (const uint64_t*)pkg,
                       (uint32_t*)out, n, A, P);
    return (int)hipGetLastError();
}
int exp_rt2(const void* rob, const void* pkg, const void* tab, void* out, int n, int A, int P, hipStream_t s) {
    hipLaunchKernelGGL(k_rt2, dim3((n + 3) / 4), dim3(256), 0, s, (const uint32_t*)rob, (const uint64_t*)pkg,
                       (const uint8_t*)tab, (uint32_t*)out, n, A, P);
    return (int)hipGetLastError();
}
}
