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

// the same round trip with the step kernel's 544-byte by-value argument block,
// reading fields from four of its cache lines
struct Big {
    int n, A, P, pad0;
    uint64_t pad1[60];
    const uint32_t* rob;
    const uint64_t* pkg;
    uint32_t* out;
    uint64_t pad2[4];
};
__global__ __launch_bounds__(256) void k_rt1_big(Big b) {
    const int w = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    if (w >= b.n) return;
    uint32_t r = lane < b.A ? b.rob[(size_t)w * b.A + lane] : 0u;
    uint64_t p = lane < b.P ? b.pkg[(size_t)w * b.P + lane] : 0ull;
    r += (uint32_t)p + (uint32_t)b.pad1[20] + (uint32_t)b.pad1[40];
    if (lane < b.A) b.out[(size_t)w * b.A + lane] = r;
}
extern "C" int exp_rt1_big(const void* rob, const void* pkg, void* out, int n, int A, int P, hipStream_t s) {
    Big b{};
    b.n = n; b.A = A; b.P = P; b.rob = (const uint32_t*)rob; b.pkg = (const uint64_t*)pkg; b.out = (uint32_t*)out;
    hipLaunchKernelGGL(k_rt1_big, dim3((n + 3) / 4), dim3(256), 0, s, b);
    return (int)hipGetLastError();
}

// instruction-cache probe: 2048 dependent VALU ops straight-line (8 KB of code)
// vs the same count as 128 trips of a 16-op loop body
__global__ __launch_bounds__(256) void k_icache_line(uint32_t* out, int n) {
    const int w = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (w >= n) return;
    uint32_t x = threadIdx.x;
    asm volatile(".rept 2048\n v_add_u32 %0, %0, %0\n .endr" : "+v"(x));
    if (x == 12345u) out[w] = x;
}
__global__ __launch_bounds__(256) void k_icache_loop(uint32_t* out, int n) {
    const int w = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (w >= n) return;
    uint32_t x = threadIdx.x;
    for (int i = 0; i < 128; i++) asm volatile(".rept 16\n v_add_u32 %0, %0, %0\n .endr" : "+v"(x));
    if (x == 12345u) out[w] = x;
}
extern "C" int exp_icache(int which, void* out, int n, hipStream_t s) {
    if (which == 0) hipLaunchKernelGGL(k_icache_line, dim3((n + 3) / 4), dim3(256), 0, s, (uint32_t*)out, n);
    else hipLaunchKernelGGL(k_icache_loop, dim3((n + 3) / 4), dim3(256), 0, s, (uint32_t*)out, n);
    return (int)hipGetLastError();
}

// SALU throughput probe: 2048 independent-ish SALU ops per wave (4 chains)
__global__ __launch_bounds__(256) void k_salu(uint32_t* out, int n) {
    const int w = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (w >= n) return;
    uint32_t a = w, b = w + 1, c = w + 2, d = w + 3;
    for (int i = 0; i < 128; i++)
        asm volatile(".rept 4\n s_add_u32 %0, %0, %1\n s_add_u32 %1, %1, %2\n s_add_u32 %2, %2, %3\n s_add_u32 %3, %3, %0\n .endr"
                     : "+s"(a), "+s"(b), "+s"(c), "+s"(d));
    if ((a ^ b ^ c ^ d) == 12345u) out[w] = a;
}
// mixed: 1024 VALU + 1024 SALU interleaved
__global__ __launch_bounds__(256) void k_mixed(uint32_t* out, int n) {
    const int w = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (w >= n) return;
    uint32_t a = w, b = w + 1;
    uint32_t x = threadIdx.x, y = threadIdx.x + 7;
    for (int i = 0; i < 128; i++)
        asm volatile(".rept 4\n s_add_u32 %0, %0, %1\n v_add_u32 %2, %2, %3\n s_add_u32 %1, %1, %0\n v_add_u32 %3, %3, %2\n .endr"
                     : "+s"(a), "+s"(b), "+v"(x), "+v"(y));
    if ((a ^ b ^ x ^ y) == 12345u) out[w] = a;
}
extern "C" int exp_salu(int which, void* out, int n, hipStream_t s) {
    if (which == 0) hipLaunchKernelGGL(k_salu, dim3((n + 3) / 4), dim3(256), 0, s, (uint32_t*)out, n);
    else hipLaunchKernelGGL(k_mixed, dim3((n + 3) / 4), dim3(256), 0, s, (uint32_t*)out, n);
    return (int)hipGetLastError();
}
