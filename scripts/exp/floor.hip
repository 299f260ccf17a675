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

// kernel-argument cache-line probe: the round trip of k_rt1 after reading NL
// distinct 64-byte lines of a 576-byte argument block (values pinned in SGPRs)
struct KLines {
    uint64_t line[9][8];  // 9 lines of 64 B
};
template <int NL>
__global__ __launch_bounds__(256) void k_klines(KLines k, const uint32_t* __restrict__ rob,
                                                uint32_t* __restrict__ out, int n) {
    const int w = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < NL; i++) {
        uint64_t v = k.line[i][i % 8];
        asm volatile("" : "+s"(v));
        acc += v;
    }
    if (w >= n) return;
    uint32_t r = lane < 5 ? rob[(size_t)w * 5 + lane] : 0u;
    r += (uint32_t)acc;
    if (lane < 5) out[(size_t)w * 5 + lane] = r;
}
extern "C" int exp_klines(int nl, const void* rob, void* out, int n, hipStream_t s) {
    KLines k{};
    switch (nl) {
        case 1: hipLaunchKernelGGL(k_klines<1>, dim3((n + 3) / 4), dim3(256), 0, s, k, (const uint32_t*)rob, (uint32_t*)out, n); break;
        case 3: hipLaunchKernelGGL(k_klines<3>, dim3((n + 3) / 4), dim3(256), 0, s, k, (const uint32_t*)rob, (uint32_t*)out, n); break;
        case 6: hipLaunchKernelGGL(k_klines<6>, dim3((n + 3) / 4), dim3(256), 0, s, k, (const uint32_t*)rob, (uint32_t*)out, n); break;
        default: hipLaunchKernelGGL(k_klines<9>, dim3((n + 3) / 4), dim3(256), 0, s, k, (const uint32_t*)rob, (uint32_t*)out, n); break;
    }
    return (int)hipGetLastError();
}

// v_readlane cost probe: 64 independent readlanes (into SGPRs, summed by SALU)
__global__ __launch_bounds__(256) void k_rl(uint32_t* out, int n, int reps) {
    const int w = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (w >= n) return;
    int x = threadIdx.x * 7 + w;
    int acc = 0;
    for (int r = 0; r < reps; r++) {
#pragma unroll
        for (int j = 0; j < 64; j++) acc += __builtin_amdgcn_readlane(x, j);
        x += acc;
    }
    if ((threadIdx.x & 63) == 0) out[w] = acc;
}
// same count of v_add (independent pairs) for scale
__global__ __launch_bounds__(256) void k_va(uint32_t* out, int n, int reps) {
    const int w = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (w >= n) return;
    int x = threadIdx.x * 7 + w, y = x + 1;
    for (int r = 0; r < reps; r++) {
#pragma unroll
        for (int j = 0; j < 32; j++) asm volatile("v_add_u32 %0, %0, %1\n v_add_u32 %1, %1, %0" : "+v"(x), "+v"(y));
    }
    if (x == 12345) out[w] = y;
}
extern "C" int exp_rl(int which, void* out, int n, int reps, hipStream_t s) {
    if (which == 0) hipLaunchKernelGGL(k_rl, dim3((n + 3) / 4), dim3(256), 0, s, (uint32_t*)out, n, reps);
    else hipLaunchKernelGGL(k_va, dim3((n + 3) / 4), dim3(256), 0, s, (uint32_t*)out, n, reps);
    return (int)hipGetLastError();
}

// dependency-latency probes: 64 chained pairs per rep (inline asm, exact sequences)
#define PROBE(name, body, ...)                                                                  \
    __global__ __launch_bounds__(256) void name(uint32_t* out, int n, int reps) {                \
        const int w = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  \
        if (w >= n) return;                                                                      \
        int v1 = threadIdx.x, v2 = threadIdx.x * 3;                                              \
        int s10 = w, s11 = w + 1;                                                                \
        for (int r = 0; r < reps; r++) asm volatile(".rept 64\n" body "\n.endr" __VA_ARGS__ : : "scc");           \
        if (v1 == 123456) out[w] = v2 + s10 + s11;                                               \
    }
// P1 VALU(readlane)->SALU
PROBE(k_p1, "v_readlane_b32 %2, %0, 3\n s_add_u32 %3, %3, %2", : "+v"(v1), "+v"(v2), "+s"(s10), "+s"(s11))
// P2 readlane->VALU use (full loop-carried chain through v1)
PROBE(k_p2, "v_readlane_b32 %2, %0, 3\n v_add_u32 %0, %2, %0", : "+v"(v1), "+v"(v2), "+s"(s10), "+s"(s11))
// P3 SALU->VALU->SALU chain: v_add reads s10, readlane writes s10, s_add
PROBE(k_p3, "s_add_u32 %2, %2, 1\n v_add_u32 %0, %2, %0", : "+v"(v1), "+v"(v2), "+s"(s10), "+s"(s11))
// P4 VALU chain
PROBE(k_p4, "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1", : "+v"(v1), "+v"(v2), "+s"(s10), "+s"(s11))
// P5 SALU chain
PROBE(k_p5, "s_add_u32 %2, %2, %3\n s_add_u32 %2, %2, %3", : "+v"(v1), "+v"(v2), "+s"(s10), "+s"(s11))
// P6 DPP chain (2 wait states before each DPP read)
PROBE(k_p6, "s_nop 1\n v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 1\n v_add_u32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf", : "+v"(v1), "+v"(v2), "+s"(s10), "+s"(s11))
extern "C" int exp_probe(int which, void* out, int n, int reps, hipStream_t s) {
    switch (which) {
        case 1: hipLaunchKernelGGL(k_p1, dim3((n + 3) / 4), dim3(256), 0, s, (uint32_t*)out, n, reps); break;
        case 2: hipLaunchKernelGGL(k_p2, dim3((n + 3) / 4), dim3(256), 0, s, (uint32_t*)out, n, reps); break;
        case 3: hipLaunchKernelGGL(k_p3, dim3((n + 3) / 4), dim3(256), 0, s, (uint32_t*)out, n, reps); break;
        case 4: hipLaunchKernelGGL(k_p4, dim3((n + 3) / 4), dim3(256), 0, s, (uint32_t*)out, n, reps); break;
        case 5: hipLaunchKernelGGL(k_p5, dim3((n + 3) / 4), dim3(256), 0, s, (uint32_t*)out, n, reps); break;
        default: hipLaunchKernelGGL(k_p6, dim3((n + 3) / 4), dim3(256), 0, s, (uint32_t*)out, n, reps); break;
    }
    return (int)hipGetLastError();
}

// kernel-argument lines on an exposed chain: NL lines, then one load round trip,
// then 1024 dependent VALU ops (so the wave outlives the launch floor)
template <int NL>
__global__ __launch_bounds__(256) void k_klines_chain(KLines k, const uint32_t* __restrict__ rob,
                                                      uint32_t* __restrict__ out, int n) {
    const int w = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < NL; i++) {
        uint64_t v = k.line[i][i % 8];
        asm volatile("" : "+s"(v));
        acc += v;
    }
    if (w >= n) return;
    uint32_t r = lane < 5 ? rob[(size_t)w * 5 + lane] : 0u;
    r += (uint32_t)acc;
    asm volatile(".rept 1024\n v_add_u32 %0, %0, %0\n .endr" : "+v"(r));
    if (lane < 5) out[(size_t)w * 5 + lane] = r;
}
extern "C" int exp_klines_chain(int nl, const void* rob, void* out, int n, hipStream_t s) {
    KLines k{};
    if (nl == 1) hipLaunchKernelGGL(k_klines_chain<1>, dim3((n + 3) / 4), dim3(256), 0, s, k, (const uint32_t*)rob, (uint32_t*)out, n);
    else hipLaunchKernelGGL(k_klines_chain<9>, dim3((n + 3) / 4), dim3(256), 0, s, k, (const uint32_t*)rob, (uint32_t*)out, n);
    return (int)hipGetLastError();
}
