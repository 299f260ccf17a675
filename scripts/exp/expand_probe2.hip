// expand_probe2.hip -- config-5-shaped flat map emission (round 4, profiling only).
//
// Config 5's observations are 95 % actor-map planes (16 agents x 6 x 64 x 64 floats per env, 1.65 MB per
// env); the general builder streams them wave-per-env at 4.47 TB/s.  Here: a flat pass over a 4096-env
// chunk (6.4 GB of maps), thread q writing float4 q, its 4 bits taken from small per-env records (5 cell
// bitsets of 128 words + 2 words per agent: ~2.7 KB per env, 11 MB per chunk, L2/MALL-resident) with
//   map1   one record load per float4 (the shared planes' form)
//   map2   two loads (bitset word + the agent's cell word, the one-hot planes' form)
//   map3   the real plane mix: ch 0/3/4 one bitset word, ch 1/5 one agent word, ch 2 two words
// against a plain fill of the same bytes and the wave-per-env slab shape (and 2 / 4 / 8 / 64 / 256 waves per env's slab, split or interleaved; persistent waves).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/expand_probe2.hip -o scripts/exp/expand_probe2.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

constexpr int A = 16, HW = 4096, NW = HW / 32, PER4 = A * 6 * HW / 4;   // float4s of one env's actor maps
constexpr int RW = 5 * NW + 2 * A + 32;                                 // record words per env

typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 nib(uint32_t b) {
    return f32x4{(float)(b & 1), (float)((b >> 1) & 1), (float)((b >> 2) & 1), (float)(b >> 3)};
}

__global__ __launch_bounds__(256) void k_fill(f32x4* __restrict__ out, size_t n4) {
    const size_t q = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (q < n4) out[q] = f32x4{1.f, 0.f, 1.f, 0.f};
}

__global__ __launch_bounds__(256) void k_slab(f32x4* __restrict__ out, int n) {
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w >= n) return;
    f32x4* o = out + (size_t)w * PER4;
    for (int q = lane; q < PER4; q += 64) o[q] = f32x4{1.f, 0.f, 1.f, 0.f};
}

// S waves per env, wave s of env w writing the s-th of S equal parts of the env's slab
template <int S>
__global__ __launch_bounds__(256) void k_slabs(f32x4* __restrict__ out, int n) {
    const int w2 = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int w = w2 / S, s = w2 % S;
    if (w >= n) return;
    f32x4* o = out + (size_t)w * PER4 + (size_t)s * (PER4 / S);
    for (int q = lane; q < PER4 / S; q += 64) o[q] = f32x4{1.f, 0.f, 1.f, 0.f};
}

// S waves per env (S = 4: one workgroup), interleaved: the S waves write consecutive 1 KB pieces, so the
// env's slab is written as one stream advancing S KB per round instead of S streams
template <int S>
__global__ __launch_bounds__(256) void k_slabs_il(f32x4* __restrict__ out, int n) {
    const int w2 = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int w = w2 / S, s = w2 % S;
    if (w >= n) return;
    f32x4* o = out + (size_t)w * PER4;
    for (int q = s * 64 + lane; q < PER4; q += 64 * S) o[q] = f32x4{1.f, 0.f, 1.f, 0.f};
}

// persistent: NWV waves in all, wave v writing the slabs of envs v, v + NWV, ... one after another
__global__ __launch_bounds__(256) void k_slab_persist(f32x4* __restrict__ out, int n, int nwv) {
    const int v = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    for (int w = v; w < n; w += nwv) {
        f32x4* o = out + (size_t)w * PER4;
        for (int q = lane; q < PER4; q += 64) o[q] = f32x4{1.f, 0.f, 1.f, 0.f};
    }
}

template <int MODE>
__global__ __launch_bounds__(256) void k_map(f32x4* __restrict__ out, size_t n4, const uint32_t* __restrict__ rec) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;   // n4 < 2^32
    if (q >= n4) return;
    const uint32_t e = q / (uint32_t)PER4, j = q - e * (uint32_t)PER4;
    const uint32_t pp = j >> 10, c0 = (j & 1023u) << 2;                               // HW / 4 = 1024 float4 per plane
    const uint32_t a = pp / 6u, ch = pp - 6u * a;
    const uint32_t* r = rec + (size_t)e * RW;
    const uint32_t sh = c0 & 31u;
    uint32_t b;
    if (MODE == 1) {
        b = (r[(ch % 5u) * NW + (c0 >> 5)] >> sh) & 15u;
    } else if (MODE == 2) {
        const uint32_t own = r[5 * NW + 2 * a];
        b = ((r[(ch % 5u) * NW + (c0 >> 5)] >> sh) & 15u) ^ (own - c0 < 4u ? 1u << (own - c0) : 0u);
    } else {
        if (ch == 1 || ch == 5) {
            const uint32_t cl = r[5 * NW + 2 * a + (ch == 5)];
            b = cl - c0 < 4u ? 1u << (cl - c0) : 0u;
        } else {
            const int set = ch == 0 ? 0 : ch == 3 ? 2 : ch == 4 ? 3 : 1;
            b = (r[set * NW + (c0 >> 5)] >> sh) & 15u;
            if (ch == 2) {
                const uint32_t own = r[5 * NW + 2 * a];
                b = (b & ~(own - c0 < 4u ? 1u << (own - c0) : 0u)) | ((r[4 * NW + (c0 >> 5)] >> sh) & 15u);
            }
        }
    }
    out[q] = nib(b);
}

int main() {
    const int n = 4096;
    const size_t n4 = (size_t)n * PER4;
    const double bytes = 16.0 * n4;
    f32x4* out;
    uint32_t* rec;
    CK(hipMalloc(&out, n4 * 16));
    CK(hipMalloc(&rec, (size_t)n * RW * 4));
    std::vector<uint32_t> h((size_t)n * RW);
    for (size_t i = 0; i < h.size(); i++) h[i] = (uint32_t)(i * 2654435761u);
    for (int e = 0; e < n; e++)
        for (int k = 0; k < 2 * A; k++) h[(size_t)e * RW + 5 * NW + k] = (uint32_t)((e * 37 + k * 101) % HW);
    CK(hipMemcpy(rec, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto launch) {
        for (int i = 0; i < 2; i++) launch();
        (void)hipDeviceSynchronize();
        std::vector<float> t;
        for (int r = 0; r < 7; r++) {
            (void)hipEventRecord(e0, 0);
            launch();
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        return t[3];
    };
    auto rep = [&](const char* k, float us) {
        printf("{\"kind\": \"%s\", \"us\": %.1f, \"TBs\": %.2f}\n", k, us, bytes / (us * 1e-6) / 1e12);
        fflush(stdout);
    };
    const unsigned nb = (unsigned)((n4 + 255) / 256);
    for (int round = 0; round < 2; round++) {
        rep("fill", timeit([&] { hipLaunchKernelGGL(k_fill, dim3(nb), dim3(256), 0, 0, out, n4); }));
        rep("slab", timeit([&] { hipLaunchKernelGGL(k_slab, dim3(n / 4), dim3(256), 0, 0, out, n); }));
        rep("slab_x2", timeit([&] { hipLaunchKernelGGL(k_slabs<2>, dim3(2 * n / 4), dim3(256), 0, 0, out, n); }));
        rep("slab_x4", timeit([&] { hipLaunchKernelGGL(k_slabs<4>, dim3(4 * n / 4), dim3(256), 0, 0, out, n); }));
        rep("slab_x8", timeit([&] { hipLaunchKernelGGL(k_slabs<8>, dim3(8 * n / 4), dim3(256), 0, 0, out, n); }));
        rep("slab_il2", timeit([&] { hipLaunchKernelGGL(k_slabs_il<2>, dim3(2 * n / 4), dim3(256), 0, 0, out, n); }));
        rep("slab_il4", timeit([&] { hipLaunchKernelGGL(k_slabs_il<4>, dim3(4 * n / 4), dim3(256), 0, 0, out, n); }));
        rep("slab_x64", timeit([&] { hipLaunchKernelGGL(k_slabs<64>, dim3(64 * n / 4), dim3(256), 0, 0, out, n); }));
        rep("slab_x256", timeit([&] { hipLaunchKernelGGL(k_slabs<256>, dim3(256 * n / 4), dim3(256), 0, 0, out, n); }));
        rep("persist1024", timeit([&] { hipLaunchKernelGGL(k_slab_persist, dim3(256), dim3(256), 0, 0, out, n, 1024); }));
        rep("persist2048", timeit([&] { hipLaunchKernelGGL(k_slab_persist, dim3(512), dim3(256), 0, 0, out, n, 2048); }));
        rep("map1", timeit([&] { hipLaunchKernelGGL(k_map<1>, dim3(nb), dim3(256), 0, 0, out, n4, rec); }));
        rep("map2", timeit([&] { hipLaunchKernelGGL(k_map<2>, dim3(nb), dim3(256), 0, 0, out, n4, rec); }));
        rep("map3", timeit([&] { hipLaunchKernelGGL(k_map<3>, dim3(nb), dim3(256), 0, 0, out, n4, rec); }));
    }
    return 0;
}
