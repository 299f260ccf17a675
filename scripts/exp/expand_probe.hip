// expand_probe.hip -- ceiling of a decoupled observation emission (round 4, profiling only).
//
// Question: if a per-env pass writes a compact record per env (a few KB, wave per env) and a
// second, flat pass expands the records into the float32 outputs (one float4 per thread, blocks in
// address order: the chip-wide moving write window of a fill), what rate does the pair reach for
// config 3's 325 MB (16384 envs x 19,840 B) and config 3b's 638 MB?
//
//   fill1      one float4 per thread, grid = n4 / 256 blocks (no loop)
//   fill2      two float4 per thread (q, q + n4/2)
//   flat64k    grid-stride over 65,536 blocks (the round-3 probe's best)
//   slab       wave per env, its contiguous slab (the builders' store shape)
//   rec        the record pass alone: wave per env writes REC bytes (slab shape)
//   expand     one float4 per thread: env = q / per4, one u32 read from the env's record, 4 bits
//              -> 4 floats (the map planes' form); the record pass before it (rec+expand), alone
//   expand_v   the same with a per-float select among 3 record words (vector form)
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/expand_probe.hip -o /tmp/expand_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                           \
        }                                                                       \
    } while (0)

__global__ __launch_bounds__(256) void k_fill1(float4* __restrict__ out, unsigned n4) {
    const unsigned q = blockIdx.x * 256 + threadIdx.x;
    if (q < n4) out[q] = make_float4(1.f, 0.f, 1.f, 0.f);
}

__global__ __launch_bounds__(256) void k_fill2(float4* __restrict__ out, unsigned n4) {
    const unsigned h = (n4 + 1) / 2;
    const unsigned q = blockIdx.x * 256 + threadIdx.x;
    if (q < h) out[q] = make_float4(1.f, 0.f, 1.f, 0.f);
    if (q + h < n4) out[q + h] = make_float4(1.f, 0.f, 1.f, 0.f);
}

__global__ __launch_bounds__(256) void k_flat(float4* __restrict__ out, size_t n4) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
        out[i] = make_float4(1.f, 0.f, 1.f, 0.f);
}

// wave per env: env w's slab of per4 float4s
__global__ __launch_bounds__(256) void k_slab(float4* __restrict__ out, int n, int per4) {
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w >= n) return;
    float4* o = out + (size_t)w * per4;
    for (int q = lane; q < per4; q += 64) o[q] = make_float4(1.f, 0.f, 1.f, 0.f);
}

// wave per env: a record of rw u32 words (the per-env pass's stores)
__global__ __launch_bounds__(256) void k_rec(uint32_t* __restrict__ rec, int n, int rw, uint32_t salt) {
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w >= n) return;
    uint4* r = reinterpret_cast<uint4*>(rec + (size_t)w * rw);
    for (int q = lane; q < rw / 4; q += 64) {
        const uint32_t v = (uint32_t)(w * 2654435761u) ^ (q * 40503u) ^ salt;
        r[q] = make_uint4(v, v * 3u, v * 5u, v * 7u);
    }
}

__device__ __forceinline__ unsigned divmagic(unsigned x, unsigned m, unsigned s) { return __umulhi(x, m) >> s; }

// one float4 per thread from one record word (map-plane form)
__global__ __launch_bounds__(256) void k_expand(float4* __restrict__ out, unsigned n4, const uint32_t* __restrict__ rec,
                                                int rw, unsigned per4, unsigned m, unsigned s) {
    const unsigned q = blockIdx.x * 256 + threadIdx.x;
    if (q >= n4) return;
    const unsigned e = divmagic(q, m, s), j = q - e * per4;
    const uint32_t wd = rec[(size_t)e * rw + ((j >> 3) % (unsigned)rw)];
    const uint32_t b = (wd >> ((j & 7) * 4)) & 15u;
    out[q] = make_float4((float)(b & 1), (float)((b >> 1) & 1), (float)((b >> 2) & 1), (float)(b >> 3));
}

// vector form: each float picks a record word by interval (data / zero / tail)
__global__ __launch_bounds__(256) void k_expand_v(float4* __restrict__ out, unsigned n4, const uint32_t* __restrict__ rec,
                                                  int rw, unsigned per4, unsigned m, unsigned s, unsigned ndata) {
    const unsigned q = blockIdx.x * 256 + threadIdx.x;
    if (q >= n4) return;
    const unsigned e = divmagic(q, m, s), j = 4 * (q - e * per4);
    const uint32_t* r = rec + (size_t)e * rw;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const unsigned f = j + i;
        const bool data = f < ndata;
        const bool tail = f == 4 * per4 - 1;
        v[i] = data ? __uint_as_float(r[f % (unsigned)rw] & 0x3f7fffffu) : tail ? 0.5f : 0.0f;
    }
    out[q] = make_float4(v[0], v[1], v[2], v[3]);
}

static void magic_for(unsigned d, unsigned& m, unsigned& s) {
    // floor(x / d) = umulhi(x, m) >> s for every x < 2^31 (round-up method)
    for (s = 0; s < 32; s++) {
        const unsigned long long two = 1ull << (32 + s);
        const unsigned long long mm = (two + d - 1) / d;
        if (mm < (1ull << 32) && mm * d - two <= (1ull << s)) {
            m = (unsigned)mm;
            return;
        }
    }
    m = 0;
}

int main() {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto launch) {
        for (int i = 0; i < 3; i++) launch();
        (void)hipDeviceSynchronize();
        std::vector<float> t;
        for (int r = 0; r < 21; r++) {
            (void)hipEventRecord(e0, 0);
            launch();
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        return t[10];
    };
    struct Cfg { const char* name; int n, per4, rw; };
    // per4: float4s per env (config 3: 19,840 B; 3b: 38,944 B); rw: record words per env
    const Cfg cfgs[] = {{"c3", 16384, 1240, 752}, {"c3b", 16384, 2434, 752}, {"c3_rec2k", 16384, 1240, 512}};
    for (const Cfg& c : cfgs) {
        const unsigned n4 = (unsigned)c.n * c.per4;
        const double bytes = 16.0 * n4;
        float4* out;
        uint32_t* rec;
        CK(hipMalloc(&out, (size_t)n4 * 16));
        CK(hipMalloc(&rec, (size_t)c.n * c.rw * 4));
        unsigned m, s;
        magic_for(c.per4, m, s);
        auto rep = [&](const char* k, float us, double by) {
            printf("{\"cfg\": \"%s\", \"kind\": \"%s\", \"us\": %.1f, \"TBs_out\": %.2f}\n", c.name, k, us, by / (us * 1e-6) / 1e12);
            fflush(stdout);
        };
        const unsigned nb1 = (n4 + 255) / 256, nb2 = ((n4 + 1) / 2 + 255) / 256;
        rep("fill1", timeit([&] { hipLaunchKernelGGL(k_fill1, dim3(nb1), dim3(256), 0, 0, out, n4); }), bytes);
        rep("fill2", timeit([&] { hipLaunchKernelGGL(k_fill2, dim3(nb2), dim3(256), 0, 0, out, n4); }), bytes);
        rep("flat64k", timeit([&] { hipLaunchKernelGGL(k_flat, dim3(65536), dim3(256), 0, 0, out, (size_t)n4); }), bytes);
        rep("slab", timeit([&] { hipLaunchKernelGGL(k_slab, dim3(c.n / 4), dim3(256), 0, 0, out, c.n, c.per4); }), bytes);
        rep("rec", timeit([&] { hipLaunchKernelGGL(k_rec, dim3(c.n / 4), dim3(256), 0, 0, rec, c.n, c.rw, 1u); }),
            4.0 * c.n * c.rw);
        rep("expand", timeit([&] { hipLaunchKernelGGL(k_expand, dim3(nb1), dim3(256), 0, 0, out, n4, rec, c.rw, c.per4, m, s); }), bytes);
        rep("rec+expand", timeit([&] {
                hipLaunchKernelGGL(k_rec, dim3(c.n / 4), dim3(256), 0, 0, rec, c.n, c.rw, 2u);
                hipLaunchKernelGGL(k_expand, dim3(nb1), dim3(256), 0, 0, out, n4, rec, c.rw, c.per4, m, s);
            }), bytes);
        rep("expand_v", timeit([&] { hipLaunchKernelGGL(k_expand_v, dim3(nb1), dim3(256), 0, 0, out, n4, rec, c.rw, c.per4, m, s, 300u); }), bytes);
        rep("rec+expand_v", timeit([&] {
                hipLaunchKernelGGL(k_rec, dim3(c.n / 4), dim3(256), 0, 0, rec, c.n, c.rw, 3u);
                hipLaunchKernelGGL(k_expand_v, dim3(nb1), dim3(256), 0, 0, out, n4, rec, c.rw, c.per4, m, s, 300u);
            }), bytes);
        rep("fill1", timeit([&] { hipLaunchKernelGGL(k_fill1, dim3(nb1), dim3(256), 0, 0, out, n4); }), bytes);
        rep("slab", timeit([&] { hipLaunchKernelGGL(k_slab, dim3(c.n / 4), dim3(256), 0, 0, out, c.n, c.per4); }), bytes);
        CK(hipFree(out));
        CK(hipFree(rec));
    }
    return 0;
}
