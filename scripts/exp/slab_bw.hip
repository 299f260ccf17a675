// Probe (profiling only): the write bandwidth of the observation builders' store shape with no
// compute -- one wave per env writes its contiguous output slab (config 3b: 38,944 B per env,
// 16384 envs = 638 MB) as float4 stores -- against occupancy (a dynamic LDS request per wave, as
// the builder's slice limits it) and workgroup size, and against a flat grid-stride fill.
//   hipcc --offload-arch=gfx950 -O3 scripts/exp/slab_bw.hip -o build/slab_bw && build/slab_bw
// One JSON line per case: microseconds per launch (median of 20) and TB/s.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

// wave w writes float4s [w * slab, (w + 1) * slab) of out
__global__ __launch_bounds__(1024) void k_slab(float4* __restrict__ out, int n, int slab, int wpb) {
    extern __shared__ float4 lds[];
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * wpb + wave;
    if (wave >= wpb || w >= n) return;
    lds[wave * 64 + lane] = make_float4(0.f, 0.f, 0.f, 0.f);   // touch the slice (occupancy only)
    float4* o = out + (size_t)w * slab;
    const float4 v = make_float4(1.f, 2.f, 3.f, (float)w);
    for (int q0 = 0; q0 < slab; q0 += 64) o[min(q0 + lane, slab - 1)] = v;
}

// the same bytes, grid-stride float4 stores by every lane of a full-chip grid
__global__ __launch_bounds__(256) void k_flat(float4* __restrict__ out, size_t n4) {
    const float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) out[i] = v;
}

int main() {
    const int n = 16384, slab = 38944 / 16;   // float4s per env (config 3b)
    const size_t n4 = (size_t)n * slab, bytes = n4 * 16;
    float4* out;
    CK(hipMalloc(&out, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto launch) {
        for (int i = 0; i < 3; i++) launch();
        CK(hipDeviceSynchronize());
        std::vector<float> t;
        for (int r = 0; r < 20; r++) {
            CK(hipEventRecord(e0, 0));
            launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        return t[10];
    };
    for (int wpb : {1, 4, 16})
        for (int lds_kb : {1, 8, 16, 32}) {
            const size_t lds = (size_t)lds_kb * 1024 * wpb;
            if (lds > 160 * 1024) continue;
            const int blocks = (n + wpb - 1) / wpb;
            const float us = timeit([&] {
                hipLaunchKernelGGL(k_slab, dim3(blocks), dim3(64 * wpb), lds, 0, out, n, slab, wpb);
            });
            printf("{\"kind\": \"slab\", \"waves_per_block\": %d, \"lds_kb_per_wave\": %d, \"us\": %.1f, \"TBs\": %.2f}\n",
                   wpb, lds_kb, us, bytes / (us * 1e-6) / 1e12);
        }
    for (int blocks : {1024, 4096, 16384}) {
        const float us = timeit([&] { hipLaunchKernelGGL(k_flat, dim3(blocks), dim3(256), 0, 0, out, n4); });
        printf("{\"kind\": \"flat\", \"blocks\": %d, \"us\": %.1f, \"TBs\": %.2f}\n", blocks, us, bytes / (us * 1e-6) / 1e12);
    }
    CK(hipFree(out));
    return 0;
}
