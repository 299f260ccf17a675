// Probe (profiling only): the store shape of the observation builders.  A
// wave-per-env builder writes each env's rows of the four output tensors (actor maps [E][A][6][H][W],
// actor vectors [E][A][Dv], critic map [E][4][H][W], critic vector [E][Dg]): config 3 12,000 + 1,040
// + 1,600 + 5,204 = 19,844 B per env, config 3b (1007-dim actor vectors) 12,000 + 20,140 + 1,600 +
// 5,204 = 38,944 B, 16,384 envs.  This probe writes exactly those rows with no compute, per store
// width (one dword, two dwords or four dwords per lane and wave-instruction: 256 / 512 / 1,024 B) and
// per residency (8, 12, 16 waves per CU forced by the workgroup's LDS request, or uncapped), and
// reports TB/s of output.  The wide forms write each row's unaligned head and tail as dwords (what
// the builders do); the dword form needs no alignment.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/obs_store_shapes.hip -o scripts/exp/obs_store_shapes.bin
// One JSON line per case: median microseconds of 20 launches and TB/s.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

struct Parts {
    float* p[4];
    int dw[4];   // dwords per env of each tensor
};

// one row of `n` dwords at o (4-B aligned), W dwords per lane per instruction (W = 1, 2, 4); wider
// stores only on the 4W-B-aligned middle, the head and tail as dwords
template <int W>
__device__ __forceinline__ void row_store(float* o, int n, int lane, float v) {
    if constexpr (W == 1) {
        for (int q = lane; q < n; q += 64) o[q] = v;
    } else {
        const int mis = (int)(((uintptr_t)o >> 2) & (W - 1));
        const int head = mis ? min(n, W - mis) : 0;
        if (lane < head) o[lane] = v;
        float* m = o + head;
        const int nm = (n - head) / W;
        typedef float fv __attribute__((ext_vector_type(W)));
        fv vv;
        for (int i = 0; i < W; i++) vv[i] = v;
        fv* mv = reinterpret_cast<fv*>(m);
        for (int q = lane; q < nm; q += 64) mv[q] = vv;
        const int tail0 = head + nm * W;
        if (tail0 + lane < n) o[tail0 + lane] = v;
    }
}

template <int W>
__global__ __launch_bounds__(256) void k_parts(Parts P, int n) {
    extern __shared__ unsigned char lds[];   // only to cap residency
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int e = blockIdx.x * 4 + wave;
    if (e >= n) return;
    if (lane == 64) lds[0] = 0;   // keep the allocation
    const float v = (float)e;
#pragma unroll
    for (int t = 0; t < 4; t++) row_store<W>(P.p[t] + (size_t)e * P.dw[t], P.dw[t], lane, v);
}

int main() {
    const int n = 16384;
    const int cfg3[4] = {12000 / 4, 1040 / 4, 1600 / 4, 5204 / 4};
    const int cfg3b[4] = {12000 / 4, 20140 / 4, 1600 / 4, 5204 / 4};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int c = 0; c < 2; c++) {
        const int* dw = c == 0 ? cfg3 : cfg3b;
        Parts P;
        size_t bytes = 0;
        for (int t = 0; t < 4; t++) {
            P.dw[t] = dw[t];
            CK(hipMalloc(&P.p[t], (size_t)n * dw[t] * 4));
            bytes += (size_t)n * dw[t] * 4;
        }
        for (int wpc : {0, 8, 12, 16}) {   // waves per CU (0: no LDS request)
            // 4-wave workgroups: 160 KiB / (wpc / 4) of LDS each caps the CU at wpc waves
            const size_t lds = wpc ? std::min<size_t>(64 * 1024, (160 * 1024) / (wpc / 4) - 1024) : 0;
            for (int W : {1, 2, 4}) {
                auto launch = [&] {
                    if (W == 1) hipLaunchKernelGGL(k_parts<1>, dim3(n / 4), dim3(256), lds, 0, P, n);
                    else if (W == 2) hipLaunchKernelGGL(k_parts<2>, dim3(n / 4), dim3(256), lds, 0, P, n);
                    else hipLaunchKernelGGL(k_parts<4>, dim3(n / 4), dim3(256), lds, 0, P, n);
                };
                for (int i = 0; i < 3; i++) launch();
                CK(hipDeviceSynchronize());
                std::vector<float> ts;
                for (int r = 0; r < 20; r++) {
                    CK(hipEventRecord(e0, 0));
                    launch();
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    ts.push_back(ms * 1e3f);
                }
                std::sort(ts.begin(), ts.end());
                printf("{\"config\": \"%s\", \"bytes_per_env\": %zu, \"store_dwords_per_lane\": %d, \"waves_per_cu_cap\": %d, "
                       "\"lds_per_wg\": %zu, \"us\": %.1f, \"TBs\": %.2f}\n",
                       c == 0 ? "3" : "3b", bytes / n, W, wpc, lds, ts[10], bytes / (ts[10] * 1e-6) / 1e12);
                fflush(stdout);
            }
        }
        for (int t = 0; t < 4; t++) CK(hipFree(P.p[t]));
    }
    return 0;
}
