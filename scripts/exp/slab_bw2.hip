// Probe (profiling only): what limits the observation builders' store shape (one wave per env
// writing its contiguous output slab, 16384 envs x 38,944 B = 638 MB, config 3b) below a plain
// fill.  Variants of the same bytes:
//   slab      -- the builders' shape: wave w streams its slab front to back, float4 per lane
//   slab_rot  -- the same, each wave starting at a slab offset rotated by its env index (so the
//                waves in flight are not all at the same slab offset)
//   slab_x2   -- each lane writes 32 contiguous bytes per step (two float4 stores)
//   slab_nt   -- slab with nontemporal stores
//   slab_wg4  -- the 4 waves of a workgroup write the 4 adjacent slabs of their envs together,
//                1 KB of each in turn (concurrent stores of a workgroup land in one 156 KB span)
//   flat      -- grid-stride float4 stores over the whole buffer (blocks x 256 threads)
//   flat_x4   -- flat, each thread 4 consecutive float4 per step
//   memset    -- hipMemsetD32Async of the same bytes
//   splitK    -- each env's slab written by K waves, one contiguous K-th each
//   strideS   -- slab, its 1 KB pieces in the order 0, S, 2S, .., 1, S+1, .. (stores S KB apart)
//   chunk     -- block b writes one contiguous chunk, its 4 waves interleaved at 1 KB; _perm: chunks
//                (or flat's first positions) permuted over the blocks (no moving write window)
//   hipcc --offload-arch=gfx950 -O3 scripts/exp/slab_bw2.hip -o build/slab_bw2 && build/slab_bw2
// One JSON line per case: microseconds per launch (median of 20) and TB/s.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <int MODE>   // 0 slab, 1 rotated start, 2 two float4 per lane, 3 nontemporal
__global__ __launch_bounds__(256) void k_slab(float4* __restrict__ out, int n, int slab) {
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + wave;
    if (w >= n) return;
    float4* o = out + (size_t)w * slab;
    const float4 v = make_float4(1.f, 2.f, 3.f, (float)w);
    if (MODE == 0) {
        for (int q0 = 0; q0 < slab; q0 += 64) o[min(q0 + lane, slab - 1)] = v;
    } else if (MODE == 1) {
        const int nst = (slab + 63) / 64;
        const int s0 = (w * 7) % nst;
        for (int k = 0; k < nst; k++) {
            int st = s0 + k;
            st = st >= nst ? st - nst : st;
            o[min(st * 64 + lane, slab - 1)] = v;
        }
    } else if (MODE == 2) {
        for (int q0 = 0; q0 < slab; q0 += 128) {
            o[min(q0 + 2 * lane, slab - 1)] = v;
            o[min(q0 + 2 * lane + 1, slab - 1)] = v;
        }
    } else {
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 vv = {v.x, v.y, v.z, v.w};
        f4* o4 = reinterpret_cast<f4*>(o);
        for (int q0 = 0; q0 < slab; q0 += 64) __builtin_nontemporal_store(vv, &o4[min(q0 + lane, slab - 1)]);
    }
}

// 4 waves of a workgroup, envs 4b..4b+3: step k, wave v writes float4s [k*64, k*64+64) of env 4b+v's slab
// in the order (k, v) -> the workgroup's stores interleave over its 4 slabs as the slab shape does,
// but every wave also writes a neighbour's slab part in turn (round robin over the 4 slabs)
__global__ __launch_bounds__(256) void k_slab_wg4(float4* __restrict__ out, int n, int slab) {
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const size_t base = (size_t)blockIdx.x * 4 * slab;   // the 4 slabs are adjacent: one span
    const int span = 4 * slab;
    const float4 v = make_float4(1.f, 2.f, 3.f, (float)wave);
    // the span as 1 KB pieces dealt to the 4 waves round robin: consecutive in flight
    for (int q0 = wave * 64; q0 < span; q0 += 256) out[base + min(q0 + lane, span - 1)] = v;
}

// the slab's 1 KB pieces (64 float4s) in the order 0, S, 2S, ..., 1, S+1, ...: consecutive stores of
// a wave land S KB apart instead of back to back
template <int S>
__global__ __launch_bounds__(256) void k_slab_stride(float4* __restrict__ out, int n, int slab) {
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + wave;
    if (w >= n) return;
    float4* o = out + (size_t)w * slab;
    const float4 v = make_float4(1.f, 2.f, 3.f, (float)w);
    const int np = (slab + 63) / 64;
    for (int r = 0; r < S; r++)
        for (int k = r; k < np; k += S) o[min(k * 64 + lane, slab - 1)] = v;
}

// env w / K's slab split in K contiguous parts, part w % K written by wave w (K waves per env)
template <int K>
__global__ __launch_bounds__(256) void k_slab_split(float4* __restrict__ out, int n, int slab) {
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + wave;
    const int env = w / K, part = w % K;
    if (env >= n) return;
    const int per = (slab + K - 1) / K;
    const int q_end = min(slab, (part + 1) * per);
    float4* o = out + (size_t)env * slab;
    const float4 v = make_float4(1.f, 2.f, 3.f, (float)w);
    for (int q0 = part * per; q0 < q_end; q0 += 64) o[min(q0 + lane, q_end - 1)] = v;
}

// block b writes its own contiguous chunk of n4 / gridDim.x float4s, the 4 waves interleaved at 1 KB
// (wave v: pieces v, v + 4, ...); PERM: block b takes chunk (b * 7919) mod gridDim.x instead of b
template <bool PERM>
__global__ __launch_bounds__(256) void k_chunk(float4* __restrict__ out, size_t n4) {
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const size_t nb = gridDim.x, per = (n4 + nb - 1) / nb;
    const size_t b = PERM ? ((size_t)blockIdx.x * 7919u) % nb : blockIdx.x;
    const size_t q0 = b * per, q1 = min(n4, q0 + per);
    const float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
    for (size_t q = q0 + wave * 64; q < q1; q += 256) out[min(q + lane, q1 - 1)] = v;
}

// flat grid-stride, block b's first position permuted as in k_chunk
__global__ __launch_bounds__(256) void k_flat_perm(float4* __restrict__ out, size_t n4) {
    const float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
    const size_t nb = gridDim.x, b = ((size_t)blockIdx.x * 7919u) % nb;
    for (size_t i = b * 256 + threadIdx.x; i < n4; i += nb * 256) out[i] = v;
}

__global__ __launch_bounds__(256) void k_flat(float4* __restrict__ out, size_t n4) {
    const float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) out[i] = v;
}

__global__ __launch_bounds__(256) void k_flat_x4(float4* __restrict__ out, size_t n4) {
    const float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
    const size_t stride = (size_t)gridDim.x * 1024;
    for (size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x; i < n4; i += stride) {
        out[i] = v;
        if (i + 256 < n4) out[i + 256] = v;
        if (i + 512 < n4) out[i + 512] = v;
        if (i + 768 < n4) out[i + 768] = v;
    }
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
    auto report = [&](const char* kind, int blocks, float us) {
        printf("{\"kind\": \"%s\", \"blocks\": %d, \"us\": %.1f, \"TBs\": %.2f}\n", kind, blocks, us,
               bytes / (us * 1e-6) / 1e12);
    };
    const int sb = n / 4;
    report("slab", sb, timeit([&] { hipLaunchKernelGGL(k_slab<0>, dim3(sb), dim3(256), 0, 0, out, n, slab); }));
    report("slab_rot", sb, timeit([&] { hipLaunchKernelGGL(k_slab<1>, dim3(sb), dim3(256), 0, 0, out, n, slab); }));
    report("slab_x2", sb, timeit([&] { hipLaunchKernelGGL(k_slab<2>, dim3(sb), dim3(256), 0, 0, out, n, slab); }));
    report("slab_nt", sb, timeit([&] { hipLaunchKernelGGL(k_slab<3>, dim3(sb), dim3(256), 0, 0, out, n, slab); }));
    report("slab_wg4", sb, timeit([&] { hipLaunchKernelGGL(k_slab_wg4, dim3(sb), dim3(256), 0, 0, out, n, slab); }));
    for (int blocks : {4096, 16384, 65536})
        report("flat", blocks, timeit([&] { hipLaunchKernelGGL(k_flat, dim3(blocks), dim3(256), 0, 0, out, n4); }));
    for (int blocks : {2048, 8192, 32768})
        report("flat_x4", blocks, timeit([&] { hipLaunchKernelGGL(k_flat_x4, dim3(blocks), dim3(256), 0, 0, out, n4); }));
    report("memset", 0, timeit([&] { CK(hipMemsetD32Async((hipDeviceptr_t)out, 0x3f800000, n4 * 4, 0)); }));
    report("slab", sb, timeit([&] { hipLaunchKernelGGL(k_slab<0>, dim3(sb), dim3(256), 0, 0, out, n, slab); }));
    for (int blocks : {16384, 65536}) {
        report("chunk", blocks, timeit([&] { hipLaunchKernelGGL(k_chunk<false>, dim3(blocks), dim3(256), 0, 0, out, n4); }));
        report("chunk_perm", blocks, timeit([&] { hipLaunchKernelGGL(k_chunk<true>, dim3(blocks), dim3(256), 0, 0, out, n4); }));
        report("flat_perm", blocks, timeit([&] { hipLaunchKernelGGL(k_flat_perm, dim3(blocks), dim3(256), 0, 0, out, n4); }));
    }
    report("stride2", sb, timeit([&] { hipLaunchKernelGGL(k_slab_stride<2>, dim3(sb), dim3(256), 0, 0, out, n, slab); }));
    report("stride4", sb, timeit([&] { hipLaunchKernelGGL(k_slab_stride<4>, dim3(sb), dim3(256), 0, 0, out, n, slab); }));
    report("stride8", sb, timeit([&] { hipLaunchKernelGGL(k_slab_stride<8>, dim3(sb), dim3(256), 0, 0, out, n, slab); }));
    report("stride16", sb, timeit([&] { hipLaunchKernelGGL(k_slab_stride<16>, dim3(sb), dim3(256), 0, 0, out, n, slab); }));
    report("split2", sb * 2, timeit([&] { hipLaunchKernelGGL(k_slab_split<2>, dim3(sb * 2), dim3(256), 0, 0, out, n, slab); }));
    report("split4", sb * 4, timeit([&] { hipLaunchKernelGGL(k_slab_split<4>, dim3(sb * 4), dim3(256), 0, 0, out, n, slab); }));
    report("split8", sb * 8, timeit([&] { hipLaunchKernelGGL(k_slab_split<8>, dim3(sb * 8), dim3(256), 0, 0, out, n, slab); }));
    report("split16", sb * 16, timeit([&] { hipLaunchKernelGGL(k_slab_split<16>, dim3(sb * 16), dim3(256), 0, 0, out, n, slab); }));
    CK(hipFree(out));
    return 0;
}
