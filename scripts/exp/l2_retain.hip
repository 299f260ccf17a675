// Probe (profiling only): the latency of the step kernel's state round trip across launches.
// Each wave loads one env's rows in the step's shape (robot u32 x5, package u64 x50, state u16
// x50, tracker u64 x50, env record 16 B: SoA arrays, env-major) or the same bytes as one
// contiguous per-env record (AoS), waits for them, writes the robot words back (as the step's
// write-back does), and records s_memtime around the round trip.  Launch sequences:
//   same   -- env w on wave w every launch (graph replay: the same workgroup -> XCD mapping);
//   flip   -- the env <-> wave mapping shifted by half the batch every other launch (another XCD's L2);
//   cold   -- a 1 GiB streaming write between launches (the state evicted from L2 and MALL).
//   hipcc --offload-arch=gfx950 -O3 scripts/exp/l2_retain.hip -o build/l2_retain && build/l2_retain
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int A = 5, P = 50;
constexpr int REC = 1024;   // AoS bytes per env: rob 20 | pad | pkg 400 | pst 100 | trk 400 | es 16

__global__ __launch_bounds__(256) void k_soa(uint32_t* __restrict__ rob, const uint64_t* __restrict__ pkg,
                                             const uint16_t* __restrict__ pst, const uint64_t* __restrict__ trk,
                                             const uint4* __restrict__ es, int n, int shift,
                                             unsigned long long* __restrict__ cyc) {
    const int w = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    if (w >= n) return;
    const int e = (w + shift) % n;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    uint32_t r = lane < A ? rob[(size_t)e * A + lane] : 0u;
    uint64_t p = lane < P ? pkg[(size_t)e * P + lane] : 0ull;
    uint32_t s = lane < P ? pst[(size_t)e * P + lane] : 0u;
    uint64_t t = lane < P ? trk[(size_t)e * P + lane] : 0ull;
    const uint4 v = es[e];
    r += (uint32_t)p + s + (uint32_t)(t >> 7) + v.x;
    asm volatile("" : "+v"(r));
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane < A) rob[(size_t)e * A + lane] = r | 1u;
    if (lane == 0) cyc[w] = t1 - t0;
}

__global__ __launch_bounds__(256) void k_aos(unsigned char* __restrict__ rec, int n, int shift,
                                             unsigned long long* __restrict__ cyc) {
    const int w = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    if (w >= n) return;
    const int e = (w + shift) % n;
    unsigned char* b = rec + (size_t)e * REC;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    uint32_t r = lane < A ? ((uint32_t*)b)[lane] : 0u;
    uint64_t p = lane < P ? ((const uint64_t*)(b + 64))[lane] : 0ull;
    uint32_t s = lane < P ? ((const uint16_t*)(b + 464))[lane] : 0u;
    uint64_t t = lane < P ? ((const uint64_t*)(b + 576))[lane] : 0ull;
    const uint4 v = *(const uint4*)(b + 976);
    r += (uint32_t)p + s + (uint32_t)(t >> 7) + v.x;
    asm volatile("" : "+v"(r));
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane < A) ((uint32_t*)b)[lane] = r | 1u;
    if (lane == 0) cyc[w] = t1 - t0;
}

// SoA with per-env strides (elements) and wpb envs per workgroup: padded strides keep every
// cache line to one env (or to envs of one workgroup, i.e. one XCD)
__global__ __launch_bounds__(1024) void k_soa_pad(uint32_t* __restrict__ rob, const uint64_t* __restrict__ pkg,
                                                  const uint16_t* __restrict__ pst, const uint64_t* __restrict__ trk,
                                                  uint4* __restrict__ es, int n, int shift, int sr, int sp, int ss,
                                                  int wpb, int xcd, unsigned long long* __restrict__ cyc) {
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // xcd: workgroups are dealt round-robin to the 8 XCDs; give XCD x's workgroups one contiguous env range
    const int nb = gridDim.x, b = blockIdx.x;
    const int slot = xcd ? (b & 7) * (nb >> 3) + min(b & 7, nb & 7) + (b >> 3) : b;
    const int w = slot * wpb + wave;
    const int lane = threadIdx.x & 63;
    if (w >= n) return;
    const int e = (w + shift) % n;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    uint32_t r = lane < A ? rob[(size_t)e * sr + lane] : 0u;
    uint64_t p = lane < P ? pkg[(size_t)e * sp + lane] : 0ull;
    uint32_t s = lane < P ? pst[(size_t)e * ss + lane] : 0u;
    uint64_t t = lane < P ? trk[(size_t)e * sp + lane] : 0ull;
    const uint4 v = es[e];
    r += (uint32_t)p + s + (uint32_t)(t >> 7) + v.x;
    asm volatile("" : "+v"(r));
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane < A) rob[(size_t)e * sr + lane] = r | 1u;
    if (lane < P) ((uint16_t*)pst)[(size_t)e * ss + lane] = (uint16_t)(s + 1);   // the step rewrites changed state words
    if (lane == 0) {
        es[e] = uint4{v.x + 1, v.y, v.z, v.w};
        cyc[w] = t1 - t0;
    }
}

// per-env records (AoS) in the step's full shape: wpb envs per workgroup, XCD-contiguous slots,
// the robot words, state words and env record written back
__global__ __launch_bounds__(1024) void k_aos_full(unsigned char* __restrict__ rec, int n, int shift, int wpb,
                                                   unsigned long long* __restrict__ cyc) {
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nb = gridDim.x, b = blockIdx.x;
    const int w = ((b & 7) * (nb >> 3) + min(b & 7, nb & 7) + (b >> 3)) * wpb + wave;
    const int lane = threadIdx.x & 63;
    if (w >= n) return;
    const int e = (w + shift) % n;
    unsigned char* bb = rec + (size_t)e * REC;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    uint32_t r = lane < A ? ((uint32_t*)bb)[lane] : 0u;
    uint64_t p = lane < P ? ((const uint64_t*)(bb + 64))[lane] : 0ull;
    uint32_t s = lane < P ? ((const uint16_t*)(bb + 464))[lane] : 0u;
    uint64_t t = lane < P ? ((const uint64_t*)(bb + 576))[lane] : 0ull;
    const uint4 v = *(const uint4*)(bb + 976);
    r += (uint32_t)p + s + (uint32_t)(t >> 7) + v.x;
    asm volatile("" : "+v"(r));
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane < A) ((uint32_t*)bb)[lane] = r | 1u;
    if (lane < P) ((uint16_t*)(bb + 464))[lane] = (uint16_t)(s + 1);
    if (lane == 0) {
        *(uint4*)(bb + 976) = uint4{v.x + 1, v.y, v.z, v.w};
        cyc[w] = t1 - t0;
    }
}

__global__ void k_flush(float4* p, size_t n4) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) p[i] = make_float4(1, 2, 3, 4);
}

int main() {
    const int Emax = 4096;
    uint32_t* rob;
    uint64_t *pkg, *trk;
    uint16_t* pst;
    uint4* es;
    unsigned char* rec;
    unsigned long long* cyc;
    float4* junk;
    const size_t junk4 = (size_t)1 << 26;   // 1 GiB
    CK(hipMalloc(&rob, Emax * A * 4));
    CK(hipMalloc(&pkg, Emax * P * 8));
    CK(hipMalloc(&pst, Emax * P * 2));
    CK(hipMalloc(&trk, Emax * P * 8));
    CK(hipMalloc(&es, Emax * 16));
    CK(hipMalloc(&rec, (size_t)Emax * REC));
    CK(hipMalloc(&cyc, Emax * 8));
    CK(hipMalloc(&junk, junk4 * 16));
    CK(hipMemset(rob, 0, Emax * A * 4));
    CK(hipMemset(pkg, 0, Emax * P * 8));
    CK(hipMemset(pst, 0, Emax * P * 2));
    CK(hipMemset(trk, 0, Emax * P * 8));
    CK(hipMemset(es, 0, Emax * 16));
    CK(hipMemset(rec, 0, (size_t)Emax * REC));
    std::vector<unsigned long long> h(Emax);
    for (int aos = 0; aos < 2; aos++)
        for (int E : {1024, 4096})
            for (int mode = 0; mode < 3; mode++) {   // same, flip, cold
                std::vector<unsigned long long> med;
                for (int it = 0; it < 40; it++) {
                    const int shift = (mode == 1 && (it & 1)) ? E / 2 + 4 : 0;
                    if (mode == 2) hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, junk, junk4);
                    if (aos) hipLaunchKernelGGL(k_aos, dim3(E / 4), dim3(256), 0, 0, rec, E, shift, cyc);
                    else hipLaunchKernelGGL(k_soa, dim3(E / 4), dim3(256), 0, 0, rob, pkg, pst, trk, es, E, shift, cyc);
                    CK(hipDeviceSynchronize());
                    if (it < 10) continue;
                    CK(hipMemcpy(h.data(), cyc, E * 8, hipMemcpyDeviceToHost));
                    std::vector<unsigned long long> v(h.begin(), h.begin() + E);
                    std::sort(v.begin(), v.end());
                    med.push_back(v[E / 2]);
                }
                std::sort(med.begin(), med.end());
                printf("{\"layout\": \"%s\", \"envs\": %d, \"mode\": \"%s\", \"round_trip_cycles_median\": %llu}\n",
                       aos ? "aos" : "soa", E, mode == 0 ? "same" : mode == 1 ? "flip" : "cold", med[med.size() / 2]);
            }
    // SoA, 16 waves per workgroup (the config-2 step's shape), writing rob + state words + env records
    // as the step does: unpadded strides vs strides padded to whole 128-B lines per env
    uint32_t* rob2;
    uint16_t* pst2;
    uint64_t *pkg2, *trk2;
    CK(hipMalloc(&rob2, Emax * 32 * 4));
    CK(hipMalloc(&pst2, Emax * 64 * 2));
    CK(hipMalloc(&pkg2, Emax * 64 * 8));
    CK(hipMalloc(&trk2, Emax * 64 * 8));
    CK(hipMemset(rob2, 0, Emax * 32 * 4));
    CK(hipMemset(pst2, 0, Emax * 64 * 2));
    CK(hipMemset(pkg2, 0, Emax * 64 * 8));
    CK(hipMemset(trk2, 0, Emax * 64 * 8));
    for (int pad = 0; pad < 3; pad++)   // packed, padded, packed + XCD-contiguous env ranges
        for (int wpb : {4, 16})
            for (int E : {1024, 4096})
                for (int mode = 0; mode < 2; mode++) {
                    const int sr = pad == 1 ? 32 : A, sp = pad == 1 ? 64 : P, ss = pad == 1 ? 64 : P;
                    std::vector<unsigned long long> med;
                    for (int it = 0; it < 40; it++) {
                        const int shift = (mode == 1 && (it & 1)) ? E / 2 + 4 : 0;
                        hipLaunchKernelGGL(k_soa_pad, dim3(E / wpb), dim3(64 * wpb), 0, 0, rob2, pkg2, pst2, trk2, es, E,
                                           shift, sr, sp, ss, wpb, pad == 2, cyc);
                        CK(hipDeviceSynchronize());
                        if (it < 10) continue;
                        CK(hipMemcpy(h.data(), cyc, E * 8, hipMemcpyDeviceToHost));
                        std::vector<unsigned long long> v(h.begin(), h.begin() + E);
                        std::sort(v.begin(), v.end());
                        med.push_back(v[E / 2]);
                    }
                    std::sort(med.begin(), med.end());
                    printf("{\"layout\": \"soa_%s\", \"waves_per_block\": %d, \"envs\": %d, \"mode\": \"%s\", "
                           "\"round_trip_cycles_median\": %llu}\n",
                           pad == 1 ? "padded" : pad == 2 ? "packed_xcd" : "packed", wpb, E,
                           mode == 0 ? "same" : "flip", med[med.size() / 2]);
                }
    for (int wpb : {4, 16})
        for (int E : {1024, 4096})
            for (int mode = 0; mode < 2; mode++) {
                std::vector<unsigned long long> med;
                for (int it = 0; it < 40; it++) {
                    const int shift = (mode == 1 && (it & 1)) ? E / 2 + 4 : 0;
                    hipLaunchKernelGGL(k_aos_full, dim3(E / wpb), dim3(64 * wpb), 0, 0, rec, E, shift, wpb, cyc);
                    CK(hipDeviceSynchronize());
                    if (it < 10) continue;
                    CK(hipMemcpy(h.data(), cyc, E * 8, hipMemcpyDeviceToHost));
                    std::vector<unsigned long long> v(h.begin(), h.begin() + E);
                    std::sort(v.begin(), v.end());
                    med.push_back(v[E / 2]);
                }
                std::sort(med.begin(), med.end());
                printf("{\"layout\": \"aos_full_xcd\", \"waves_per_block\": %d, \"envs\": %d, \"mode\": \"%s\", "
                       "\"round_trip_cycles_median\": %llu}\n", wpb, E, mode == 0 ? "same" : "flip", med[med.size() / 2]);
            }
    return 0;
}
