// Host <-> GPU round-trip latency of the ways a single-env dict-API call could reach the
// device (one env per call: every path is latency, not bandwidth).  Standalone probe:
//   hipcc --offload-arch=gfx950 -O2 scripts/exp/latency.hip -o build/latency && build/latency
// Prints one JSON line of mean / median microseconds per round trip for each path.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void k_empty() {}

// writes seq into device memory (the stream-sync paths)
__global__ void k_dev(unsigned* d, unsigned seq) {
    if (threadIdx.x == 0) d[0] = seq;
}

// reads 8 bytes of host-mapped input, writes 64 bytes + a flag to host-mapped output
__global__ void k_host_io(const unsigned* in, unsigned* out, unsigned seq) {
    const unsigned v = __hip_atomic_load(&in[threadIdx.x & 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (threadIdx.x < 16) __hip_atomic_store(&out[1 + threadIdx.x], v + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if (threadIdx.x == 0) __hip_atomic_store(&out[0], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// persistent responder: polls a host-mapped doorbell; exits on STOP or after idle_ticks of
// the 100 MHz constant clock without a request (every wave reaches an exit)
__global__ void k_server(unsigned* db, unsigned* out, unsigned long long idle_ticks) {
    unsigned seen = 0;
    unsigned long long last = wall_clock64();
    for (;;) {
        const unsigned d = __hip_atomic_load(&db[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (d == 0xffffffffu) break;
        if (d != seen) {
            seen = d;
            const unsigned v = __hip_atomic_load(&db[1 + (threadIdx.x & 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (threadIdx.x < 16)
                __hip_atomic_store(&out[1 + threadIdx.x], v + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            if (threadIdx.x == 0) __hip_atomic_store(&out[0], d, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            last = wall_clock64();
        } else {
            if (wall_clock64() - last > idle_ticks) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (threadIdx.x == 0) __hip_atomic_store(&out[0], 0xfffffffeu, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static void stats(const char* name, std::vector<double>& v, bool last = false) {
    std::sort(v.begin(), v.end());
    double s = 0;
    for (double x : v) s += x;
    printf("\"%s\": {\"mean_us\": %.3f, \"median_us\": %.3f, \"p10_us\": %.3f, \"p90_us\": %.3f}%s", name, s / v.size(),
           v[v.size() / 2], v[v.size() / 10], v[v.size() * 9 / 10], last ? "" : ", ");
}

static inline unsigned vload(volatile unsigned* p) { return *p; }

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 2000;
    if (argc > 2 && atoi(argv[2]) == 1) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    CK(hipSetDevice(0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned* d;
    CK(hipMalloc(&d, 256));
    unsigned *hin, *hout, *pin;
    CK(hipHostMalloc((void**)&hin, 4096, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc((void**)&hout, 4096, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc((void**)&pin, 4096, hipHostMallocDefault));
    hin[0] = 7; hin[1] = 9;
    std::vector<double> v;
    printf("{");
    // 1. empty kernel + stream synchronize
    for (int i = 0; i < 50; i++) { k_empty<<<1, 64, 0, s>>>(); CK(hipStreamSynchronize(s)); }
    v.clear();
    for (int i = 0; i < N; i++) {
        const double t0 = now_us();
        k_empty<<<1, 64, 0, s>>>();
        CK(hipStreamSynchronize(s));
        v.push_back(now_us() - t0);
    }
    stats("launch_streamsync", v);
    // 2. launch only (host cost of the launch call)
    v.clear();
    for (int i = 0; i < N; i++) {
        const double t0 = now_us();
        k_empty<<<1, 64, 0, s>>>();
        v.push_back(now_us() - t0);
        CK(hipStreamSynchronize(s));
    }
    stats("launch_call_only", v);
    // 3. event record + event synchronize
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    v.clear();
    for (int i = 0; i < N; i++) {
        const double t0 = now_us();
        k_empty<<<1, 64, 0, s>>>();
        CK(hipEventRecord(ev, s));
        CK(hipEventSynchronize(ev));
        v.push_back(now_us() - t0);
    }
    stats("launch_eventsync", v);
    // 4. H2D 8 B + kernel + D2H 64 B + stream sync (the current dict path's shape)
    v.clear();
    for (int i = 0; i < N; i++) {
        const double t0 = now_us();
        CK(hipMemcpyAsync(d, pin, 8, hipMemcpyHostToDevice, s));
        k_dev<<<1, 64, 0, s>>>(d, i + 1);
        CK(hipMemcpyAsync(pin + 64, d, 64, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        v.push_back(now_us() - t0);
    }
    stats("h2d_kernel_d2h_streamsync", v);
    // 5. kernel reading / writing host-mapped memory, host spins on the flag (no sync call)
    v.clear();
    for (int i = 0; i < N; i++) {
        const unsigned seq = (unsigned)i + 1;
        const double t0 = now_us();
        k_host_io<<<1, 64, 0, s>>>(hin, hout, seq);
        while (vload(hout) != seq) {}
        v.push_back(now_us() - t0);
    }
    CK(hipStreamSynchronize(s));
    stats("launch_hostmapped_spin", v);
    // 6. persistent responder: doorbell in host memory, host spins on the response flag
    hout[0] = 0;
    hin[0] = 0;
    k_server<<<1, 64, 0, s>>>(hin, hout, 100000000ull /* 1 s idle */);
    for (int i = 0; i < 100; i++) {   // warm
        __atomic_store_n(&hin[1], (unsigned)i, __ATOMIC_RELAXED);
        __atomic_store_n(&hin[0], (unsigned)i + 1, __ATOMIC_RELEASE);
        while (vload(hout) != (unsigned)i + 1) {}
    }
    v.clear();
    for (int i = 100; i < 100 + N; i++) {
        const double t0 = now_us();
        __atomic_store_n(&hin[1], (unsigned)i, __ATOMIC_RELAXED);
        __atomic_store_n(&hin[0], (unsigned)i + 1, __ATOMIC_RELEASE);
        while (vload(hout) != (unsigned)i + 1) {}
        v.push_back(now_us() - t0);
    }
    __atomic_store_n(&hin[0], 0xffffffffu, __ATOMIC_RELEASE);
    CK(hipStreamSynchronize(s));
    const bool stopped = vload(hout) == 0xfffffffeu;
    stats("persistent_doorbell", v, true);
    printf(", \"server_stopped\": %s, \"n\": %d, \"spin_flag\": %d}\n", stopped ? "true" : "false", N,
           argc > 2 ? atoi(argv[2]) : 0);
    return 0;
}
