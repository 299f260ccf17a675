// Probe (profiling only): host-side cost of replaying a hipGraph of N kernel launches as the
// bench does (the driver's 20-step timed region is one replay of a 20-kernel graph), against
// the kernel-argument size (8 B vs the step kernel's ~720 B StepArgs-sized struct) and the
// per-kernel work (empty, or a ~4 us busy wave per env like k_step at 4096 envs).
//   hipcc --offload-arch=gfx950 -O2 scripts/exp/graph_gaps.hip -o build/graph_gaps && build/graph_gaps
// One JSON line per case: wall and event microseconds per replay (medians of reps).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

struct Big {
    unsigned long long w[90];   // 720 bytes, like StepKarg + StepArgs
};

__device__ __forceinline__ void busy(unsigned long long ticks, int* sink) {
    if (ticks == 0) return;
    const unsigned long long t0 = wall_clock64();   // 100 MHz constant clock
    int x = 0;
    while (wall_clock64() - t0 < ticks) x++;
    if (x == -7) sink[0] = x;
}

__global__ __launch_bounds__(1024) void k_small(int* sink, unsigned long long ticks) { busy(ticks, sink); }
__global__ __launch_bounds__(1024) void k_big(Big b, int* sink, unsigned long long ticks) {
    busy(ticks + (b.w[3] & 1), sink);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    CK(hipSetDevice(0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int* sink;
    CK(hipMalloc(&sink, 64));
    Big b{};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int big = 0; big < 2; big++)
        for (unsigned long long ticks : {0ull, 300ull})   // 0 or ~3 us of busy time per wave
            for (int N : {20, 100}) {
                hipGraph_t g;
                hipGraphExec_t ge;
                CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
                for (int i = 0; i < N; i++) {
                    if (big) hipLaunchKernelGGL(k_big, dim3(256), dim3(1024), 0, s, b, sink, ticks);
                    else hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, s, sink, ticks);
                }
                CK(hipStreamEndCapture(s, &g));
                CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
                CK(hipGraphUpload(ge, s));
                CK(hipGraphLaunch(ge, s));
                CK(hipStreamSynchronize(s));
                std::vector<double> wall, ev;
                for (int r = 0; r < 30; r++) {
                    // some eager launches first, as the bench's warmup
                    for (int i = 0; i < 5; i++) hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, s, sink, ticks);
                    CK(hipStreamSynchronize(s));
                    const double t0 = now_us();
                    CK(hipEventRecord(e0, s));
                    CK(hipGraphLaunch(ge, s));
                    CK(hipEventRecord(e1, s));
                    CK(hipStreamSynchronize(s));
                    wall.push_back(now_us() - t0);
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    ev.push_back(ms * 1e3);
                }
                // the same N launches issued one by one from this host loop (no graph)
                std::vector<double> wall2, ev2;
                for (int r = 0; r < 30; r++) {
                    for (int i = 0; i < 5; i++) hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, s, sink, ticks);
                    CK(hipStreamSynchronize(s));
                    const double t0 = now_us();
                    CK(hipEventRecord(e0, s));
                    for (int i = 0; i < N; i++) {
                        if (big) hipLaunchKernelGGL(k_big, dim3(256), dim3(1024), 0, s, b, sink, ticks);
                        else hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, s, sink, ticks);
                    }
                    CK(hipEventRecord(e1, s));
                    CK(hipStreamSynchronize(s));
                    wall2.push_back(now_us() - t0);
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    ev2.push_back(ms * 1e3);
                }
                std::sort(wall.begin(), wall.end());
                std::sort(ev.begin(), ev.end());
                std::sort(wall2.begin(), wall2.end());
                std::sort(ev2.begin(), ev2.end());
                printf("{\"kernarg_bytes\": %d, \"busy_ticks\": %llu, \"nodes\": %d, \"wall_us_median\": %.1f, "
                       "\"event_us_median\": %.1f, \"wall_us_per_node\": %.2f, \"event_us_per_node\": %.2f, "
                       "\"loop_wall_us_per_launch\": %.2f, \"loop_event_us_per_launch\": %.2f}\n",
                       big ? (int)sizeof(Big) + 16 : 16, ticks, N, wall[15], ev[15], wall[15] / N, ev[15] / N,
                       wall2[15] / N, ev2[15] / N);
                CK(hipGraphExecDestroy(ge));
                CK(hipGraphDestroy(g));
            }
    return 0;
}
