// FETCH_SIZE calibration for the step kernel's access shapes.
//
// rocprofv3's FETCH_SIZE on gfx950 is documented (MI355X_MICROARCH.md, HBM section) only for
// 16-B-per-lane streaming reads, where it reports exactly half of the bytes.  The step kernel
// (k_step, config 2: 4096 envs, one wave per env) instead reads short rows per env with narrow
// lanes: u8 x 5 (actions), u32 x 5 (robots), u16 x 50 (package states), u64 x 50 (package
// table, tracker data), one 16-B record.  Each kernel below reads ONE of those shapes (or all of
// them, "step_shape") with the step's launch geometry and a known algorithmic byte count, and
// writes 4 B per env so nothing is optimised away.  Run it under
//   rocprofv3 --pmc FETCH_SIZE -- build/fetch_cal
// and divide the per-dispatch FETCH_SIZE (KB) by the printed byte counts.  Two placements:
//   "hot"  -- the same buffers every launch (the step's situation: its state is re-read every step)
//   "cold" -- a rotation over 32 copies (123 MB), so no line can still be in an XCD's 4 MB L2.
// The 16-B/lane streaming read of 256 MB is the documented control (expected ratio 0.5).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int E = 4096, A = 5, P = 50, WPB = 16;   // config 2; the step's 16-wave workgroups at 4096 envs

struct Rows {
    const uint8_t* act;   // [E][A]
    const uint32_t* rob;  // [E][A]
    const uint16_t* pst;  // [E][P]
    const uint64_t* pkg;  // [E][P]
    const uint64_t* trk;  // [E][P]
    const uint4* es;      // [E]
};

// which: bit 0 act, 1 rob, 2 pst, 3 pkg, 4 trk, 5 es
template <int WHICH>
__global__ __launch_bounds__(64 * WPB) void k_rows(Rows r, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const int e = blockIdx.x * WPB + (threadIdx.x >> 6);
    if (e >= E) return;
    uint64_t acc = 0;
    if ((WHICH & 1) && lane < A) acc += r.act[(size_t)e * A + lane];
    if ((WHICH & 2) && lane < A) acc += r.rob[(size_t)e * A + lane];
    if ((WHICH & 4) && lane < P) acc += r.pst[(size_t)e * P + lane];
    if ((WHICH & 8) && lane < P) acc += r.pkg[(size_t)e * P + lane];
    if ((WHICH & 16) && lane < P) acc += r.trk[(size_t)e * P + lane];
    if ((WHICH & 32) && lane == 0) {
        const uint4 v = r.es[e];
        acc += v.x + v.y + v.z + v.w;
    }
    // a wave sum so every load is live; one 4-B store per env
    for (int o = 32; o; o >>= 1) acc += __shfl_xor((unsigned long long)acc, o);
    if (lane == 0) out[e] = (uint32_t)acc;
}

__global__ __launch_bounds__(256) void k_stream16(const uint4* __restrict__ src, size_t n16, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = src[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;   // practically never: keeps the loads
}

static size_t bytes_of(int which) {
    size_t b = 0;
    if (which & 1) b += (size_t)E * A;
    if (which & 2) b += (size_t)E * A * 4;
    if (which & 4) b += (size_t)E * P * 2;
    if (which & 8) b += (size_t)E * P * 8;
    if (which & 16) b += (size_t)E * P * 8;
    if (which & 32) b += (size_t)E * 16;
    return b;
}

template <int W>
static void run(const char* name, std::vector<Rows>& sets, uint32_t* out, int reps, hipStream_t s) {
    for (int rot = 0; rot < 2; rot++) {
        for (int i = 0; i < reps; i++) {
            const Rows& r = sets[rot ? (size_t)i % sets.size() : 0];
            hipLaunchKernelGGL(k_rows<W>, dim3(E / WPB), dim3(64 * WPB), 0, s, r, out);
        }
        CK(hipStreamSynchronize(s));
        printf("{\"kernel\": \"k_rows<%d>\", \"shape\": \"%s\", \"placement\": \"%s\", \"dispatches\": %d, "
               "\"algorithmic_read_bytes\": %zu, \"write_bytes\": %d}\n",
               W, name, rot ? "cold" : "hot", reps, bytes_of(W), E * 4);
    }
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 64;
    CK(hipSetDevice(0));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const int NSET = 32;
    std::vector<Rows> sets(NSET);
    std::vector<void*> allocs;
    for (int k = 0; k < NSET; k++) {
        auto mk = [&](size_t bytes) {
            void* p;
            CK(hipMalloc(&p, bytes));
            CK(hipMemset(p, k + 1, bytes));
            allocs.push_back(p);
            return p;
        };
        sets[k].act = (const uint8_t*)mk((size_t)E * A);
        sets[k].rob = (const uint32_t*)mk((size_t)E * A * 4);
        sets[k].pst = (const uint16_t*)mk((size_t)E * P * 2);
        sets[k].pkg = (const uint64_t*)mk((size_t)E * P * 8);
        sets[k].trk = (const uint64_t*)mk((size_t)E * P * 8);
        sets[k].es = (const uint4*)mk((size_t)E * 16);
    }
    uint32_t* out;
    CK(hipMalloc(&out, E * 4));
    run<1>("u8 x 5 per env (actions)", sets, out, reps, s);
    run<2>("u32 x 5 per env (robots)", sets, out, reps, s);
    run<4>("u16 x 50 per env (package states)", sets, out, reps, s);
    run<8>("u64 x 50 per env (package table)", sets, out, reps, s);
    run<16>("u64 x 50 per env (tracker data)", sets, out, reps, s);
    run<32>("16 B per env (env record)", sets, out, reps, s);
    run<63>("step_shape: all of the step's reads", sets, out, reps, s);
    // control: 16-B/lane streaming read of 256 MB (MI355X_MICROARCH.md: FETCH_SIZE = bytes / 2)
    const size_t big = 256ull << 20;
    void* src;
    CK(hipMalloc(&src, big));
    CK(hipMemset(src, 3, big));
    for (int i = 0; i < 8; i++) hipLaunchKernelGGL(k_stream16, dim3(4096), dim3(256), 0, s, (const uint4*)src, big / 16, out);
    CK(hipStreamSynchronize(s));
    printf("{\"kernel\": \"k_stream16\", \"shape\": \"16 B per lane streaming\", \"placement\": \"stream\", "
           "\"dispatches\": 8, \"algorithmic_read_bytes\": %zu, \"write_bytes\": 0}\n", big);
    for (void* p : allocs) CK(hipFree(p));
    CK(hipFree(src));
    CK(hipFree(out));
    return 0;
}
