// mdl_rollout.hip -- device-resident rollout glue around the step engine
// (SURVEY.md §8(f)1): action sampling from policy logits and GAE, so a
// MAPPO rollout (MAPPO/trainer.py:133-290) never leaves the GPU.
//
//   k_sample  Categorical(logits).sample() + log_prob   MAPPO/trainer.py:141-143
//             (inverse CDF of softmax(logits) on a Philox4x32-10 uniform;
//             the stream is this library's own, keyed by (seed, offset, row))
//   k_gae     the GAE recursion of MAPPO/trainer.py:266-276, same float32
//             operation order as the reference's torch expressions
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdio.h>

#include "mdl_engine.h"
#include "mdl_kernels.hpp"

namespace mdl {

// Philox4x32-10 (Salmon et al. 2011), counter (c0..c3), key (k0, k1).
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = (uint32_t)p1;
        c[2] = n2;
        c[3] = (uint32_t)p0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// One row of logits per thread: u = philox(seed; offset, row)[0] >> 8 as a
// 24-bit uniform in [0, 1); action = first i with u*S < e_0+..+e_i where
// e_i = exp(l_i - max) and S = sum e_i (sequential fp32 sums); log_prob =
// (l_a - max) - log(S).  Rows whose logits are all -inf get action 0, -inf.
// off_dev (graph-capturable form): the offset is *off_dev + off_lo|off_hi<<32.
__global__ __launch_bounds__(256) void k_sample(const float* __restrict__ logits, int64_t n_rows, int n_act,
                                                uint32_t k0, uint32_t k1, uint32_t off_lo, uint32_t off_hi,
                                                const uint64_t* __restrict__ off_dev, uint8_t* __restrict__ actions,
                                                float* __restrict__ log_probs) {
    const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= n_rows) return;
    if (off_dev) {
        const uint64_t o = *off_dev + ((uint64_t)off_hi << 32 | off_lo);
        off_lo = (uint32_t)o;
        off_hi = (uint32_t)(o >> 32);
    }
    const float* l = logits + row * n_act;
    float m = -INFINITY;
    for (int i = 0; i < n_act; i++) m = fmaxf(m, l[i]);
    float S = 0.0f;
    for (int i = 0; i < n_act; i++) S = S + expf(l[i] - m);
    uint32_t c[4] = {off_lo, off_hi, (uint32_t)row, (uint32_t)(row >> 32)};
    philox4x32_10(c, k0, k1);
    const float u = (float)(c[0] >> 8) * 0x1p-24f;
    const float target = u * S;
    int a = -1, last = 0;
    float cum = 0.0f;
    for (int i = 0; i < n_act; i++) {
        const float ei = expf(l[i] - m);
        cum = cum + ei;
        if (ei > 0.0f) last = i;
        if (a < 0 && target < cum) a = i;
    }
    if (a < 0) a = last;  // u*S rounded up to the full sum
    actions[row] = (uint8_t)a;
    if (log_probs) log_probs[row] = (m == -INFINITY) ? -INFINITY : (l[a] - m) - logf(S);
}

// One env per thread, t = T-1 .. 0 (MAPPO/trainer.py:266-276):
//   nnt   = 1.0 - done[t]
//   nv    = t == T-1 ? next_value : values[t+1]
//   delta = (r[t] + (gamma * nv) * nnt) - values[t]
//   last  = delta + (gamma_lambda * nnt) * last        (last = 0 before t = T-1)
//   adv[t] = last;  ret[t] = adv[t] + values[t]
// gamma_lambda is float32(GAMMA * GAE_LAMBDA) formed in double, as the Python
// expression `GAMMA * GAE_LAMBDA * tensor` does.  Loads of step t-1 are issued
// ahead of step t's arithmetic (they do not depend on the recursion).
__global__ __launch_bounds__(256) void k_gae(const float* __restrict__ r, const float* __restrict__ v,
                                             const float* __restrict__ next_value,
                                             const uint8_t* __restrict__ dones, int T, int64_t n, float gamma,
                                             float gamma_lambda, float* __restrict__ adv, float* __restrict__ ret) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n || T <= 0) return;
    float last = 0.0f;
    float nv = next_value[e];
    int t = T - 1;
    float rt = r[(int64_t)t * n + e], vt = v[(int64_t)t * n + e];
    uint8_t dt = dones[(int64_t)t * n + e];
    for (; t >= 0; t--) {
        float rp = 0.0f, vp = 0.0f;
        uint8_t dp = 0;
        if (t > 0) {
            rp = r[(int64_t)(t - 1) * n + e];
            vp = v[(int64_t)(t - 1) * n + e];
            dp = dones[(int64_t)(t - 1) * n + e];
        }
        const float nnt = 1.0f - (dt ? 1.0f : 0.0f);
        const float delta = (rt + (gamma * nv) * nnt) - vt;
        last = delta + (gamma_lambda * nnt) * last;
        adv[(int64_t)t * n + e] = last;
        ret[(int64_t)t * n + e] = last + vt;
        nv = vt;
        rt = rp;
        vt = vp;
        dt = dp;
    }
}

__global__ void k_counter_add(uint64_t* __restrict__ c, uint64_t v) {
    if (threadIdx.x == 0) *c += v;
}

}  // namespace mdl

namespace {
thread_local char g_rerr[256];
int rfail(const char* msg, hipError_t e = hipSuccess) {
    if (e != hipSuccess) snprintf(g_rerr, sizeof g_rerr, "%s: %s", msg, hipGetErrorString(e));
    else snprintf(g_rerr, sizeof g_rerr, "%s", msg);
    mdl::set_error(g_rerr);
    return -1;
}
}  // namespace

extern "C" {

int mdl_sample_actions(const float* logits, int64_t n_rows, int32_t n_actions, uint64_t seed, uint64_t offset,
                       uint8_t* actions, float* log_probs, void* stream) {
    if (!logits || !actions) return rfail("mdl_sample_actions: null argument");
    if (n_rows < 0 || n_actions < 1 || n_actions > 256) return rfail("mdl_sample_actions: bad sizes");
    if (n_rows == 0) return 0;
    const int64_t blocks = (n_rows + 255) / 256;
    hipLaunchKernelGGL(mdl::k_sample, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, logits, n_rows,
                       (int)n_actions, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)offset,
                       (uint32_t)(offset >> 32), (const uint64_t*)nullptr, actions, log_probs);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : rfail("mdl_sample_actions: launch failed", e);
}

int mdl_sample_actions_dev(const float* logits, int64_t n_rows, int32_t n_actions, uint64_t seed,
                           const uint64_t* offset_dev, uint64_t offset_add, uint8_t* actions, float* log_probs,
                           void* stream) {
    if (!logits || !actions || !offset_dev) return rfail("mdl_sample_actions_dev: null argument");
    if (n_rows < 0 || n_actions < 1 || n_actions > 256) return rfail("mdl_sample_actions_dev: bad sizes");
    if (n_rows == 0) return 0;
    const int64_t blocks = (n_rows + 255) / 256;
    hipLaunchKernelGGL(mdl::k_sample, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, logits, n_rows,
                       (int)n_actions, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)offset_add,
                       (uint32_t)(offset_add >> 32), offset_dev, actions, log_probs);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : rfail("mdl_sample_actions_dev: launch failed", e);
}

int mdl_counter_add(uint64_t* counter, uint64_t value, void* stream) {
    if (!counter) return rfail("mdl_counter_add: null argument");
    hipLaunchKernelGGL(mdl::k_counter_add, dim3(1), dim3(64), 0, (hipStream_t)stream, counter, value);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : rfail("mdl_counter_add: launch failed", e);
}

int mdl_gae(const float* rewards, const float* values, const float* next_value, const uint8_t* dones, int32_t T,
            int64_t n, float gamma, float gamma_lambda, float* advantages, float* returns, void* stream) {
    if (!rewards || !values || !next_value || !dones || !advantages || !returns) return rfail("mdl_gae: null argument");
    if (T < 0 || n < 0) return rfail("mdl_gae: bad sizes");
    if (T == 0 || n == 0) return 0;
    const int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(mdl::k_gae, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, rewards, values,
                       next_value, dones, (int)T, n, gamma, gamma_lambda, advantages, returns);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : rfail("mdl_gae: launch failed", e);
}

}  // extern "C"
