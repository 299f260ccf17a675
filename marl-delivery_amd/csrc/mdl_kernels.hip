// mdl_kernels.hip -- gfx950 kernels of the marl-delivery batched step engine.
//
//   k_seed         RandomState(seed) + the constructor's reset  env.py:40-41
//   k_reset        Environment.reset()                          env.py:81-125
//   k_step<S,NCH>  Environment.step + compute_shaped_rewards + tracker update
//                  + reset-on-done                              env.py:173-316,
//                  MAPPO/helper.py:257-369, MAPPO/trainer.py:95-130,211-257
//   k_obs<S>       convert_observation / generate_vector_features /
//                  convert_global_state for every agent         MAPPO/helper.py:6-255
//   k_views_*      the same builders / shaping fed from packed dict views
//   k_export       int32 snapshot of the SoA state
//
// One wavefront per env; `wpb` envs per 256-thread workgroup, each with its
// own LDS slice of `lds_stride` bytes (dynamic shared memory).  Waves never
// block on each other, so a workgroup's envs may take different paths.
//
// k_step keeps the whole env in registers: robot a on lane a, package j on
// lane j%64 of chunk j/64 (NCH chunks, compile-time).  Cross-lane work is
// readlane / ballot only; LDS is touched only when an env resets.
#include <cstring>

#include "mdl_kernels.hpp"
#include "mdl_features.hpp"
#include "mdl_obs_small.hpp"
#include "mdl_altfeat.hpp"


namespace mdl {

// Diagnostic build only (scripts/exp/stamps.py): s_memtime at section
// boundaries of k_step, kept in SGPRs and stored once at the end; the
// scheduling barriers keep every instruction inside its section.
#ifdef MDL_STAMPS
__device__ uint64_t g_stamps[65536 * 16];
#define STAMP(k)                                      \
    do {                                              \
        __builtin_amdgcn_sched_barrier(0);            \
        stamp_[k] = __builtin_amdgcn_s_memtime();     \
        __builtin_amdgcn_sched_barrier(0);            \
    } while (0)
#else
#define STAMP(k) \
    do {         \
    } while (0)
#endif

// floats of the vector staging slice: max(actor rows of `na` agents, critic row)
__host__ __device__ inline int stage_floats(int A, int na, int MO, int MPc, int MR, int MPsc) {
    const int dc = actor_compact_dim(A, MO, MPc);
    const int a = actor_group(na, dc) * dc, cr = critic_compact_dim(A, MR, MPsc);
    return a > cr ? a : cr;
}

// --------------------------------------------------------------- reset LDS
struct ResetLds {
    uint64_t* pk;       // [P] new package table
    uint64_t* scratch;  // [P]
    uint32_t* mt;       // [624]
    uint16_t* taken;    // [64]
    uint8_t* pst;       // [P]
};

__host__ __device__ inline size_t reset_lds_bytes(int P) {
    return align16(8 * (size_t)P) * 2 + align16(4 * MT_N) + align16(2 * 64) + align16((size_t)P);
}

__device__ inline ResetLds reset_carve(unsigned char* b, int P) {
    ResetLds L;
    size_t o = 0;
    L.pk = (uint64_t*)(b + o); o += align16(8 * (size_t)P);
    L.scratch = (uint64_t*)(b + o); o += align16(8 * (size_t)P);
    L.mt = (uint32_t*)(b + o); o += align16(4 * MT_N);
    L.taken = (uint16_t*)(b + o); o += align16(2 * 64);
    L.pst = b + o;
    return L;
}

__device__ inline void load_mt(const DevParams& p, int e, uint32_t* key) {
    const uint32_t* g = p.mt + (size_t)e * MT_N;
    for (int i = lane_id(); i < MT_N; i += WAVE) key[i] = g[i];
    wave_sync();
}

__device__ inline void store_mt(const DevParams& p, int e, const uint32_t* key, int pos) {
    uint32_t* g = p.mt + (size_t)e * MT_N;
    for (int i = lane_id(); i < MT_N; i += WAVE) g[i] = key[i];
    if (lane_id() == 0) p.mt_pos[e] = pos;
}

// One Environment.reset() (env.py:81-125) into LDS; returns this lane's robot cell.
__device__ inline int do_reset(const DevParams& p, int e, const MapDesc& md, ResetLds& L, bool seeded_in_lds) {
    if (!seeded_in_lds) load_mt(p, e, L.mt);
    MTState ms{L.mt, seeded_in_lds ? MT_N : p.mt_pos[e]};
    const int cell = reset_env(ms, p, md, L.pk, L.pst, L.scratch, L.taken);
    store_mt(p, e, L.mt, ms.pos);
    return cell;
}

// Tracker update on lane-resident package state (MAPPO/trainer.py:95-130):
// insert ids spawned at t that are absent (in id order), then carried ->
// in_transit, in_transit & not carried -> delete.  An inserted entry's order
// key is implicit (ORD_EPISODE + slot) until the next reset.
template <int NCH, int AU = 0>
__device__ inline void tracker_update_regs(uint32_t (&ps)[NCH], uint64_t (&td)[NCH], bool (&dirty)[NCH],
                                           const uint64_t (&pk)[NCH], int P, int A, int carry, int t) {
    const int lane = lane_id();
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        const int j = c * WAVE + lane;
        // selects, not branches: a branch here costs a vector-to-scalar hand-off
        const bool ins = (j < P) & (pk_st(pk[c]) == t) & !(ps[c] & PS_PRESENT);
        ps[c] = ins ? ((ps[c] & PS_STATUS) | PS_PRESENT) : ps[c];
        td[c] = ins ? pk[c] : td[c];
        dirty[c] = dirty[c] || ins;
    }
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        const int id = c * WAVE + lane + 1;
        bool carried = false;
        if constexpr (AU > 0) {  // A <= AU: lanes >= A carry 0 and ids start at 1, so no bound is needed
            uint32_t ci[AU], mn = 0xffffffffu;  // min of (carry_i ^ id): zero iff some robot carries id
#pragma unroll
            for (int i = 0; i < AU; i++) ci[i] = (uint32_t)rdl(carry, i);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < AU; i++) mn = min(mn, ci[i] ^ (uint32_t)id);
            carried = mn == 0u;
        } else {
            for (int i = 0; i < A; i++) carried |= rdl(carry, i) == id;
        }
        const uint32_t upd = carried ? (ps[c] | PS_TRANSIT) : (ps[c] & PS_TRANSIT) ? (ps[c] & PS_STATUS) : ps[c];
        ps[c] = (ps[c] & PS_PRESENT) ? upd : ps[c];
    }
}

// The same update with the carried test precomputed: bit c of `carried_bits` (this lane)
// is set when some robot carries id c * 64 + lane + 1.
template <int NCH>
__device__ inline void tracker_update_bits(uint32_t (&ps)[NCH], uint64_t (&td)[NCH], bool (&dirty)[NCH],
                                           const uint64_t (&pk)[NCH], int P, int t, uint32_t carried_bits) {
    const int lane = lane_id();
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        const int j = c * WAVE + lane;
        const bool ins = (j < P) & (pk_st(pk[c]) == t) & !(ps[c] & PS_PRESENT);
        ps[c] = ins ? ((ps[c] & PS_STATUS) | PS_PRESENT) : ps[c];
        td[c] = ins ? pk[c] : td[c];
        dirty[c] = dirty[c] || ins;
        const bool carried = (carried_bits >> c) & 1u;
        const uint32_t upd = carried ? (ps[c] | PS_TRANSIT) : (ps[c] & PS_TRANSIT) ? (ps[c] & PS_STATUS) : ps[c];
        ps[c] = (ps[c] & PS_PRESENT) ? upd : ps[c];
    }
}

// Reset with a persistent tracker: every present entry becomes a survivor
// whose key is its rank in the current dict order (keys `tq`: survivor rank
// or ORD_EPISODE + slot, distinct), so keys stay below ORD_EPISODE forever.
// The new rank lands in the state word's rank bits (and in `tq`).
template <int NCH>
__device__ inline void survivors_at_reset(uint32_t (&ps)[NCH], uint32_t (&tq)[NCH], int P) {
    const int lane = lane_id();
    uint32_t rk[NCH];
#pragma unroll
    for (int c = 0; c < NCH; c++) rk[c] = 0;
#pragma unroll
    for (int c2 = 0; c2 < NCH; c2++) {
        uint64_t m = ballot(c2 * WAVE + lane < P && (ps[c2] & PS_PRESENT));
        while (m) {
            const uint32_t ki = (uint32_t)rdl((int)tq[c2], ffs64(m));
            m &= m - 1;
#pragma unroll
            for (int c = 0; c < NCH; c++) rk[c] += ki < tq[c] ? 1u : 0u;
        }
    }
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        if (c * WAVE + lane < P && (ps[c] & PS_PRESENT)) {
            tq[c] = rk[c];
            ps[c] = (ps[c] & PS_FLAGS) | PS_SURVIVOR | (rk[c] << PS_RANK_SHIFT);
        } else {
            ps[c] &= PS_STATUS;
        }
    }
}

// ------------------------------------------------------------------ seed
__global__ __launch_bounds__(256) void k_seed(DevParams p, const uint32_t* __restrict__ seeds, int wpb,
                                              int lds_stride) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = wave_id();
    const int lane = lane_id();
    const int e = blockIdx.x * wpb + wave;
    if (wave >= wpb || e >= p.E) return;
    ResetLds L = reset_carve(smem + (size_t)wave * lds_stride, p.P);
    const MapDesc md = p.maps[p.env_map ? p.env_map[e] : 0];
    if (lane == 0) {  // init_genrand: a serial recurrence
        uint32_t s = seeds[e];
        for (int i = 0; i < MT_N; i++) {
            L.mt[i] = s;
            s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
        }
    }
    wave_sync();
    const int cell = do_reset(p, e, md, L, true);
    if (lane < p.A)
        p.rob[(size_t)e * p.A + lane] = rob_pack(cell, 0, p.movevalid[md.grid_off + cell_r(cell) * md.W + cell_c(cell)]);
    for (int j = lane; j < p.P; j += WAVE) {
        const size_t g = (size_t)e * p.P + j;
        p.pkg[g] = L.pk[j];
        p.pstate[g] = L.pst[j];  // tracker empty (MAPPO/trainer.py:92)
    }
    if (lane == 0) {
        EnvScalars s;
        s.t = 0;
        s.ctr = 0;
        s.total = 0.0;
        p.es[e] = s;
        p.ep_total[e] = 0.0;
        p.ep_len[e] = 0;
    }
}

// ------------------------------------------------------------------ reset
// Environment.reset() for listed envs.  Stale tracker: present entries become
// survivors, then the update with the reset state (no clear).
template <int NCH>
__global__ __launch_bounds__(256) void k_reset(DevParams p, const int* __restrict__ env_ids, int n, int wpb,
                                               int lds_stride) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = wave_id();
    const int lane = lane_id();
    const int w = xcd_block() * wpb + wave;
    if (wave >= wpb || w >= n) return;
    const int e = env_ids ? env_ids[w] : w;
    if ((unsigned)e >= (unsigned)p.E) return;  // device-side ids: out of range -> skipped
    const int A = p.A, P = p.P;
    ResetLds L = reset_carve(smem + (size_t)wave * lds_stride, P);
    const MapDesc md = p.maps[p.env_map ? p.env_map[e] : 0];
    uint32_t ps[NCH], tq[NCH];
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        const int j = c * WAVE + lane;
        ps[c] = j < P ? p.pstate[(size_t)e * P + j] : 0u;
        tq[c] = (p.stale && (ps[c] & PS_SURVIVOR)) ? ps[c] >> PS_RANK_SHIFT : ORD_EPISODE + (uint32_t)j;
    }
    const int cell = do_reset(p, e, md, L, false);
    uint64_t pk[NCH], td[NCH];
    bool dirty[NCH];
    if (p.stale) survivors_at_reset<NCH>(ps, tq, P);
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        const int j = c * WAVE + lane;
        pk[c] = j < P ? L.pk[j] : 0;
        ps[c] = (j < P ? L.pst[j] : 0u) | (p.stale ? (ps[c] & ~PS_STATUS) : 0u);
        td[c] = pk[c];
        dirty[c] = false;
    }
    if (p.stale) tracker_update_regs<NCH>(ps, td, dirty, pk, P, A, 0, 0);
    if (lane < A)
        p.rob[(size_t)e * A + lane] = rob_pack(cell, 0, p.movevalid[md.grid_off + cell_r(cell) * md.W + cell_c(cell)]);
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        const int j = c * WAVE + lane;
        if (j < P) {
            const size_t g = (size_t)e * P + j;
            p.pkg[g] = pk[c];
            p.pstate[g] = (uint16_t)ps[c];
            if (dirty[c]) p.trk[g] = td[c];
        }
    }
    if (lane == 0) {
        EnvScalars s;
        s.t = 0;
        s.ctr = 0;
        s.total = 0.0;
        p.es[e] = s;
    }
}

__global__ __launch_bounds__(256) void k_tracker_clear(DevParams p, const int* __restrict__ env_ids, int n) {
    const int wave = wave_id();
    const int w = blockIdx.x * 4 + wave;
    if (w >= n) return;
    const int e = env_ids ? env_ids[w] : w;
    if ((unsigned)e >= (unsigned)p.E) return;
    for (int j = lane_id(); j < p.P; j += WAVE) {
        const size_t g = (size_t)e * p.P + j;
        p.pstate[g] &= (uint16_t)PS_STATUS;
    }
    if (lane_id() == 0) p.es[e].ctr = 0;
}

// ------------------------------------------------------------------- step
// FUSED (bench mode): K consecutive steps of each env in
// one launch with the state held in registers between them; actions [K][n][A],
// outputs [K][n].  FUSED=false is the API's one step per launch (K = 1).
// at most 4 waves per workgroup (the engine's step_wpb)
#define MDL_STEP_LB 256
// Waves per SIMD the step kernels (k_step, k_step_obs) are compiled for.  Left to itself the
// compiler spends 106 SGPRs, which allows 7 waves per SIMD; amdgpu_waves_per_eu(8) keeps the SGPRs
// within the 8-wave budget at the same instruction count (+1 VALU).  Same-box A/B
// (profiles/r03/wpe8_ab.txt): config 5 (131072 envs) 113.7 -> 99.5 us per step, its 16384-env slice
// 16.6 -> 15.3, config 4 34.3 -> 31.5; config 2 (4 waves per SIMD) and k_step_obs unchanged;
// the general builder k_obs 1.3 % slower with it, so it keeps the compiler's choice.
// Only the one- and two-chunk (P <= 128) per-launch forms: the fused bench kernel and the wider
// package chunkings need more registers than the 8-wave budget and would spill (1 = no constraint).
template <int NCH, bool FUSED>
constexpr int step_wpe() { return (NCH <= 2 && !FUSED) ? 8 : 1; }
#define MDL_STEP_ATTR(NCH, FUSED) __attribute__((amdgpu_waves_per_eu(step_wpe<NCH, FUSED>())))
// AU > 0: A <= AU robots (AU = 8, or AU = A exactly for the configs' A = 5 and 16) -- the
// per-robot scans are unrolled over AU lanes (independent
// readlanes, no loop-carried branch), the latency-critical form at the configs' A = 5.
// The step kernel's arguments as one struct: its layout is the kernarg segment's,
// so the write-back can fetch its pointers from the segment in one late batch.
struct StepArgs {
    DevParams p;
    const uint8_t* actions;
    const int* env_ids;
    double* r_out;
    float* sh_out;
    uint8_t* done_out;
    int fmt, n, auto_reset, wpb, lds_stride, K;
};
typedef __attribute__((address_space(4))) const StepArgs* KargPtr;
static_assert(sizeof(StepArgs) + 256 <= 4096, "the step's kernel arguments stay inside the 4 KiB kernarg segment");

// The step kernel's leading arguments are preloaded into SGPRs by the command
// processor (gfx950 kernarg preloading, -amdgpu-kernarg-preload-count=14 for this
// file: 14 dwords): the state pointers, A | P << 16 and n | wpb << 24 | flags.  So
// the state loads issue at wave start, overlapping the kernel-argument fetch
// instead of waiting for it.  StepKarg mirrors the kernarg layout.
struct StepKarg {
    const uint32_t* rob;
    const uint64_t* pkg;
    const uint16_t* pst;
    const u32x4* es;
    const uint64_t* trk;
    const uint8_t* act;
    uint32_t ap, nw;
    StepArgs args;
};
constexpr uint32_t NW_IDS = 1u << 29, NW_MAP = 1u << 30;
// k_step_halves: every map of the engine fits 64 x 64 (the pick-ups' 4096-bit cell maps)
constexpr uint32_t NW_SMALLMAP = 1u << 31;
// ap = A (7 bits) | P << 7 (11 bits) | the launch's block count << AP_NB_SHIFT (0 when it does not
// fit: launch-order slots)
constexpr int AP_NB_SHIFT = 18;
inline uint32_t pack_ap(int A, int P, int nblocks) {
    const uint32_t nb = nblocks < (1 << (32 - AP_NB_SHIFT)) ? (uint32_t)nblocks : 0u;
    return (uint32_t)A | ((uint32_t)P << 7) | (nb << AP_NB_SHIFT);
}

// The fused step + observation launch's extra arguments (after StepArgs in its kernarg
// segment, so the StepKarg prefix -- preloaded SGPRs, the late kernarg batch -- is the same).
struct ObsArgs {
    float* amap;
    float* avec;
    float* cmap;
    float* cvec;
};

// the completion tail of a Publish launch (every wave of the grid runs it, or the `expect`
// waves that reach it); a one-wave launch (ctr == nullptr) publishes straight after its release
__device__ __forceinline__ void publish_tail(const Publish& pb) {
    __atomic_thread_fence(__ATOMIC_RELEASE);   // this wave's stores, before it is counted
    if (!pb.ctr) {
        if (lane_id() == 0) __hip_atomic_store(pb.seq, pb.value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    if (lane_id() == 0) {
        const unsigned waves = pb.expect ? pb.expect : gridDim.x * (blockDim.x / WAVE);
        if (atomicAdd(pb.ctr, 1u) - pb.base == waves - 1u) {   // the last wave of the grid
            __atomic_thread_fence(__ATOMIC_ACQ_REL);
            __hip_atomic_store(pb.seq, pb.value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// The dict-API mailbox step's extra arguments (mdl_mail_step): the rows of the envs it steps go
// straight from the wave's registers into the engine's host-mapped mailbox (k_mail_export's
// layout), then the launch publishes the call's completion word.  Up to MAIL_INLINE_CODES action
// bytes travel here in the kernel arguments (no round trip to host memory for them).
constexpr int MAIL_INLINE_CODES = 256;
struct MailArgs {
    MailRows m;
    Publish pb;
    uint8_t codes[MAIL_INLINE_CODES];
};

// The step kernel's body.  OBS (NCH = 1, A <= 8, k_obs_small's configurations): after the
// write-back the wave builds the env's observations of the new state from the registers the
// step leaves (robots on lanes < A, package j on lane j), as MAPPO/trainer.py:229-286 does
// after every env.step -- one launch and no state reload instead of k_step + k_obs_small.
// MAIL: after the write-back the wave writes its env's mailbox rows and counts itself toward
// the call's completion word (MailArgs).
// Sixteen-robot movement test: lane L compares robot L & 15 with robot 4 (L >> 4) + k;
// the lanes where that partner has the lower index.
__host__ __device__ constexpr uint64_t move_lt_lanes(int k) {
    uint64_t m = 0;
    for (int l = 0; l < 64; l++)
        if (((l >> 4) << 2) + k < (l & 15)) m |= 1ull << l;
    return m;
}

template <bool STALE, int NCH, bool FUSED, int AU, bool OBS, bool MAIL = false>
__device__ __forceinline__ void step_body(const uint32_t* __restrict__ rob_pre, const uint64_t* __restrict__ pkg_pre,
                                          const uint16_t* __restrict__ pst_pre, const u32x4* __restrict__ es_pre,
                                          const uint64_t* __restrict__ trk_pre, const uint8_t* __restrict__ act_pre,
                                          uint32_t ap, uint32_t nw, const StepArgs& args, const ObsArgs& oa,
                                          const MailArgs* ma = nullptr) {
    static_assert(!OBS || (NCH == 1 && !FUSED && AU > 0 && AU <= 8), "fused observations: P <= 64, A <= 8");
    extern __shared__ __align__(16) unsigned char smem[];
    const DevParams& p = args.p;
    // (the other scalar arguments are read only after the state loads are issued: read
    // here, their scalar loads would be hoisted in between and waited for)
#ifdef MDL_STAMPS
    uint64_t stamp_[16];
#endif
    STAMP(0);
    // Preloaded (SGPR) arguments: everything the state loads need.
    const int A = (int)(ap & 0x7fu), P = (int)((ap >> 7) & 0x7ffu);
    const int n_ = (int)(nw & 0xffffffu), wpb_ = (int)((nw >> 24) & 31u);
    GLOBAL const uint32_t* robp = (GLOBAL const uint32_t*)rob_pre;
    GLOBAL const uint64_t* pkgp = (GLOBAL const uint64_t*)pkg_pre;
    GLOBAL const uint16_t* pstp = (GLOBAL const uint16_t*)pst_pre;
    GLOBAL const u32x4* esp = (GLOBAL const u32x4*)es_pre;   // EnvScalars {t, ctr, total lo, total hi}
    GLOBAL const uint64_t* trkp = (GLOBAL const uint64_t*)trk_pre;
    GLOBAL const uint8_t* actp = (GLOBAL const uint8_t*)act_pre;
    STAMP(1);

    const int wave = wave_id();
    const int lane = lane_id();
    // XCD-contiguous workgroup slots (xcd_block) from the block count packed in `ap` (a preloaded
    // SGPR: gridDim.x would cost a dispatch-packet load ahead of every state load); 0 = launch order
    const int nbp = (int)(ap >> AP_NB_SHIFT);
    const int w = (nbp ? xcd_slot((int)blockIdx.x, nbp) : (int)blockIdx.x) * wpb_ + wave;
    if (wave >= wpb_ || w >= n_) return;
    int e = w;
    if (nw & NW_IDS) {   // subset stepping: one more load; an id outside [0, E) is skipped
        e = uni(((GLOBAL const int*)args.env_ids)[w]);
        if ((unsigned)e >= (unsigned)args.p.E) return;
    }

    STAMP(2);
    // ---- loads: one round trip, everything independent ----
    const bool act = lane < A;
    const uint32_t rv = act ? robp[(size_t)e * A + lane] : 0u;
    int araw = act ? (int)actp[(size_t)w * A + lane] : 0;
    uint64_t pk[NCH], td[NCH];
    uint32_t ps[NCH], ps_in[NCH], tq[NCH];
    bool dirty[NCH];
    // the env's rows as scalar bases: each load is one SGPR base + a 32-bit lane offset
    GLOBAL const uint64_t* pkge = pkgp + (size_t)e * P;
    GLOBAL const uint16_t* pste = pstp + (size_t)e * P;
    GLOBAL const uint64_t* trke = trkp + (size_t)e * P;
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        const int j = c * WAVE + lane;
        pk[c] = 0;
        ps[c] = 0;
        td[c] = 0;
        tq[c] = 0;
        dirty[c] = false;
        if constexpr (NCH == 1) {
            if (j < P) {
                pk[c] = pkge[(uint32_t)j];
                ps[c] = pste[(uint32_t)j];
                if (STALE) td[c] = trke[(uint32_t)j];
            }
        } else {
            // Several chunks: every lane loads (slot 0 where j >= P, discarded below).  As one
            // exec-masked block per chunk, the copies out of each block waited for its loads, so
            // each chunk's loads issued only after the previous chunk's had returned.
            const uint32_t o = j < P ? (uint32_t)j : 0u;
            pk[c] = pkge[o];
            ps[c] = pste[o];
            if (STALE) td[c] = trke[o];
        }
    }
    const u32x4 esv = esp[e];
    __builtin_amdgcn_sched_barrier(0);  // every load above is issued before any use
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        if constexpr (NCH > 1) {
            const bool jv = c * WAVE + lane < P;
            pk[c] = jv ? pk[c] : 0ull;
            ps[c] = jv ? ps[c] : 0u;
            td[c] = jv ? td[c] : 0ull;
        }
        ps_in[c] = ps[c];
    }
    // The other kernel arguments, fetched now in one scalar batch while the state
    // loads are in flight, and pinned by ONE asm statement (one wait; separate pins let
    // the compiler wait after the first few and issue the rest behind that wait).  The
    // batch touches every kernarg line the step reads later, so those hit the cache.
    double* __restrict__ r_out = args.r_out;
    const int fmt = args.fmt, auto_reset = args.auto_reset, lds_stride = args.lds_stride, K = args.K;
    int T = p.T;
    GLOBAL const uint8_t* env_map = (GLOBAL const uint8_t*)p.env_map;
    int mvoff = p.maps[0].mvc_off;
    int fmt_ = fmt;
    float c_touch = p.shaping[8];
    const uint8_t* c_touch2 = p.movevalid_cell;
    double* c_touch3 = r_out;
    double c_touch4 = p.cost_sum[0], c_touch5 = p.cost_sum[8];
    int c_touch6 = lds_stride;
    asm volatile(""
                 : "+s"(T), "+s"(env_map), "+s"(mvoff), "+s"(fmt_), "+s"(c_touch), "+s"(c_touch2),
                   "+s"(c_touch3), "+s"(c_touch4), "+s"(c_touch5), "+s"(c_touch6));
    int mi = 0;
    if (nw & NW_MAP) {
        mi = uni(env_map[e]);
        mvoff = p.maps[mi].mvc_off;
    }
    int cell = rob_cell(rv), carry = rob_carry(rv);
    uint32_t vmask = rob_valid(rv);
    int t_cur = (int)esv.x;
    double tot_cur = __hiloint2double((int)esv.w, (int)esv.z);
    bool any_rst = false;
    GLOBAL double* rop;
    GLOBAL float* shp;
    GLOBAL uint8_t* dnp;
    GLOBAL uint32_t* robw;
    GLOBAL uint16_t* pstw;
    GLOBAL uint64_t* trkw;
    GLOBAL u32x4* esw;
    const int KK = FUSED ? K : 1;
    uint32_t rfl = 0;   // the last step's reward terms (EnvScalars::rterms)
    for (int k = 0; k < KK; k++) {
        int mv, op;
        decode_action(araw, fmt_, mv, op);   // every lane (no exec-masked block), then masked
        mv = act ? mv : MV_S;
        op = act ? op : 0;
        if (FUSED && k + 1 < KK) araw = act ? (int)actp[((size_t)(k + 1) * n_ + w) * A + lane] : 0;
        const int t0 = t_cur;
        uint32_t ps0[NCH];
#pragma unroll
        for (int c = 0; c < NCH; c++) ps0[c] = ps[c];
        // tracker_prev view: data / iteration order key (< 0x800) per slot
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            const int j = c * WAVE + lane;
            if (!STALE || !(ps0[c] & PS_SURVIVOR)) {
                td[c] = pk[c];
                tq[c] = STALE ? ORD_EPISODE + (uint32_t)j : (uint32_t)j;
            } else {
                tq[c] = ps0[c] >> PS_RANK_SHIFT;
            }
        }

        // The pre-step carried package of each robot, gathered from its package lane
        // now (ds_bpermute) so the LDS round trip overlaps the movement: its table
        // entry (drops), its tracker_prev entry and flags (shaped reward).
        const int pj = carry - 1;
        uint32_t g_pf = 0;
        uint64_t g_td = 0, g_pk = 0;
#pragma unroll
        for (int c = 0; c < NCH && !(MDL_ABLATE & 64); c++) {
            const int src = (pj & 63) << 2;
            const uint32_t f = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)ps0[c]);
            const uint32_t tlo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)td[c]);
            const uint32_t thi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(td[c] >> 32));
            const uint32_t plo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)pk[c]);
            const uint32_t phi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(pk[c] >> 32));
            if ((pj >> 6) == c) {
                g_pf = f;
                g_td = (uint64_t)tlo | ((uint64_t)thi << 32);
                g_pk = (uint64_t)plo | ((uint64_t)phi << 32);
            }
        }

        // The shaped reward's candidates (tracker_prev's waiting entries, MAPPO/helper.py:257-369):
        // pre-step state only, so computed here, where they can fill the movement's dependent
        // readlane chain instead of waiting behind it.
        bool wv[NCH];
        int stc[NCH];
        uint32_t klo[NCH];  // low key bits: order key << 10 | slot, or ~0 for no candidate
        uint64_t wvm[NCH], anyw = 0;
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            const uint32_t f = ps0[c];
            const bool waiting = STALE ? ((f & PS_PRESENT) && !(f & PS_TRANSIT)) : ((f & PS_STATUS) == ST_WAITING);
            wv[c] = waiting && pk_st(td[c]) <= t0;
            stc[c] = pk_start(td[c]);
            klo[c] = wv[c] ? (tq[c] << 10) | (uint32_t)(c * WAVE + lane) : 0xffffffffu;
            wvm[c] = ballot(wv[c]);
            anyw |= wvm[c];
        }

        STAMP(3);
        // ---- movement (env.py:188-257) ----
        // moved = least fixed point of
        //   moved[i] = mover[i] & winner(prop[i]) == i & (occ(prop[i]) none | moved[occ])
        // winner = lowest-index mover into the cell: the reference's restart-from-0
        // loop, checked against the oracle's literal restatement.
        const int pcell = cell, pcarry = carry;
        // bits 1..4 of vmask only: S / other moves never move; L -256, R +256, U -1, D +1
        // the cell delta of each move code from one 64-bit table of 10-bit entries
        // (S 0, L -256, R +256, U -1, D +1, other 0), masked by the move's validity bit
        constexpr uint64_t DTAB = (uint64_t)(0x3ffu & (uint32_t)-256) << 10 | (uint64_t)256 << 20 |
                                  (uint64_t)(0x3ffu & (uint32_t)-1) << 30 | (uint64_t)1 << 40;
        const int dtab = __builtin_amdgcn_sbfe((int)(uint32_t)(DTAB >> (10 * mv)), 0, 10);
        const int vok = __builtin_amdgcn_sbfe((int)vmask, mv, 1);   // 0 or -1
        const int dlt = dtab & vok;
        const int prop = cell + (int)(lmask(act) & (uint32_t)dlt);   // a vector mask: no exec-masked block
        const bool mover = !(MDL_ABLATE & 4) && act && prop != cell;
        const uint64_t movers = ballot(mover);
        // the proposed cell's move-validity bits, fetched now (every mover) so the load
        // overlaps the resolution below; consumed only at write-back, for robots that moved
        // (every lane loads: prop is a cell of the map on every lane, 0 on lanes >= A)
        uint32_t pvm = (MDL_ABLATE & 16) ? vmask : (uint32_t)(p.movevalid_cell + mvoff)[(uint32_t)prop];
        uint64_t moved = 0;
        STAMP(12);
        if (movers) {
            // blocked: a lower-index mover proposes the same cell; occ: the robot
            // now standing on the proposed cell (robots stand on distinct cells)
            int blocked = 0, occ = -1;
            if constexpr (AU == 16) {
                // Sixteen robots: lane l tests robot i = l & 15 against robots j = 4g..4g+3
                // (g = l >> 4, the lane group), fetched by ds_bpermute; the four groups' answers
                // are combined so that lanes 0..15 end with robot i's -- 4 fetches instead of
                // 32 readlanes, 32 compares and 32 selects.  A mover is a robot whose proposal
                // differs from its cell.  One word per robot: its proposal if it moves (0xffff otherwise: a non-mover
                // blocks nobody) | its cell << 16 (0xfffe on lanes >= A), so one fetch per
                // partner; the "lower-index" test is a constant lane mask per k, and the
                // blocked hits of the four groups are ORed on the scalar unit.
                const uint32_t wd = ((act && prop != cell) ? (uint32_t)prop : 0xffffu) |
                                    ((act ? (uint32_t)cell : 0xfffeu) << 16);
                const int i = lane & 15, g4 = (lane >> 4) << 2;
                const uint32_t pi = (uint32_t)__builtin_amdgcn_ds_bpermute(i << 2, act ? prop : 0xfffd);
                uint32_t wj[4];
#pragma unroll
                for (int k = 0; k < 4; k++) wj[k] = (uint32_t)__builtin_amdgcn_ds_bpermute((g4 + k) << 2, (int)wd);
                uint64_t H = 0;
                int oc = -1;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    H |= ballot((wj[k] & 0xffffu) == pi) & move_lt_lanes(k);
                    oc = (wj[k] >> 16) == pi ? g4 + k : oc;   // robots stand on distinct cells: one match at most
                }
                oc = max(oc, (int)xor_lane<16>((uint32_t)oc));
                oc = max(oc, (int)xor_lane<32>((uint32_t)oc));
                const uint64_t h16 = (H | (H >> 16) | (H >> 32) | (H >> 48)) & 0xffffull;
                blocked = sel64(h16, 0u, 1u) != 0u;
                occ = oc;
            } else if constexpr (AU > 0) {
                // Every test is one compare of this lane's proposal against a readlane'd
                // scalar, folded into vector registers (hit bits / occupant index): the
                // chain never hands a vector result to the scalar unit, whose forwarding
                // latency (~20 cycles per hand-off) would otherwise set the pace.
                // Lanes >= A read as sentinels that match no cell.
                const int propx = act ? prop : -2, cellx = act ? cell : -3;
                // Three phases kept apart so no instruction waits on the one before it:
                // all readlanes, all compares, then the selects.
                int pj[AU], cj[AU];
#pragma unroll
                for (int j = 0; j < AU; j++) {
                    pj[j] = rdl(propx, j);
                    cj[j] = rdl(cellx, j);
                }
                __builtin_amdgcn_sched_barrier(0);
                bool hj[AU], oj[AU];
#pragma unroll
                for (int j = 0; j < AU; j++) {
                    hj[j] = pj[j] == prop;
                    oj[j] = cj[j] == prop;
                }
                __builtin_amdgcn_sched_barrier(0);
                uint32_t hit = 0;
#pragma unroll
                for (int j = 0; j < AU; j++) {
                    hit |= hj[j] ? (1u << j) : 0u;
                    occ = oj[j] ? j : occ;
                }
                // a lower-index mover into the same cell (only lanes < A are movers)
                blocked = (hit & ((1u << (lane & 31)) - 1u) & (uint32_t)movers) != 0u;
            } else {
                for (uint64_t m = movers; m; m &= m - 1) {
                    const int j = ffs64(m);
                    blocked |= (int)(j < lane) & (int)(rdl(prop, j) == prop);
                }
                for (int j = 0; j < A; j++) occ = rdl(cell, j) == prop ? j : occ;
            }
            STAMP(13);
            STAMP(14);
            const uint32_t Mbase = lmask(mover && !blocked), Mfree = lmask(occ < 0);
            moved = ballot((Mbase & Mfree) != 0u);
            if (ballot((Mbase & ~Mfree) != 0u)) {  // some walk into an occupied cell: resolve the chains
                for (int it = 0; it < A; it++) {
                    const uint64_t nm = ballot((Mbase & (Mfree | vbit(moved, occ & 63))) != 0u);
                    if (nm == moved) break;
                    moved = nm;
                }
            }
            STAMP(15);
            if ((moved >> lane) & 1ull) {
                cell = prop;

            }
        }
        const int n_cost = popc64(moved);

        STAMP(4);
        // ---- package actions (env.py:259-292) ----
        // Robots sit on distinct cells, so pick-ups of different robots take from
        // disjoint package sets and drops touch only carried packages: the robot
        // order of the reference loop cannot change any outcome.
        uint64_t pickers = ballot(!(MDL_ABLATE & 8) && act && op == 1 && carry == 0);
        uint64_t tookany = 0;   // some package was picked up (the carried set changed)
        if (pickers) {
            // per robot: the lowest-index waiting package at its cell
            int sw[NCH];
            uint64_t took[NCH];
#pragma unroll
            for (int c = 0; c < NCH; c++) {
                sw[c] = (ps[c] & PS_STATUS) == ST_WAITING ? pk_start(pk[c]) : -2;  // unused lanes are ST_NONE
                took[c] = 0;
            }
            int cnew = carry;
            bool by_bits = false;
            if constexpr (AU == 16) {
                const MapDesc& md = p.maps[mi];
                if (md.H <= 64 && md.W <= 64) {   // cells (r, c) -> bit r * 64 + c of a 4096-bit map
                    by_bits = true;
                    uint32_t* pb = (uint32_t*)(smem + (size_t)wave * lds_stride);
                    auto bit_of = [](int cl) { return ((cl & 63) << 6) | ((cl >> 8) & 63); };
                    wave_sync();
                    reinterpret_cast<uint2*>(pb)[lane] = uint2{0u, 0u};
                    wave_sync();
                    if ((pickers >> lane) & 1ull) {
                        const int ix = bit_of(cell);
                        atomicOr(&pb[ix >> 5], 1u << (ix & 31));
                    }
                    wave_sync();
                    uint64_t left = pickers;
#pragma unroll
                    for (int c = 0; c < NCH; c++) {
                        const int ix = bit_of(sw[c]);   // sw < 0: any in-range bit, masked below
                        const uint64_t mt = ballot(sw[c] >= 0 && ((pb[ix >> 5] >> (ix & 31)) & 1u));
                        // waiting packages under a picker, in index order: the first one at a
                        // picker's cell is its lowest-index package (robot cells are distinct)
                        for (uint64_t m = mt; m && left; m &= m - 1) {
                            const int j = ffs64(m);
                            const uint64_t who = ballot(cell == rdl(sw[c], j)) & left;
                            if (who) {
                                const int i = ffs64(who);
                                left &= ~(1ull << i);
                                took[c] |= 1ull << j;
                                cnew = lane == i ? c * WAVE + j + 1 : cnew;
                            }
                        }
                    }
                }
            }
            if (!by_bits) {
                for (; pickers; pickers &= pickers - 1) {
                    const int i = ffs64(pickers);
                    const int ci = rdl(cell, i);
                    int fnd = -1;
#pragma unroll
                    for (int c = 0; c < NCH; c++) {
                        const uint64_t b = ballot(sw[c] == ci);
                        took[c] |= fnd < 0 ? (b & (0ull - b)) : 0ull;
                        fnd = (fnd < 0 && b != 0ull) ? c * WAVE + ffs64(b) : fnd;
                    }
                    cnew = lane == i ? fnd + 1 : cnew;  // not found: stays 0
                }
            }
            carry = cnew;
#pragma unroll
            for (int c = 0; c < NCH; c++) {
                ps[c] = vbit(took[c], lane) ? ((ps[c] & ~PS_STATUS) | ST_IN_TRANSIT) : ps[c];
                tookany |= took[c];
            }
        }
        // drops: a robot with op 2 carrying a package (its pre-step one: it did not
        // pick) and standing on that package's target delivers it
        const bool drop = !(MDL_ABLATE & 8) && act && op == 2 && carry != 0 && pk_target(g_pk) == cell;
        const uint64_t dmask = ballot(drop), omask = ballot(drop && t0 <= pk_dl(g_pk));
        carry = drop ? 0 : carry;
        for (uint64_t m = dmask; m; m &= m - 1) {
            const int j = rdl(pj, ffs64(m));
#pragma unroll
            for (int c = 0; c < NCH; c++)
                ps[c] = (c * WAVE + lane == j) ? ((ps[c] & ~PS_STATUS) | ST_DELIVERED) : ps[c];
        }
        // reward: fp64 fold in the reference's order (move costs, then deliveries)
        double rr;
        if constexpr (AU > 0 && AU <= 8) {
            rr = p.cost_sum[n_cost];  // n_cost <= A <= 8: the same fold, tabulated on the host
        } else {
            rr = p.cost_fold[n_cost];  // n_cost <= A <= 64: likewise (one scalar load, no fp64 chain)
        }
        for (uint64_t m = dmask; m; m &= m - 1) {
            const int i = ffs64(m);
            rr += ((omask >> i) & 1ull) ? p.delivery_reward : p.delay_reward;
        }
        // which of env.py's reward terms fired (the reference's r stays the int 0 until one
        // does, env.py:181,256,288,291): move cost, on-time delivery, late delivery
        rfl = (n_cost ? RT_MOVE : 0u) | (omask ? RT_ONTIME : 0u) | ((dmask & ~omask) ? RT_LATE : 0u);
        const int t1 = t0 + 1;
        const double total = tot_cur + rr;

        STAMP(5);
        // ---- terminate (env.py:308-316) + spawn (get_state env.py:133-137) ----
        int ndel = 0;
        uint64_t spawned = 0;
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            const int j = c * WAVE + lane;
            ndel += popc64(ballot((ps[c] & PS_STATUS) == ST_DELIVERED));
            const bool sp = j < P && pk_st(pk[c]) == t1;
            spawned |= ballot(sp);
            if (sp) ps[c] = (ps[c] & ~PS_STATUS) | ST_WAITING;
        }
        const bool done = (t1 == T) || (ndel == P);

        STAMP(6);
        // ---- shaped reward with the pre-step tracker (MAPPO/helper.py:257-369) ----
        // Agents on lanes.  Each agent that needs the nearest waiting package of
        // tracker_prev (st <= t_prev) gets it from one DPP minimum over the package
        // lanes of (distance << 11 | order key); idle-nearby is that distance <= 3.
        // The reference's if-chains become selects: adding 0.0f is exact here
        // (s starts at +0 and never becomes -0).
        float s_lane = 0.0f;
        if (!(MDL_ABLATE & 1)) {
            // tracker_prev entry of each agent's previously carried id (gathered above)
            const uint32_t pf = g_pf;
            const uint64_t pdat = g_td;
            // Lane predicates as vector masks (lmask): combined on the vector ALU.
            const uint32_t Mact = lmask(act), Mpc0 = lmask(pcarry == 0), Mc0 = lmask(carry == 0);
            const uint32_t Mpres =
                Mact & ~Mpc0 & lmask(pcarry <= P) &
                (STALE ? lmask((pf & PS_PRESENT) != 0)
                       : lmask((pf & PS_STATUS) == ST_WAITING) | lmask((pf & PS_STATUS) == ST_IN_TRANSIT));
            const uint32_t Mmov = lmask(pcell != cell), MS = lmask(mv == MV_S);
            const uint32_t Mop1 = lmask(op == 1), Mop2 = lmask(op == 2);
            const bool need_near = (Mact & Mmov & (Mpc0 | ~Mpres)) != 0u;
            const bool need_idle = (Mact & ~Mmov & MS & Mpc0) != 0u;
            const bool need_can = (Mact & Mop1 & Mpc0 & Mc0) != 0u;
            STAMP(7);
            // per-agent answers: bit masks in SGPRs, the nearest start cell written
            // into the agent's lane
            uint32_t Midle = 0, Mcan = 0;
            int best_cell = -1;
            if (anyw && !(MDL_ABLATE & 32)) {
                // key = distance << 21 | order key << 10 | slot (distance <= 508,
                // order keys < 0x800, slots < 1024): the minimum names the nearest
                // package with the reference's tie-break and carries its slot
                uint64_t q = ballot(need_near || need_idle);
                if constexpr (AU > 8) {
                    // Every agent at once: the waiting candidates of tracker_prev are packed
                    // into the wave's LDS slice (the reset scratch, unused until a reset below)
                    // as {start cell, key bits}; lane l scans every (64/AP)-th candidate for
                    // agent l % AP, and a butterfly over the lane groups leaves agent a's
                    // minimum on lane a.  A few VALU ops per candidate and group instead of one
                    // wave reduction per agent and package chunk.
                    static_assert(AU <= 16, "agents of one lane group");
                    constexpr int AP = AU <= 8 ? 8 : 16, LG = AU <= 8 ? 3 : 4;
                    uint64_t* cand = (uint64_t*)(smem + (size_t)wave * lds_stride);
                    constexpr int GS = 64 / AP;   // lane groups = candidates per scan step
                    int nw = 0;
#pragma unroll
                    for (int c = 0; c < NCH; c++) {
                        const int idx = nw + popc64(wvm[c] & lanemask_lt());
                        if (wv[c]) cand[idx] = (uint64_t)(uint32_t)stc[c] | ((uint64_t)klo[c] << 32);
                        nw += popc64(wvm[c]);
                    }
                    // sentinels up to a multiple of 2 GS (key bits ~0: never below a real key;
                    // cell ~0: no map cell), so the scan needs no bound per candidate and
                    // takes two candidates per lane and step (two LDS reads in flight)
                    const int nwg = (nw + 2 * GS - 1) & ~(2 * GS - 1);
                    if (lane < nwg - nw) cand[nw + lane] = ~0ull;
                    wave_sync();
                    const int grp = lane >> LG;
                    const int pa = __builtin_amdgcn_ds_bpermute((lane & (AP - 1)) << 2, pcell);
                    // the same scan answers "a waiting package starts at my (new) cell" for
                    // the can-pick-up test: one compare per candidate into a lane mask (the
                    // OR over candidates on the scalar unit)
                    const int ca = __builtin_amdgcn_ds_bpermute((lane & (AP - 1)) << 2, cell);
                    const uint64_t* cp = cand + grp;
                    uint32_t kmin = 0xffffffffu;
                    uint64_t hm = 0;
                    for (int i0 = 0; i0 < nwg; i0 += 2 * GS) {   // wave-uniform trip count
                        const uint64_t ce = cp[i0], cf = cp[i0 + GS];
                        const uint32_t ke = ((uint32_t)manhattan_sad(pa, (int)(uint32_t)ce) << 21) | (uint32_t)(ce >> 32);
                        const uint32_t kf = ((uint32_t)manhattan_sad(pa, (int)(uint32_t)cf) << 21) | (uint32_t)(cf >> 32);
                        kmin = min(kmin, min(ke, kf));
                        hm |= ballot((int)(uint32_t)ce == ca) | ballot((int)(uint32_t)cf == ca);
                    }
                    uint32_t o;
                    if constexpr (AP == 8) {
                        o = xor_lane<8>(kmin);
                        kmin = o < kmin ? o : kmin;
                    }
                    o = xor_lane<16>(kmin);
                    kmin = o < kmin ? o : kmin;
                    o = xor_lane<32>(kmin);
                    kmin = o < kmin ? o : kmin;
                    // agent a's hit: bit a of the lane groups' masks ORed (AP = 16 here)
                    static_assert(AP == 16, "the hit fold assumes four groups of 16 lanes");
                    const uint64_t h16 = (hm | (hm >> 16) | (hm >> 32) | (hm >> 48)) & 0xffffull;
                    // Mcan matters only on lanes with op 1 and no package before or after
                    // (Mwpick below), i.e. exactly where the per-agent loop would set it
                    Mcan = sel64(h16, 0u, ~0u);
                    // the nearest candidate's start cell, from its slot's lane
                    const int js = (int)(kmin & 1023u);
                    int bc = __builtin_amdgcn_ds_bpermute((js & 63) << 2, stc[0]);
#pragma unroll
                    for (int c = 1; c < NCH; c++) {
                        const int v = __builtin_amdgcn_ds_bpermute((js & 63) << 2, stc[c]);
                        bc = (js >> 6) == c ? v : bc;
                    }
                    const bool found = act && kmin != 0xffffffffu;
                    Midle = lmask(found && (kmin >> 21) <= 3u);
                    best_cell = found ? bc : -1;
                    q = 0;
                }
                if constexpr (NCH == 1) {
                    // two agents per pass: their minima interleave
                    for (; q & (q - 1); q &= q - 1, q &= q - 1) {
                        const int a = ffs64(q), b = ffs64(q & (q - 1));
                        const int pa = rdl(pcell, a), pb = rdl(pcell, b);
                        uint32_t ka, kb;
                        wave_min_u32x2(((uint32_t)manhattan_sad(pa, stc[0]) << 21) | klo[0],
                                       ((uint32_t)manhattan_sad(pb, stc[0]) << 21) | klo[0], ka, kb);
                        const int ca = rdl(stc[0], (int)(ka & 63u)), cb = rdl(stc[0], (int)(kb & 63u));
                        const bool sa = lane == a, sb = lane == b;
                        Midle = ((sa && (ka >> 21) <= 3u) || (sb && (kb >> 21) <= 3u)) ? ~0u : Midle;
                        best_cell = sa ? ca : sb ? cb : best_cell;
                    }
                }
                for (; q; q &= q - 1) {
                    const int a = ffs64(q);
                    const int pa = rdl(pcell, a);
                    uint32_t kmin = 0xffffffffu;
#pragma unroll
                    for (int c = 0; c < NCH; c++) {
                        const uint32_t key = ((uint32_t)manhattan_sad(pa, stc[c]) << 21) | klo[c];
                        const uint32_t m = wave_min_u32(key);
                        kmin = m < kmin ? m : kmin;
                    }
                    const int js = (int)(kmin & 1023u);
                    int bc = rdl(stc[0], js & 63);
#pragma unroll
                    for (int c = 1; c < NCH; c++) {
                        const int v = rdl(stc[c], js & 63);
                        bc = (js >> 6) == c ? v : bc;
                    }
                    const bool sel = lane == a;
                    Midle = (sel && (kmin >> 21) <= 3u) ? ~0u : Midle;
                    best_cell = sel ? bc : best_cell;
                }
                for (uint64_t q = AU > 8 ? 0ull : ballot(need_can); q; q &= q - 1) {
                    const int a = ffs64(q);
                    const int ca = rdl(cell, a);
                    uint64_t h = 0;
#pragma unroll
                    for (int c = 0; c < NCH; c++) h |= ballot(stc[c] == ca) & wvm[c];
                    Mcan = (lane == a && h != 0) ? ~0u : Mcan;
                }
            }
            STAMP(8);
            // the constants, pinned in SGPRs
            float cs[9];
#pragma unroll
            for (int k = 0; k < 9; k++) {
                cs[k] = p.shaping[k];
                pin(cs[k]);
            }
            // The reference's if-chains, term by term.  Each term is a masked constant
            // (+0.0f when no branch fires; the alternatives within a term are disjoint).
            const int ptg = pk_target(pdat);
            const uint32_t Mtg = lmask(cell == ptg);
            // 1. pickup / delivery
            const uint32_t Mpick = Mpc0 & ~Mc0;
            const uint32_t Mdeliv = ~Mpc0 & Mc0 & Mpres & Mtg;
            const float t1v = fmask(Mpick, cs[SH_PICK]) +
                              fmask(Mdeliv, fpick(lmask(t1 <= pk_dl(pdat)), cs[SH_ONTIME], cs[SH_LATE]));
            // 2. wasted operations
            const uint32_t Mwpick = Mop1 & (~Mpc0 | (Mc0 & ~Mcan));
            const uint32_t Mwdrop = Mop2 & (Mpc0 | (~Mc0 & Mpres & ~Mtg));
            const float t2v = fmask(Mwpick, cs[SH_WPICK]) + fmask(Mwdrop, cs[SH_WDROP]);
            // 3. movement
            const float t3v = fmask(~MS & ~Mmov, cs[SH_STUCK]);
            const int tgt = ipick(~Mpc0 & Mpres, ptg, best_cell);
            const int db = manhattan_sad(pcell, tgt), da = manhattan_sad(cell, tgt);  // garbage for tgt < 0: masked
            const uint32_t Mt = lmask(tgt >= 0) & Mmov;
            const float t4v = fmask(Mt & lmask(da < db), cs[SH_CLOSER]) + fmask(Mt & lmask(da > db), cs[SH_AWAY]);
            // 4. idle next to an available package
            const float t5v = fmask(~Mmov & MS & Mpc0 & Midle, cs[SH_IDLE]);
            // (0.0f + t1v == t1v: t1v is a sum of two terms of which one is +0, so never -0)
            float s = t1v;
            s = s + t2v;
            s = s + t3v;
            s = s + t4v;
            s = s + t5v;
            s_lane = fmask(Mact, s);
        }
        const float shaped = (float)rr + np_sum_step<AU>(s_lane, A);

        STAMP(9);
        // ---- tracker update with the new state; a done env that resets here skips
        // it and updates with the reset state instead (MAPPO/trainer.py:230-259) ----
        const bool do_rst = done && auto_reset;
        // After an update, the present entries in transit are exactly the carried ones; with
        // no pick-up, no drop and no spawn at t1 the update is a no-op, so it is skipped.
        if (STALE && !do_rst && !(MDL_ABLATE & 2) && (tookany | dmask | spawned))
        {
            if constexpr (AU == 16) {
                // sixteen robots: the carried ids as a per-lane bitmask in the wave's LDS slice
                // (free again: the shaping's candidates are consumed) -- one atomic OR per robot
                // instead of 16 readlanes and 16 compares per package chunk
                uint32_t* cm = (uint32_t*)(smem + (size_t)wave * lds_stride);
                cm[lane] = 0u;
                wave_sync();
                if (act && carry != 0) atomicOr(&cm[(carry - 1) & 63], 1u << ((carry - 1) >> 6));
                wave_sync();
                tracker_update_bits<NCH>(ps, td, dirty, pk, P, t1, cm[lane]);
            } else {
                tracker_update_regs<NCH, AU>(ps, td, dirty, pk, P, A, carry, t1);
            }
        }

        // ---- reset on done (MAPPO/trainer.py:230-235) ----
        int t_out = t1;
        double total_out = total;
        if (do_rst) {
            ResetLds L = reset_carve(smem + (size_t)wave * lds_stride, P);
            const MapDesc md = p.maps[mi];
            const int nc = do_reset(p, e, md, L, false);
            if (act) {
                cell = nc;
                carry = 0;
                vmask = p.movevalid_cell[(uint32_t)(mvoff + cell)];
            }
            if (STALE) survivors_at_reset<NCH>(ps, tq, P);
#pragma unroll
            for (int c = 0; c < NCH; c++) {
                const int j = c * WAVE + lane;
                pk[c] = j < P ? L.pk[j] : 0;
                ps[c] = (j < P ? L.pst[j] : 0u) | (STALE ? (ps[c] & ~PS_STATUS) : 0u);
            }
            if (STALE) tracker_update_regs<NCH, AU>(ps, td, dirty, pk, P, A, 0, 0);
            t_out = 0;
            total_out = 0.0;
            any_rst = true;
        }
        t_cur = t_out;
        tot_cur = total_out;
        // Settle the move-validity load here, before the first store: vmcnt counts
        // stores too, so waiting for it after the (lane-0, branchy) output stores
        // would wait for those stores' round trip.  (A robot that moved and then
        // reset takes its new cell's bits from the reset above.)
        vmask = (((moved >> lane) & 1ull) && !do_rst) ? pvm : vmask;
        asm volatile("" : "+v"(vmask));
        // The store pointers of the outputs and of the common write-back, fetched here in
        // one scalar batch (one scalar-cache round trip instead of one per pointer; they
        // are not held in SGPRs across the step itself).  Rare stores (episode ends,
        // resets) reload theirs.
        {
            // an opaque copy of the segment pointer: the loads below cannot be hoisted
            // above this point (where their registers would have to live across the step)
            KargPtr ka = (KargPtr)((__attribute__((address_space(4))) const char*)
                                       __builtin_amdgcn_kernarg_segment_ptr() + offsetof(StepKarg, args));
            asm volatile("" : "+s"(ka));
            rop = (GLOBAL double*)ka->r_out;
            shp = (GLOBAL float*)ka->sh_out;
            dnp = (GLOBAL uint8_t*)ka->done_out;
            robw = (GLOBAL uint32_t*)ka->p.rob;
            pstw = (GLOBAL uint16_t*)ka->p.pstate;
            trkw = (GLOBAL uint64_t*)ka->p.trk;
            esw = (GLOBAL u32x4*)ka->p.es;
        }
        pin(rop); pin(shp); pin(dnp); pin(robw); pin(pstw); pin(trkw); pin(esw);
        if (lane == 0) {
            if (done) {
                p.ep_total[e] = total;
                p.ep_len[e] = t1;
            }
            const size_t o = (size_t)k * n_ + w;
            if (rop) rop[o] = rr;
            if (shp) shp[o] = shaped;
            if (dnp) dnp[o] = done ? 1 : 0;
        }
    }  // steps

    STAMP(10);
    // ---- write back only what changed ----
    if (act) robw[(size_t)e * A + lane] = rob_pack(cell, carry, vmask);
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        const int j = c * WAVE + lane;
        if (j < P) {
            const size_t eb = (size_t)e * P;   // uniform row base; the lane offset stays 32-bit
            if (ps[c] != ps_in[c]) (pstw + eb)[(uint32_t)j] = (uint16_t)ps[c];
            if (any_rst) ((GLOBAL uint64_t*)p.pkg + eb)[(uint32_t)j] = pk[c];
            if (STALE && dirty[c]) (trkw + eb)[(uint32_t)j] = td[c];
        }
    }
    if (lane == 0)
        esw[e] = u32x4{(uint32_t)t_cur, rfl, (uint32_t)__double2loint(tot_cur), (uint32_t)__double2hiint(tot_cur)};
    STAMP(11);
#ifdef MDL_STAMPS
    if (lane == 0)
        for (int k = 0; k < 16; k++) g_stamps[(size_t)w * 16 + k] = stamp_[k];
#endif
    if constexpr (OBS)   // full batch only (no env_ids): output row w = env e
        obs_small_emit<STALE>(p, w, mi, act ? rob_pack(cell, carry, vmask) : 0u, pk[0], ps[0], STALE ? td[0] : 0ull,
                              t_cur, oa.amap, oa.avec, oa.cmap, oa.cvec, smem + (size_t)wave * lds_stride);
    if constexpr (MAIL) {   // row w of the call: k_mail_export's layout, from the registers
        const MailRows& m = ma->m;
        if (act) {
            int32_t* o = m.robots + ((size_t)w * A + lane) * 3;
            o[0] = cell_r(cell);
            o[1] = cell_c(cell);
            o[2] = carry;
        }
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            const int j = c * WAVE + lane;
            if (j < P) {
                int4* o = (int4*)(m.pkgs + ((size_t)w * P + j) * 8);
                const uint64_t d = pk[c];
                o[0] = int4{cell_r(pk_start(d)), cell_c(pk_start(d)), cell_r(pk_target(d)), cell_c(pk_target(d))};
                o[1] = int4{pk_st(d), pk_dl(d), j + 1, (int)(ps[c] & PS_STATUS)};
            }
        }
        if (lane == 0) {
            m.t[w] = t_cur;
            m.total[w] = tot_cur;
            m.rterms[w] = (int32_t)rfl;
        }
        publish_tail(ma->pb);   // pb.expect = n: the waves of rows [0, n) count themselves
    }
}

template <bool STALE, int NCH, bool FUSED, int AU>
__global__ __launch_bounds__(MDL_STEP_LB) MDL_STEP_ATTR(NCH, FUSED) void k_step(const uint32_t* __restrict__ rob_pre,
                                                      const uint64_t* __restrict__ pkg_pre,
                                                      const uint16_t* __restrict__ pst_pre,
                                                      const u32x4* __restrict__ es_pre,
                                                      const uint64_t* __restrict__ trk_pre,
                                                      const uint8_t* __restrict__ act_pre, uint32_t ap,
                                                      uint32_t nw, StepArgs args) {
    step_body<STALE, NCH, FUSED, AU, false>(rob_pre, pkg_pre, pst_pre, es_pre, trk_pre, act_pre, ap, nw, args,
                                            ObsArgs{});
}

// mdl_mail_step: k_step + the mailbox rows + the completion word in one launch; the action
// bytes come from the kernel arguments when they fit (ma.pb / codes: MailArgs)
template <bool STALE, int NCH, int AU>
__global__ __launch_bounds__(MDL_STEP_LB) void k_step_mail(const uint32_t* __restrict__ rob_pre,
                                                           const uint64_t* __restrict__ pkg_pre,
                                                           const uint16_t* __restrict__ pst_pre,
                                                           const u32x4* __restrict__ es_pre,
                                                           const uint64_t* __restrict__ trk_pre,
                                                           const uint8_t* __restrict__ act_pre, uint32_t ap,
                                                           uint32_t nw, StepArgs args, MailArgs ma, int inl) {
    step_body<STALE, NCH, false, AU, false, true>(rob_pre, pkg_pre, pst_pre, es_pre, trk_pre,
                                                  inl ? ma.codes : act_pre, ap, nw, args, ObsArgs{}, &ma);
}

// mdl_step_floor: the launch floor of k_step -- the same kernel-argument layout (and so the
// same preloaded SGPRs and kernarg segment size), workgroup size, LDS request and grid, and
// no work.  bench.py replays it the way it replays the step (one graph node per step) and
// reports the difference as the step's own cost above the dispatch floor.
__global__ __launch_bounds__(MDL_STEP_LB) void k_step_floor(const uint32_t* __restrict__ rob_pre,
                                                            const uint64_t* __restrict__ pkg_pre,
                                                            const uint16_t* __restrict__ pst_pre,
                                                            const u32x4* __restrict__ es_pre,
                                                            const uint64_t* __restrict__ trk_pre,
                                                            const uint8_t* __restrict__ act_pre, uint32_t ap,
                                                            uint32_t nw, StepArgs args) {
    (void)rob_pre, (void)pkg_pre, (void)pst_pre, (void)es_pre, (void)trk_pre, (void)act_pre, (void)ap, (void)nw;
    (void)args;
}

// mdl_step_obs: k_step + k_obs_small in one launch (full batch, NCH = 1, A <= 8)
template <bool STALE, int AU>
__global__ __launch_bounds__(256) MDL_STEP_ATTR(1, false) void k_step_obs(const uint32_t* __restrict__ rob_pre,
                                                  const uint64_t* __restrict__ pkg_pre,
                                                  const uint16_t* __restrict__ pst_pre,
                                                  const u32x4* __restrict__ es_pre,
                                                  const uint64_t* __restrict__ trk_pre,
                                                  const uint8_t* __restrict__ act_pre, uint32_t ap, uint32_t nw,
                                                  StepArgs args, ObsArgs oa) {
    step_body<STALE, 1, false, AU, true>(rob_pre, pkg_pre, pst_pre, es_pre, trk_pre, act_pre, ap, nw, args, oa);
}

#include "mdl_step_rows.hpp"
#include "mdl_step_halves.hpp"

// ------------------------------------------------------------- observations
// Tracker slots staged in LDS for the feature builders (random access by id).
struct ObsLdsPre {
    uint64_t* pk;
    uint64_t* td;
    uint32_t* tq;
    uint8_t* ps;
};

__host__ __device__ inline size_t obs_pre_bytes(int P) {
    return align16(8 * (size_t)P) * 2 + align16(4 * (size_t)P) + align16((size_t)P);
}

__device__ inline ObsLdsPre obs_pre_carve(unsigned char* base, int P) {
    ObsLdsPre S;
    size_t o = 0;
    S.pk = (uint64_t*)(base + o); o += align16(8 * (size_t)P);
    S.td = (uint64_t*)(base + o); o += align16(8 * (size_t)P);
    S.tq = (uint32_t*)(base + o); o += align16(4 * (size_t)P);
    S.ps = base + o;
    return S;
}

template <bool STALE>
__global__ __launch_bounds__(256) void k_obs(DevParams p, int env_begin, int n, float* __restrict__ amap,
                                             float* __restrict__ avec, float* __restrict__ cmap,
                                             float* __restrict__ cvec, int wpb, int lds_stride) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = wave_id();
    const int lane = lane_id();
    const int w = xcd_block() * wpb + wave;
    if (wave >= wpb || w >= n) return;
    const int e = env_begin + w;
    const int A = p.A, P = p.P;
    unsigned char* base = smem + (size_t)wave * lds_stride;
    ObsLdsPre S = obs_pre_carve(base, P);
    const MapDesc md = p.maps[p.env_map ? p.env_map[e] : 0];
    FeatCtx c;
    c.A = A; c.NS = P; c.H = md.H; c.W = md.W; c.HW = md.H * md.W; c.NW = (c.HW + 31) / 32;
    c.t = p.es[e].t; c.T = p.obsT;
    c.MO = p.MO; c.MP = p.MP; c.MR = p.MR; c.MPs = p.MPs;
    c.MPc = p.MP < P ? p.MP : P;
    c.MPsc = p.MPs < P ? p.MPs : P;
    c.gridbits = p.gridbits + md.bits_off;
    c.rank = p.rank + md.rank_off;
    c.inv_hw = md.inv_hw;
    FeatDims fd{A, P, c.HW, c.MPc, c.MPsc, stage_floats(A, A, c.MO, c.MPc, c.MR, c.MPsc)};
    FeatLds L = feat_carve(base + obs_pre_bytes(P), fd);
    // plane words: reserved for the largest map; HW % 4 == 0 maps use them
    uint32_t* planes = (p.obs_plane_words > 0 && (c.HW & 3) == 0)
                           ? (uint32_t*)(base + obs_pre_bytes(P) + feat_lds_bytes(fd))
                           : nullptr;

    const bool act = lane < A;
    const uint32_t rv = act ? p.rob[(size_t)e * A + lane] : 0u;
    const int cell = rob_cell(rv);
    const int carry = rob_carry(rv);
    for (int j = lane; j < P; j += WAVE) {
        const size_t g = (size_t)e * P + j;
        const uint64_t d = p.pkg[g];
        const uint32_t f = p.pstate[g];
        S.pk[j] = d;
        S.ps[j] = (uint8_t)(f & PS_FLAGS);
        if (STALE) {
            const bool sv = (f & PS_SURVIVOR) != 0;
            S.td[j] = sv ? p.trk[g] : d;
            S.tq[j] = sv ? f >> PS_RANK_SHIFT : ORD_EPISODE + (uint32_t)j;
        }
    }
    wave_sync();
    auto run = [&](const auto& trk) {
        feat_prepare(trk, c, L, cell, carry);
        const size_t le = (size_t)w;
        float* am = amap ? amap + le * (size_t)A * 6 * c.HW : nullptr;
        float* cm = cmap ? cmap + le * 4 * (size_t)c.HW : nullptr;
        if (planes && (((uintptr_t)am | (uintptr_t)cm) & 15) == 0 && (am || cm)) {
            feat_build_planes(c, L, planes);
            if (am) emit_planes(planes, c.NW, 6 * A, c.HW, am);
            if (cm) emit_planes(planes + 6 * A * c.NW, c.NW, 4, c.HW, cm);
        } else if ((c.HW & 3) == 0 && (((uintptr_t)am | (uintptr_t)cm) & 15) == 0 && (am || cm)) {
            emit_maps_bitrows(L, c.NW, c.HW, A, am, cm);
        } else {
            if (am) emit_actor_maps(c, L, 0, A, true, am);
            if (cm) emit_critic_map(c, L, cm);
        }
        if (avec) {
            if (p.key32_dsh > 0 && P <= WAVE && A <= 8) {
                for (int a = 0; a < A; a++) feat_sort_others(c, L, a, cell);
                feat_sort_pkgs_fast<decltype(trk), 8>(trk, c, L, p.key32_dsh);
            } else {
                for (int a = 0; a < A; a++) feat_sort_agent(trk, c, L, a, cell);
            }
            const int Dv = 6 + 5 * c.MO + 5 * c.MP + 1;
            emit_actor_vecs(trk, c, L, 0, A, true, avec + le * (size_t)A * Dv);
        }
        if (cvec) {
            const int Dg = 6 * c.MR + 7 * c.MPs + 1;
            emit_critic_vec(trk, c, L, cvec + le * (size_t)Dg);
        }
    };
    if (STALE) {
        TrkStale trk{S.ps, S.td, S.tq, P};
        run(trk);
    } else {
        TrkFresh trk{S.pk, S.ps, P};
        run(trk);
    }
}

// ------------------------------------------------------ dict views (helpers)
// record: [t, A, n_slots, map] + A*(r, c, carry) + n_slots*(id, status, sr, sc, tr, tc, st, dl)
struct ViewLdsPre {
    int32_t* ids;
    uint64_t* pk;
    uint8_t* flag;
};

__host__ __device__ inline size_t view_pre_bytes(int NS) {
    const int n = NS > 0 ? NS : 1;
    return align16(4 * (size_t)n) + align16(8 * (size_t)n) + align16((size_t)n);
}

__device__ inline ViewLdsPre view_carve(unsigned char* base, int NSmax) {
    ViewLdsPre V;
    const int nsm = NSmax > 0 ? NSmax : 1;
    size_t o = 0;
    V.ids = (int32_t*)(base + o); o += align16(4 * (size_t)nsm);
    V.pk = (uint64_t*)(base + o); o += align16(8 * (size_t)nsm);
    V.flag = base + o;
    return V;
}

// The rows of a view record whose header (A, ns) the caller has read (so the caller can put its
// own independent loads beside these).
__device__ inline TrkView load_view_rows(const int32_t* rec, int A, int ns, ViewLdsPre& V, int& cell, int& carry) {
    const int lane = lane_id();
    const int32_t* rb = rec + 4;
    cell = 0;
    carry = 0;
    if (lane < A) {
        cell = rb[3 * lane] | (rb[3 * lane + 1] << 8);
        carry = rb[3 * lane + 2];
    }
    const int32_t* sl = rb + 3 * A;
    for (int j = lane; j < ns; j += WAVE) {
        const int32_t* s = sl + 8 * j;
        V.ids[j] = s[0];
        V.flag[j] = (uint8_t)(1 | (s[1] == ST_IN_TRANSIT ? 2 : 0));
        V.pk[j] = pk_make(s[2] | (s[3] << 8), s[4] | (s[5] << 8), s[6], s[7]);
    }
    wave_sync();
    return TrkView{V.ids, V.flag, V.pk, ns};
}

__device__ inline TrkView load_view(const int32_t* rec, ViewLdsPre& V, int& t, int& A, int& map, int& cell,
                                    int& carry) {
    const int lane = lane_id();
    t = rec[0];
    A = rec[1];
    const int ns = rec[2];
    map = rec[3];
    const int32_t* rb = rec + 4;
    cell = 0;
    carry = 0;
    if (lane < A) {
        cell = rb[3 * lane] | (rb[3 * lane + 1] << 8);
        carry = rb[3 * lane + 2];
    }
    const int32_t* sl = rb + 3 * A;
    for (int j = lane; j < ns; j += WAVE) {
        const int32_t* s = sl + 8 * j;
        V.ids[j] = s[0];
        V.flag[j] = (uint8_t)(1 | (s[1] == ST_IN_TRANSIT ? 2 : 0));
        V.pk[j] = pk_make(s[2] | (s[3] << 8), s[4] | (s[5] << 8), s[6], s[7]);
    }
    wave_sync();
    return TrkView{V.ids, V.flag, V.pk, ns};
}

// view record `rec`, agent index `a`, outputs row w
__device__ __forceinline__ void views_features_one(const DevParams& p, const int32_t* rec, int w, int a, int T,
                                                   int MO, int MP, int MR, int MPs, int MPc, int MPsc, int NSmax,
                                                   float* __restrict__ obs, float* __restrict__ vec,
                                                   float* __restrict__ gmap, float* __restrict__ gvec,
                                                   unsigned char* base, int HW) {
    ViewLdsPre V = view_carve(base, NSmax);
    int t, A, map, cell, carry;
    const TrkView trk = load_view(rec, V, t, A, map, cell, carry);
    const MapDesc md = p.maps[map];
    FeatCtx c;
    c.A = A; c.NS = trk.n; c.H = md.H; c.W = md.W; c.HW = md.H * md.W; c.NW = (c.HW + 31) / 32; c.t = t; c.T = T;
    c.MO = MO; c.MP = MP; c.MR = MR; c.MPs = MPs; c.MPc = MPc; c.MPsc = MPsc;
    c.gridbits = p.gridbits + md.bits_off;
    c.rank = p.rank + md.rank_off;
    c.inv_hw = md.inv_hw;
    FeatDims fd{64, NSmax, HW, MPc, MPsc, stage_floats(64, 1, MO, MPc, MR, MPsc)};
    FeatLds L = feat_carve(base + view_pre_bytes(NSmax), fd);
    feat_prepare(trk, c, L, cell, carry);
    const bool valid = a >= 0 && a < A;
    const int aa = valid ? a : 0;
    if (obs) emit_actor_maps(c, L, aa, 1, valid, obs + (size_t)w * 6 * c.HW);
    if (gmap) emit_critic_map(c, L, gmap + (size_t)w * 4 * c.HW);
    if (vec) {
        if (valid) feat_sort_agent(trk, c, L, aa, cell);
        emit_actor_vecs(trk, c, L, aa, 1, valid, vec + (size_t)w * (6 + 5 * MO + 5 * MP + 1));
    }
    if (gvec) emit_critic_vec(trk, c, L, gvec + (size_t)w * (6 * MR + 7 * MPs + 1));
}

__global__ __launch_bounds__(256) void k_views_features(DevParams p, const int32_t* __restrict__ views,
                                                        const int64_t* __restrict__ offs, int n,
                                                        const int32_t* __restrict__ agent_idx, int T, int MO, int MP,
                                                        int MR, int MPs, int MPc, int MPsc, int NSmax,
                                                        float* __restrict__ obs, float* __restrict__ vec,
                                                        float* __restrict__ gmap, float* __restrict__ gvec, int wpb,
                                                        int lds_stride, int HW, Publish pb) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = wave_id();
    const int w = blockIdx.x * wpb + wave;
    if (wave < wpb && w < n) {
        // every per-view input address / scalar first, in one round trip (the helpers pass host-mapped
        // memory, where each dependent load is a PCIe round trip)
        const int64_t off = offs[w];
        const int a = agent_idx ? agent_idx[w] : 0;
        views_features_one(p, views + off, w, a, T, MO, MP, MR, MPs, MPc, MPsc, NSmax, obs, vec, gmap, gvec,
                           smem + (size_t)wave * lds_stride, HW);
    }
    if (pb.seq) publish_tail(pb);
}

// One view whose record travels in the kernel arguments (mdl_host_view_features): the launch
// copies it into the kernarg segment, so the wave reads it from there instead of making
// dependent round trips to host memory.  One wave, one block.
template <int CAP>
__global__ __launch_bounds__(64) void k_view_features_inl(DevParams p, int a, int T, int MO, int MP, int MR, int MPs,
                                                          int MPc, int MPsc, int NSmax, float* __restrict__ obs,
                                                          float* __restrict__ vec, float* __restrict__ gmap,
                                                          float* __restrict__ gvec, int HW, Publish pb,
                                                          ViewInline<CAP> rec) {
    extern __shared__ __align__(16) unsigned char smem[];
    views_features_one(p, rec.w, 0, a, T, MO, MP, MR, MPs, MPc, MPsc, NSmax, obs, vec, gmap, gvec, smem, HW);
    if (pb.seq) publish_tail(pb);
}

// one transition: prev view record, current record [t, A] + A x 3, action codes, global reward
__device__ __forceinline__ float views_shaped_one(const int32_t* rec, const int32_t* cr, const uint8_t* acts,
                                                  double gw, const ShapingConsts& C, unsigned char* base,
                                                  int NSmax) {
    const int lane = lane_id();
    ViewLdsPre V = view_carve(base, NSmax);
    const int t_prev = rec[0], A = rec[1], ns = rec[2], t_cur = cr[0];   // the headers: one round trip
    const bool act = lane < A;
    int ccell = 0, ccarry = 0, mv = MV_S, op = 0;
    if (act) {   // the current robots and actions, issued beside the view's rows
        ccell = cr[2 + 3 * lane] | (cr[3 + 3 * lane] << 8);
        ccarry = cr[4 + 3 * lane];
        decode_action(acts[lane], 1, mv, op);
    }
    int pcell, pcarry;
    const TrkView trk = load_view_rows(rec, A, ns, V, pcell, pcarry);
    const float s_a = shaped_agent(trk, C.c, act, pcell, pcarry, ccell, ccarry, mv, op, t_prev, t_cur);
    return (float)gw + np_sum_lanes(s_a, A);
}

__global__ __launch_bounds__(256) void k_views_shaped(DevParams p, const int32_t* __restrict__ prev,
                                                      const int64_t* __restrict__ prev_offs,
                                                      const int32_t* __restrict__ cur,
                                                      const int64_t* __restrict__ cur_offs,
                                                      const uint8_t* __restrict__ acts,
                                                      const int64_t* __restrict__ act_offs,
                                                      const double* __restrict__ g, int n, ShapingConsts C,
                                                      float* __restrict__ out, int wpb, int lds_stride, int NSmax,
                                                      Publish pb) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = wave_id();
    const int w = blockIdx.x * wpb + wave;
    if (wave < wpb && w < n) {
        // every per-transition address / scalar first, in one round trip (host-mapped inputs: each
        // dependent load is a PCIe round trip)
        const int64_t po = prev_offs[w], co = cur_offs[w], ao = act_offs[w];
        const double gw = g[w];
        const float res = views_shaped_one(prev + po, cur + co, acts + ao, gw, C, smem + (size_t)wave * lds_stride,
                                           NSmax);
        if (lane_id() == 0) out[w] = res;
    }
    if (pb.seq) publish_tail(pb);
}

// One transition whose inputs travel in the kernel arguments (mdl_host_view_shaped_reward):
// rec = prev view | current record at word co | action codes at word ao.  One wave, one block.
// The result travels with the completion word: one 64-bit store of (seq, result bits) to the
// 8-byte-aligned pb.seq, so no store has to be ordered before it (no release fence).
template <int CAP>
__global__ __launch_bounds__(64) void k_view_shaped_inl(double g, ShapingConsts C, int co, int ao, int NSmax,
                                                        Publish pb, ViewInline<CAP> rec) {
    extern __shared__ __align__(16) unsigned char smem[];
    const float res = views_shaped_one(rec.w, rec.w + co, (const uint8_t*)(rec.w + ao), g, C, smem, NSmax);
    if (lane_id() == 0) {
        const uint64_t v = (uint64_t)(uint32_t)pb.value | ((uint64_t)__float_as_uint(res) << 32);
        __hip_atomic_store((uint64_t*)pb.seq, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ------------------------------------------------- IDQ / qmix featurizers
// convert_state for every agent and convert_global_state_to_tensor (7, oh, ow)
// from the engine state + tracker.
template <bool STALE>
__global__ __launch_bounds__(256) void k_alt_obs(DevParams p, int env_begin, int n, float* __restrict__ idq,
                                                 float* __restrict__ qst, int oh, int ow, int wpb, int lds_stride) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = wave_id();
    const int lane = lane_id();
    const int w = blockIdx.x * wpb + wave;
    if (wave >= wpb || w >= n) return;
    const int e = env_begin + w;
    const int A = p.A, P = p.P;
    unsigned char* base = smem + (size_t)wave * lds_stride;
    ObsLdsPre S = obs_pre_carve(base, P);
    const MapDesc md = p.maps[p.env_map ? p.env_map[e] : 0];
    const int H = md.H, W = md.W;
    AltLds L = alt_carve(base + obs_pre_bytes(P), H * W);
    const bool act = lane < A;
    const uint32_t rv = act ? p.rob[(size_t)e * A + lane] : 0u;
    const int cell = rob_cell(rv), carry = rob_carry(rv);
    const int t = p.es[e].t;
    for (int j = lane; j < P; j += WAVE) {
        const size_t g = (size_t)e * P + j;
        const uint64_t d = p.pkg[g];
        const uint32_t f = p.pstate[g];
        S.pk[j] = d;
        S.ps[j] = (uint8_t)(f & PS_FLAGS);
        if (STALE) {
            const bool sv = (f & PS_SURVIVOR) != 0;
            S.td[j] = sv ? p.trk[g] : d;
            S.tq[j] = sv ? f >> PS_RANK_SHIFT : ORD_EPISODE + (uint32_t)j;
        }
    }
    wave_sync();
    const uint8_t* grid = p.grids + md.grid_off;
    float* idq_e = idq ? idq + (size_t)w * A * 6 * H * W : nullptr;
    float* qst_e = qst ? qst + (size_t)w * 7 * oh * ow : nullptr;
    const bool fast = (H * W) % 4 == 0 && oh == H && ow == W && (((uintptr_t)idq_e | (uintptr_t)qst_e) & 15) == 0;
    auto run = [&](const auto& trk) {
        alt_prepare(trk, H * W, W, A, t, cell, carry, L);
        if (fast) {
            alt_bits(p.gridbits + md.bits_off, H * W, L);
            alt_emit_fast(trk, H, W, L, cell, carry, A, idq_e, qst_e);
            return;
        }
        if (idq) alt_emit_idq(trk, grid, H, W, L, cell, carry, 0, A, true, idq_e);
        if (qst) alt_emit_qmix(grid, H, W, L, oh, ow, qst_e);
    };
    if (STALE) {
        TrkStale trk{S.ps, S.td, S.tq, P};
        run(trk);
    } else {
        TrkFresh trk{S.pk, S.ps, P};
        run(trk);
    }
}

// The same builders on packed dict views (one agent index per view).
__global__ __launch_bounds__(256) void k_views_alt(DevParams p, const int32_t* __restrict__ views,
                                                   const int64_t* __restrict__ offs, int n,
                                                   const int32_t* __restrict__ agent_idx, float* __restrict__ idq,
                                                   float* __restrict__ qst, int oh, int ow, int wpb, int lds_stride,
                                                   int NSmax) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = wave_id();
    const int w = blockIdx.x * wpb + wave;
    if (wave >= wpb || w >= n) return;
    unsigned char* base = smem + (size_t)wave * lds_stride;
    ViewLdsPre V = view_carve(base, NSmax);
    int t, A, map, cell, carry;
    const TrkView trk = load_view(views + offs[w], V, t, A, map, cell, carry);
    wave_sync();
    const MapDesc md = p.maps[map];
    const int H = md.H, W = md.W;
    AltLds L = alt_carve(base + view_pre_bytes(NSmax), H * W);
    alt_prepare(trk, H * W, W, A, t, cell, carry, L);
    const uint8_t* grid = p.grids + md.grid_off;
    const int a = agent_idx ? agent_idx[w] : 0;
    const bool valid = a >= 0 && a < A;
    if (idq) alt_emit_idq(trk, grid, H, W, L, cell, carry, valid ? a : 0, 1, valid, idq + (size_t)w * 6 * H * W);
    if (qst) alt_emit_qmix(grid, H, W, L, oh, ow, qst + (size_t)w * 7 * oh * ow);
}

// IDQ reward_shaping on packed views: out[op_offs[w] + a] (fp64), ops_are_ints = 0
// reproduces IDQ/trainer.py's string ops.
__global__ __launch_bounds__(256) void k_views_idq_reward(const int32_t* __restrict__ prev,
                                                          const int64_t* __restrict__ prev_offs,
                                                          const int32_t* __restrict__ cur,
                                                          const int64_t* __restrict__ cur_offs,
                                                          const uint8_t* __restrict__ ops,
                                                          const int64_t* __restrict__ op_offs, int ops_are_ints, int n,
                                                          double* __restrict__ out, int wpb, int lds_stride,
                                                          int NSmax) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = wave_id();
    const int lane = lane_id();
    const int w = blockIdx.x * wpb + wave;
    if (wave >= wpb || w >= n) return;
    ViewLdsPre V = view_carve(smem + (size_t)wave * lds_stride, NSmax);
    int t_prev, A, map, pcell, pcarry;
    const TrkView trk = load_view(prev + prev_offs[w], V, t_prev, A, map, pcell, pcarry);
    wave_sync();
    const int32_t* cr = cur + cur_offs[w];
    if (lane < A) {
        const int ccell = cr[2 + 3 * lane] | (cr[3 + 3 * lane] << 8);
        const int ccarry = cr[4 + 3 * lane];
        const int op = ops_are_ints ? (int)ops[op_offs[w] + lane] : -1;
        out[op_offs[w] + lane] = idq_reward(trk, pcell, pcarry, ccell, ccarry, op, t_prev, cr[0]);
    }
}

// ------------------------------------------------------------ state export
// int32 views of the SoA state for the dict-compat layer and the tests.
__global__ __launch_bounds__(256) void k_export(DevParams p, int32_t* __restrict__ robots, int32_t* __restrict__ pkgs,
                                                int32_t* __restrict__ tt, double* __restrict__ total,
                                                int32_t* __restrict__ trk, int32_t* __restrict__ trk_data) {
    const int wave = wave_id();
    const int lane = lane_id();
    const int e = blockIdx.x * 4 + wave;
    if (e >= p.E) return;
    const int A = p.A, P = p.P;
    if (robots && lane < A) {
        const uint32_t rv = p.rob[(size_t)e * A + lane];
        int32_t* o = robots + ((size_t)e * A + lane) * 3;
        o[0] = cell_r(rob_cell(rv));
        o[1] = cell_c(rob_cell(rv));
        o[2] = rob_carry(rv);
    }
    for (int j = lane; j < P; j += WAVE) {
        const size_t g = (size_t)e * P + j;
        const uint64_t d = p.pkg[g];
        const uint32_t f = p.pstate[g];
        const int st = (int)(f & PS_STATUS);
        if (pkgs) {
            int32_t* o = pkgs + g * 8;
            o[0] = cell_r(pk_start(d)); o[1] = cell_c(pk_start(d));
            o[2] = cell_r(pk_target(d)); o[3] = cell_c(pk_target(d));
            o[4] = pk_st(d); o[5] = pk_dl(d); o[6] = j + 1; o[7] = st;
        }
        int present, intr;
        uint32_t order;
        uint64_t td = d;
        if (p.stale) {
            present = (f & PS_PRESENT) ? 1 : 0;
            intr = (f & PS_TRANSIT) ? 1 : 0;
            order = ORD_EPISODE + (uint32_t)j;
            if (f & PS_SURVIVOR) {
                td = p.trk[g];
                order = f >> PS_RANK_SHIFT;
            }
        } else {
            present = st == ST_WAITING || st == ST_IN_TRANSIT;
            intr = st == ST_IN_TRANSIT;
            order = (uint32_t)j;
        }
        if (trk) {
            int32_t* o = trk + g * 4;
            o[0] = present; o[1] = intr; o[2] = (int32_t)order; o[3] = (f & PS_SURVIVOR) ? 1 : 0;
        }
        if (trk_data) {
            int32_t* o = trk_data + g * 6;
            o[0] = cell_r(pk_start(td)); o[1] = cell_c(pk_start(td));
            o[2] = cell_r(pk_target(td)); o[3] = cell_c(pk_target(td));
            o[4] = pk_st(td); o[5] = pk_dl(td);
        }
    }
    if (lane == 0) {
        const EnvScalars s = p.es[e];
        if (tt) tt[e] = s.t;
        if (total) total[e] = s.total;
    }
}

// ------------------------------------------------------- dict-API mailbox export
// The rows of the envs a dict-API call touched (row w = env ids[w], or env w without ids),
// written straight into the engine's host-mapped mailbox (no device staging buffer, no copy
// engine), then one completion word: every wave of the grid counts itself in the running
// counter `ctr` (never reset: `base` is its value before this launch) after a system-scope
// release of its stores; the last one publishes `seq`, which the host spins on (mdl_mail_*).
// Robot / package rows are the k_export layout.
__global__ __launch_bounds__(256) void k_mail_export(DevParams p, const int32_t* __restrict__ ids, int n,
                                                     MailRows m, unsigned* __restrict__ ctr, unsigned base,
                                                     int32_t seq) {
    const int lane = lane_id();
    const int w = blockIdx.x * 4 + wave_id();
    const int A = p.A, P = p.P;
    int e = -1;
    if (w < n) e = ids ? uni(ids[w]) : w;
    if ((unsigned)e < (unsigned)p.E) {
        if (lane < A) {
            const uint32_t rv = p.rob[(size_t)e * A + lane];
            int32_t* o = m.robots + ((size_t)w * A + lane) * 3;
            o[0] = cell_r(rob_cell(rv));
            o[1] = cell_c(rob_cell(rv));
            o[2] = rob_carry(rv);
        }
        for (int j = lane; j < P; j += WAVE) {
            const size_t g = (size_t)e * P + j;
            const uint64_t d = p.pkg[g];
            int4* o = (int4*)(m.pkgs + ((size_t)w * P + j) * 8);
            o[0] = int4{cell_r(pk_start(d)), cell_c(pk_start(d)), cell_r(pk_target(d)), cell_c(pk_target(d))};
            o[1] = int4{pk_st(d), pk_dl(d), j + 1, (int)(p.pstate[g] & PS_STATUS)};
        }
        if (lane == 0) {
            const EnvScalars s = p.es[e];
            m.t[w] = s.t;
            m.total[w] = s.total;
            m.rterms[w] = (int32_t)s.ctr;
        }
    }
    publish_tail(Publish{m.seq, ctr, base, seq});   // the last wave: every row is out
}

// one wave: publish `seq` (host-mapped) once every kernel queued before it on the stream has
// ended (their stores are released at their ends) -- mdl_host_wait's completion word
__global__ __launch_bounds__(64) void k_publish(int32_t* seq, int32_t value) {
    if (threadIdx.x == 0) __hip_atomic_store(seq, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------- launchers
static int blocks_for(int n, int wpb) { return (n + wpb - 1) / wpb; }

hipError_t launch_publish(int32_t* seq, int32_t value, hipStream_t s) {
    hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, s, seq, value);
    return hipGetLastError();
}

unsigned mail_export_waves(int n) { return 4u * (unsigned)blocks_for(n > 0 ? n : 1, 4); }
unsigned grid_waves(int n, int wpb) { return 4u * (unsigned)blocks_for(n, wpb); }

hipError_t launch_mail_export(const DevParams& p, const int32_t* ids, int n, const MailRows& m, unsigned* ctr,
                              unsigned base, int32_t seq, hipStream_t s) {
    hipLaunchKernelGGL(k_mail_export, dim3(blocks_for(n > 0 ? n : 1, 4)), dim3(256), 0, s, p, ids, n, m, ctr, base,
                       seq);
    return hipGetLastError();
}

static int nch_for(int P) {
    const int c = (P + WAVE - 1) / WAVE;
    return c <= 1 ? 1 : c <= 2 ? 2 : c <= 4 ? 4 : c <= 8 ? 8 : 16;
}

hipError_t launch_seed(const DevParams& p, const uint32_t* seeds, int wpb, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL(k_seed, dim3(blocks_for(p.E, wpb)), dim3(256), lds * wpb, s, p, seeds, wpb, (int)lds);
    return hipGetLastError();
}

template <int NCH>
static void launch_reset_t(const DevParams& p, const int* ids, int n, int wpb, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL(k_reset<NCH>, dim3(blocks_for(n, wpb)), dim3(256), lds * wpb, s, p, ids, n, wpb, (int)lds);
}

hipError_t launch_reset(const DevParams& p, const int* ids, int n, int wpb, size_t lds, hipStream_t s) {
    switch (nch_for(p.P)) {
        case 1: launch_reset_t<1>(p, ids, n, wpb, lds, s); break;
        case 2: launch_reset_t<2>(p, ids, n, wpb, lds, s); break;
        case 4: launch_reset_t<4>(p, ids, n, wpb, lds, s); break;
        case 8: launch_reset_t<8>(p, ids, n, wpb, lds, s); break;
        default: launch_reset_t<16>(p, ids, n, wpb, lds, s); break;
    }
    return hipGetLastError();
}

hipError_t launch_tracker_clear(const DevParams& p, const int* ids, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_tracker_clear, dim3(blocks_for(n, 4)), dim3(256), 0, s, p, ids, n);
    return hipGetLastError();
}

template <bool ST, int NCH, bool FUSED>
static void launch_step_t(const DevParams& p, const uint8_t* actions, int fmt, const int* ids, int n, int auto_reset,
                          double* r, float* sh, uint8_t* done, int wpb, size_t lds, int K, hipStream_t s) {
    // n and wpb travel packed in one preloaded dword (n < 2^24, wpb < 32; the engine
    // checks both at creation)
    const int threads = 64 * wpb;
#ifdef MDL_EXP_NOLDS  // profiling builds only: no LDS request (valid only while no env resets)
    lds = 0;
#endif
    StepArgs a;
    a.p = p;
    a.actions = actions;
    a.env_ids = ids;
    a.r_out = r;
    a.sh_out = sh;
    a.done_out = done;
    a.fmt = fmt;
    a.n = n;
    a.auto_reset = auto_reset;
    a.wpb = wpb;
    a.lds_stride = (int)lds;
    a.K = K;
    const dim3 grid(blocks_for(n, wpb)), block(threads);
    const uint32_t ap = pack_ap(p.A, p.P, (int)grid.x);
    const uint32_t nw = (uint32_t)n | ((uint32_t)wpb << 24) | (ids ? NW_IDS : 0u) | (p.env_map ? NW_MAP : 0u);
#define MDL_STEP_ARGS p.rob, p.pkg, p.pstate, (const u32x4*)p.es, p.trk, actions, ap, nw, a
    if (NCH <= 2 && p.A == 5)
        hipLaunchKernelGGL((k_step<ST, NCH, FUSED, (NCH <= 2 ? 5 : 8)>), grid, block, lds * wpb, s, MDL_STEP_ARGS);
    else if (NCH <= 2 && p.A == 16)   // config 5's robot count
        hipLaunchKernelGGL((k_step<ST, NCH, FUSED, (NCH <= 2 ? 16 : 8)>), grid, block, lds * wpb, s, MDL_STEP_ARGS);
    else if (p.A <= 8)
        hipLaunchKernelGGL((k_step<ST, NCH, FUSED, 8>), grid, block, lds * wpb, s, MDL_STEP_ARGS);
    else
        hipLaunchKernelGGL((k_step<ST, NCH, FUSED, 0>), grid, block, lds * wpb, s, MDL_STEP_ARGS);
#undef MDL_STEP_ARGS
}

// P <= 64 (four chunks per lane).  Eight chunks (P <= 128) were built and measured slower than
// k_step at P = 100 (16,384 envs 14.2 vs 10.6 us, 65,536 39.7 vs 33.9: profiles/r05/rows_ab.txt)
bool step_rows_ok(int A, int P) { return A >= 1 && A <= 8 && P >= 1 && P <= ROW * 4; }
size_t step_rows_lds(int P) {
    const size_t a = reset_lds_bytes(P), b = rows_scratch_bytes(4);
    return a > b ? a : b;
}

// A == 16 exactly (numpy's pairwise sum of 16 values in-row; 9..15 would need its sequential
// tail), P <= 128 (four 32-lane chunks)
bool step_halves_ok(int A, int P) { return A == 16 && P >= 1 && P <= HALF * HALF_NC; }
size_t step_halves_lds(int P) {
    const size_t a = reset_lds_bytes(P), b = halves_scratch_bytes();
    return a > b ? a : b;
}

hipError_t launch_step_halves(const DevParams& p, const uint8_t* actions, int fmt, int n, int auto_reset, double* r,
                              float* sh, uint8_t* done, int wpb, size_t lds, hipStream_t s) {
    if (!step_halves_ok(p.A, p.P)) return hipErrorInvalidValue;
    StepArgs a;
    a.p = p;
    a.actions = actions;
    a.env_ids = nullptr;
    a.r_out = r;
    a.sh_out = sh;
    a.done_out = done;
    a.fmt = fmt;
    a.n = n;
    a.auto_reset = auto_reset;
    a.wpb = wpb;
    a.lds_stride = (int)lds;
    a.K = 1;
    const int waves = (n + 1) / 2;
    const dim3 grid(blocks_for(waves, wpb)), block(64 * wpb);
    const uint32_t ap = pack_ap(p.A, p.P, (int)grid.x);
    bool small = true;
    for (int k = 0; k < p.n_maps; k++) small = small && p.maps[k].H <= 64 && p.maps[k].W <= 64;
    const uint32_t nw = (uint32_t)n | ((uint32_t)wpb << 24) | (p.env_map ? NW_MAP : 0u) | (small ? NW_SMALLMAP : 0u);
#define MDL_STEP_ARGS p.rob, p.pkg, p.pstate, (const u32x4*)p.es, p.trk, actions, ap, nw, a
    const bool full3 = p.P >= 3 * HALF;
    if (p.stale && full3) hipLaunchKernelGGL((k_step_halves<true, 3>), grid, block, lds * wpb, s, MDL_STEP_ARGS);
    else if (p.stale) hipLaunchKernelGGL((k_step_halves<true, 0>), grid, block, lds * wpb, s, MDL_STEP_ARGS);
    else if (full3) hipLaunchKernelGGL((k_step_halves<false, 3>), grid, block, lds * wpb, s, MDL_STEP_ARGS);
    else hipLaunchKernelGGL((k_step_halves<false, 0>), grid, block, lds * wpb, s, MDL_STEP_ARGS);
#undef MDL_STEP_ARGS
    return hipGetLastError();
}

hipError_t launch_step_rows(const DevParams& p, const uint8_t* actions, int fmt, int n, int auto_reset, double* r,
                            float* sh, uint8_t* done, int wpb, size_t lds, hipStream_t s) {
    if (!step_rows_ok(p.A, p.P)) return hipErrorInvalidValue;
    StepArgs a;
    a.p = p;
    a.actions = actions;
    a.env_ids = nullptr;
    a.r_out = r;
    a.sh_out = sh;
    a.done_out = done;
    a.fmt = fmt;
    a.n = n;
    a.auto_reset = auto_reset;
    a.wpb = wpb;
    a.lds_stride = (int)lds;
    a.K = 1;
    const int waves = (n + 3) / 4;
    const dim3 grid(blocks_for(waves, wpb)), block(64 * wpb);
    const uint32_t ap = pack_ap(p.A, p.P, (int)grid.x);
    const uint32_t nw = (uint32_t)n | ((uint32_t)wpb << 24) | (p.env_map ? NW_MAP : 0u);
#define MDL_STEP_ARGS p.rob, p.pkg, p.pstate, (const u32x4*)p.es, p.trk, actions, ap, nw, a
#define MDL_ROWS(ST, NF)                                                                                     \
    do {                                                                                                     \
        if (p.A == 5) hipLaunchKernelGGL((k_step_rows<ST, 5, 4, NF>), grid, block, lds * wpb, s, MDL_STEP_ARGS);   \
        else hipLaunchKernelGGL((k_step_rows<ST, 8, 4, NF>), grid, block, lds * wpb, s, MDL_STEP_ARGS);      \
    } while (0)
    const bool full3 = p.P >= 3 * ROW;
    if (p.stale && full3) MDL_ROWS(true, 3);
    else if (p.stale) MDL_ROWS(true, 0);
    else if (full3) MDL_ROWS(false, 3);
    else MDL_ROWS(false, 0);
#undef MDL_ROWS
#undef MDL_STEP_ARGS
    return hipGetLastError();
}

// (the dispatch of launch_step_rows / launch_step_halves above, launch_step_obs and launch_step_t below)
int step_kernel_name(const DevParams& p, int envs_per_wave, bool obs, char* out, int cap) {
    const char* st = p.stale ? "true" : "false";
    if (envs_per_wave == 4)
        return snprintf(out, (size_t)cap, "mdl::k_step_rows<%s, %d, 4, %d>", st, p.A == 5 ? 5 : 8, p.P >= 3 * ROW ? 3 : 0);
    if (envs_per_wave == 2) return snprintf(out, (size_t)cap, "mdl::k_step_halves<%s, %d>", st, p.P >= 3 * HALF ? 3 : 0);
    if (obs) return snprintf(out, (size_t)cap, "mdl::k_step_obs<%s, %d>", st, p.A == 5 ? 5 : 8);
    const int nch = nch_for(p.P);
    const int au = (nch <= 2 && p.A == 5) ? 5 : (nch <= 2 && p.A == 16) ? 16 : p.A <= 8 ? 8 : 0;
    return snprintf(out, (size_t)cap, "mdl::k_step<%s, %d, false, %d>", st, nch, au);
}

hipError_t launch_step_floor(const DevParams& p, int n, int wpb, size_t lds, hipStream_t s, int envs_per_wave) {
    StepArgs a{};
    a.p = p;
    a.n = n;
    a.wpb = wpb;
    a.lds_stride = (int)lds;
    a.K = 1;
    const dim3 grid(blocks_for((n + envs_per_wave - 1) / envs_per_wave, wpb)), block(64 * wpb);
    const uint32_t ap = pack_ap(p.A, p.P, (int)grid.x);
    const uint32_t nw = (uint32_t)n | ((uint32_t)wpb << 24) | (p.env_map ? NW_MAP : 0u);
    hipLaunchKernelGGL(k_step_floor, grid, block, lds * wpb, s, p.rob, p.pkg, p.pstate, (const u32x4*)p.es, p.trk,
                       (const uint8_t*)nullptr, ap, nw, a);
    return hipGetLastError();
}

template <bool ST, bool FUSED>
static void launch_step_s(const DevParams& p, const uint8_t* actions, int fmt, const int* ids, int n, int auto_reset,
                          double* r, float* sh, uint8_t* done, int wpb, size_t lds, int K, hipStream_t s) {
    switch (nch_for(p.P)) {
        case 1: launch_step_t<ST, 1, FUSED>(p, actions, fmt, ids, n, auto_reset, r, sh, done, wpb, lds, K, s); break;
        case 2: launch_step_t<ST, 2, FUSED>(p, actions, fmt, ids, n, auto_reset, r, sh, done, wpb, lds, K, s); break;
        case 4: launch_step_t<ST, 4, FUSED>(p, actions, fmt, ids, n, auto_reset, r, sh, done, wpb, lds, K, s); break;
        case 8: launch_step_t<ST, 8, FUSED>(p, actions, fmt, ids, n, auto_reset, r, sh, done, wpb, lds, K, s); break;
        default: launch_step_t<ST, 16, FUSED>(p, actions, fmt, ids, n, auto_reset, r, sh, done, wpb, lds, K, s); break;
    }
}

template <bool ST, int NCH>
static void launch_step_mail_t(const StepArgs& a, const uint8_t* actions, const MailArgs& ma, int inl, int wpb,
                               size_t lds, hipStream_t s) {
    const DevParams& p = a.p;
    const dim3 grid(blocks_for(a.n, wpb)), block(64 * wpb);
    const uint32_t ap = pack_ap(p.A, p.P, (int)grid.x);
    const uint32_t nw = (uint32_t)a.n | ((uint32_t)wpb << 24) | (a.env_ids ? NW_IDS : 0u) | (p.env_map ? NW_MAP : 0u);
#define MDL_STEP_ARGS p.rob, p.pkg, p.pstate, (const u32x4*)p.es, p.trk, actions, ap, nw, a, ma, inl
    if (p.A <= 8) hipLaunchKernelGGL((k_step_mail<ST, NCH, 8>), grid, block, lds * wpb, s, MDL_STEP_ARGS);
    else hipLaunchKernelGGL((k_step_mail<ST, NCH, 0>), grid, block, lds * wpb, s, MDL_STEP_ARGS);
#undef MDL_STEP_ARGS
}

hipError_t launch_step_mail(const DevParams& p, const uint8_t* codes, const int* ids, int n, int auto_reset, double* r,
                            float* sh, uint8_t* done, int wpb, size_t lds, const MailRows& m, unsigned* ctr,
                            unsigned base, int32_t seq, hipStream_t s) {
    StepArgs a;
    a.p = p;
    a.actions = codes;
    a.env_ids = ids;
    a.r_out = r;
    a.sh_out = sh;
    a.done_out = done;
    a.fmt = 1;   // MDL_ACTION_CODES (decode_action)
    a.n = n;
    a.auto_reset = auto_reset;
    a.wpb = wpb;
    a.lds_stride = (int)lds;
    a.K = 1;
    MailArgs ma;
    ma.m = m;
    ma.pb = Publish{m.seq, ctr, base, seq, (unsigned)n};
    const size_t nb = (size_t)n * p.A;
    const int inl = nb <= (size_t)MAIL_INLINE_CODES;
    if (inl) std::memcpy(ma.codes, codes, nb);
    const bool st = p.stale != 0;
    switch (nch_for(p.P)) {
        case 1: st ? launch_step_mail_t<true, 1>(a, codes, ma, inl, wpb, lds, s) : launch_step_mail_t<false, 1>(a, codes, ma, inl, wpb, lds, s); break;
        case 2: st ? launch_step_mail_t<true, 2>(a, codes, ma, inl, wpb, lds, s) : launch_step_mail_t<false, 2>(a, codes, ma, inl, wpb, lds, s); break;
        case 4: st ? launch_step_mail_t<true, 4>(a, codes, ma, inl, wpb, lds, s) : launch_step_mail_t<false, 4>(a, codes, ma, inl, wpb, lds, s); break;
        case 8: st ? launch_step_mail_t<true, 8>(a, codes, ma, inl, wpb, lds, s) : launch_step_mail_t<false, 8>(a, codes, ma, inl, wpb, lds, s); break;
        default: st ? launch_step_mail_t<true, 16>(a, codes, ma, inl, wpb, lds, s) : launch_step_mail_t<false, 16>(a, codes, ma, inl, wpb, lds, s); break;
    }
    return hipGetLastError();
}

hipError_t launch_step(const DevParams& p, const uint8_t* actions, int fmt, const int* ids, int n, int auto_reset,
                       double* r, float* sh, uint8_t* done, int wpb, size_t lds, hipStream_t s) {
    if (p.stale) launch_step_s<true, false>(p, actions, fmt, ids, n, auto_reset, r, sh, done, wpb, lds, 1, s);
    else launch_step_s<false, false>(p, actions, fmt, ids, n, auto_reset, r, sh, done, wpb, lds, 1, s);
    return hipGetLastError();
}

// k_step_obs (mdl_step_obs): full batch, NCH = 1, A <= 8, the small observation builder;
// lds = the per-wave slice (max of the step's reset scratch and the builder's planes)
hipError_t launch_step_obs(const DevParams& p, const uint8_t* actions, int fmt, int n, int auto_reset, double* r,
                           float* sh, uint8_t* done, float* amap, float* avec, float* cmap, float* cvec, int wpb,
                           size_t lds, hipStream_t s) {
    if (nch_for(p.P) != 1 || p.A > 8 || !p.obs_small) return hipErrorInvalidValue;
    StepArgs a;
    a.p = p;
    a.actions = actions;
    a.env_ids = nullptr;
    a.r_out = r;
    a.sh_out = sh;
    a.done_out = done;
    a.fmt = fmt;
    a.n = n;
    a.auto_reset = auto_reset;
    a.wpb = wpb;
    a.lds_stride = (int)lds;
    a.K = 1;
    const ObsArgs o{amap, avec, cmap, cvec};
    const dim3 grid(blocks_for(n, wpb)), block(64 * wpb);
    const uint32_t ap = pack_ap(p.A, p.P, (int)grid.x);
    const uint32_t nw = (uint32_t)n | ((uint32_t)wpb << 24) | (p.env_map ? NW_MAP : 0u);
#define MDL_STEP_ARGS p.rob, p.pkg, p.pstate, (const u32x4*)p.es, p.trk, actions, ap, nw, a, o
    if (p.stale) {
        if (p.A == 5) hipLaunchKernelGGL((k_step_obs<true, 5>), grid, block, lds * wpb, s, MDL_STEP_ARGS);
        else hipLaunchKernelGGL((k_step_obs<true, 8>), grid, block, lds * wpb, s, MDL_STEP_ARGS);
    } else {
        if (p.A == 5) hipLaunchKernelGGL((k_step_obs<false, 5>), grid, block, lds * wpb, s, MDL_STEP_ARGS);
        else hipLaunchKernelGGL((k_step_obs<false, 8>), grid, block, lds * wpb, s, MDL_STEP_ARGS);
    }
#undef MDL_STEP_ARGS
    return hipGetLastError();
}

size_t alt_obs_lds(int P, int HW) { return obs_pre_bytes(P) + alt_lds_bytes(HW); }
size_t views_alt_lds(int NSmax, int HW) { return view_pre_bytes(NSmax) + alt_lds_bytes(HW); }

hipError_t launch_alt_obs(const DevParams& p, int env_begin, int n, float* idq, float* qst, int oh, int ow, int wpb,
                          size_t lds, hipStream_t s) {
    if (p.stale)
        hipLaunchKernelGGL(k_alt_obs<true>, dim3(blocks_for(n, wpb)), dim3(256), lds * wpb, s, p, env_begin, n, idq,
                           qst, oh, ow, wpb, (int)lds);
    else
        hipLaunchKernelGGL(k_alt_obs<false>, dim3(blocks_for(n, wpb)), dim3(256), lds * wpb, s, p, env_begin, n, idq,
                           qst, oh, ow, wpb, (int)lds);
    return hipGetLastError();
}

hipError_t launch_views_alt(const DevParams& p, const int32_t* views, const int64_t* offs, int n,
                            const int32_t* agent_idx, float* idq, float* qst, int oh, int ow, int wpb, size_t lds,
                            int NSmax, hipStream_t s) {
    hipLaunchKernelGGL(k_views_alt, dim3(blocks_for(n, wpb)), dim3(256), lds * wpb, s, p, views, offs, n, agent_idx,
                       idq, qst, oh, ow, wpb, (int)lds, NSmax);
    return hipGetLastError();
}

hipError_t launch_views_idq_reward(const int32_t* prev, const int64_t* prev_offs, const int32_t* cur,
                                   const int64_t* cur_offs, const uint8_t* ops, const int64_t* op_offs,
                                   int ops_are_ints, int n, double* out, int wpb, size_t lds, int NSmax,
                                   hipStream_t s) {
    hipLaunchKernelGGL(k_views_idq_reward, dim3(blocks_for(n, wpb)), dim3(256), lds * wpb, s, prev, prev_offs, cur,
                       cur_offs, ops, op_offs, ops_are_ints, n, out, wpb, (int)lds, NSmax);
    return hipGetLastError();
}

hipError_t launch_step_fused(const DevParams& p, const uint8_t* actions, int fmt, const int* ids, int n, int K,
                             int auto_reset, double* r, float* sh, uint8_t* done, int wpb, size_t lds,
                             hipStream_t s) {
    if (p.stale) launch_step_s<true, true>(p, actions, fmt, ids, n, auto_reset, r, sh, done, wpb, lds, K, s);
    else launch_step_s<false, true>(p, actions, fmt, ids, n, auto_reset, r, sh, done, wpb, lds, K, s);
    return hipGetLastError();
}

hipError_t launch_obs(const DevParams& p, int env_begin, int n, float* amap, float* avec, float* cmap, float* cvec,
                      int wpb, size_t lds, hipStream_t s, int rank_lds) {
    if (p.obs_small) {
        const dim3 g(blocks_for(n, wpb)), b(256);
        const size_t dyn = (size_t)rank_lds + lds * wpb;
#define MDL_OBS_SMALL(ST, RL) \
    hipLaunchKernelGGL((k_obs_small<ST, RL>), g, b, dyn, s, p, env_begin, n, amap, avec, cmap, cvec, wpb, (int)lds, rank_lds)
        if (p.stale) {
            if (rank_lds > 0) MDL_OBS_SMALL(true, true);
            else MDL_OBS_SMALL(true, false);
        } else {
            if (rank_lds > 0) MDL_OBS_SMALL(false, true);
            else MDL_OBS_SMALL(false, false);
        }
#undef MDL_OBS_SMALL
        return hipGetLastError();
    }
    if (p.stale)
        hipLaunchKernelGGL(k_obs<true>, dim3(blocks_for(n, wpb)), dim3(256), lds * wpb, s, p, env_begin, n, amap,
                           avec, cmap, cvec, wpb, (int)lds);
    else
        hipLaunchKernelGGL(k_obs<false>, dim3(blocks_for(n, wpb)), dim3(256), lds * wpb, s, p, env_begin, n, amap,
                           avec, cmap, cvec, wpb, (int)lds);
    return hipGetLastError();
}

hipError_t launch_views_features(const DevParams& p, const int32_t* views, const int64_t* offs, int n,
                                 const int32_t* agent_idx, int T, int MO, int MP, int MR, int MPs, int MPc, int MPsc,
                                 int NSmax, int HW, float* obs, float* vec, float* gmap, float* gvec, int wpb,
                                 size_t lds, hipStream_t s, const Publish& pb) {
    hipLaunchKernelGGL(k_views_features, dim3(blocks_for(n, wpb)), dim3(256), lds * wpb, s, p, views, offs, n,
                       agent_idx, T, MO, MP, MR, MPs, MPc, MPsc, NSmax, obs, vec, gmap, gvec, wpb, (int)lds, HW, pb);
    return hipGetLastError();
}

hipError_t launch_view_features_inline(const DevParams& p, const int32_t* rec, int words, int a, int T, int MO,
                                      int MP, int MR, int MPs, int MPc, int MPsc, int NSmax, int HW, float* obs,
                                      float* vec, float* gmap, float* gvec, size_t lds, hipStream_t s,
                                      const Publish& pb) {
    if (words <= VIEW_INLINE_SMALL) {
        ViewInline<VIEW_INLINE_SMALL> r;
        std::memcpy(r.w, rec, 4 * (size_t)words);
        hipLaunchKernelGGL(k_view_features_inl<VIEW_INLINE_SMALL>, dim3(1), dim3(64), lds, s, p, a, T, MO, MP, MR,
                           MPs, MPc, MPsc, NSmax, obs, vec, gmap, gvec, HW, pb, r);
    } else {
        ViewInline<VIEW_INLINE_WORDS> r;
        std::memcpy(r.w, rec, 4 * (size_t)words);
        hipLaunchKernelGGL(k_view_features_inl<VIEW_INLINE_WORDS>, dim3(1), dim3(64), lds, s, p, a, T, MO, MP, MR,
                           MPs, MPc, MPsc, NSmax, obs, vec, gmap, gvec, HW, pb, r);
    }
    return hipGetLastError();
}

hipError_t launch_view_shaped_inline(const int32_t* rec, int words, int co, int ao, double g, const ShapingConsts& C,
                                     int NSmax, size_t lds, hipStream_t s, const Publish& pb) {
    if (words <= VIEW_INLINE_SMALL) {
        ViewInline<VIEW_INLINE_SMALL> r;
        std::memcpy(r.w, rec, 4 * (size_t)words);
        hipLaunchKernelGGL(k_view_shaped_inl<VIEW_INLINE_SMALL>, dim3(1), dim3(64), lds, s, g, C, co, ao, NSmax, pb,
                           r);
    } else {
        ViewInline<VIEW_INLINE_WORDS> r;
        std::memcpy(r.w, rec, 4 * (size_t)words);
        hipLaunchKernelGGL(k_view_shaped_inl<VIEW_INLINE_WORDS>, dim3(1), dim3(64), lds, s, g, C, co, ao, NSmax, pb,
                           r);
    }
    return hipGetLastError();
}

hipError_t launch_views_shaped(const DevParams& p, const int32_t* prev, const int64_t* prev_offs, const int32_t* cur,
                               const int64_t* cur_offs, const uint8_t* acts, const int64_t* act_offs, const double* g,
                               int n, const ShapingConsts& C, float* out, int wpb, size_t lds, int NSmax,
                               hipStream_t s, const Publish& pb) {
    hipLaunchKernelGGL(k_views_shaped, dim3(blocks_for(n, wpb)), dim3(256), lds * wpb, s, p, prev, prev_offs, cur,
                       cur_offs, acts, act_offs, g, n, C, out, wpb, (int)lds, NSmax, pb);
    return hipGetLastError();
}

hipError_t launch_export(const DevParams& p, int32_t* robots, int32_t* pkgs, int32_t* t, double* total,
                         int32_t* tracker, int32_t* tracker_data, hipStream_t s) {
    hipLaunchKernelGGL(k_export, dim3(blocks_for(p.E, 4)), dim3(256), 0, s, p, robots, pkgs, t, total, tracker,
                       tracker_data);
    return hipGetLastError();
}

size_t step_lds(int P) { return reset_lds_bytes(P); }
size_t obs_lds_small(int A, int HW, int P, int MO, int MP) { return obs_small_lds(A, HW, P, MO, MP); }
bool obs_use_small(int A, int P, int key7_dsh, int maxHW, int MO, int MP) {
    return obs_small_ok(A, P, key7_dsh, maxHW, MO, MP);
}
size_t obs_lds(int A, int P, int HW, int MO, int MP, int MR, int MPs) {
    const int MPc = MP < P ? MP : P, MPsc = MPs < P ? MPs : P;
    FeatDims d{A, P, HW, MPc, MPsc, stage_floats(A, A, MO, MPc, MR, MPsc)};
    return obs_pre_bytes(P) + feat_lds_bytes(d) + 4 * (size_t)obs_plane_words(A, HW);
}
int obs_plane_words(int A, int HW) {
    const int w = plane_words(A, HW);
    return w <= 2048 ? w : 0;   // larger maps (64x64) keep the per-float4 bitset path
}
size_t views_lds(int NSmax, int HW, int MO, int MPc, int MR, int MPsc) {
    FeatDims d{64, NSmax, HW, MPc, MPsc, stage_floats(64, 1, MO, MPc, MR, MPsc)};
    return view_pre_bytes(NSmax) + feat_lds_bytes(d);
}
size_t views_shaped_lds(int NSmax) { return view_pre_bytes(NSmax); }

}  // namespace mdl

#ifdef MDL_STAMPS
extern "C" int mdl_debug_stamps(void* dst, size_t bytes) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(mdl::g_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
#endif
