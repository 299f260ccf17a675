// mdl_device.hpp -- device-side building blocks of the marl-delivery engine.
//
// Execution model (gfx950 / CDNA4): ONE WAVEFRONT (64 lanes) PER ENV INSTANCE.
//   * robots live on lanes (lane a = robot a, A <= 64), so the cell-contention
//     rule is resolved with readlane / ballot, no LDS round trips;
//   * package tables are staged in the wave's slice of LDS and scanned with
//     lanes over packages (64 per pass);
//   * every sequential piece of the reference (reward fold in robot order,
//     numpy RNG draws, numpy's pairwise float32 sum) runs as wave-uniform
//     scalar code on values broadcast by readlane.
// Waves of one workgroup are independent envs and never barrier together;
// intra-wave LDS ordering uses wave_sync() (wavefront-scope fences).
//
// Reference semantics are cited path:line under the reference tree.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Profiling-only switches change what the kernels compute (skipped sections, missing stores,
// no LDS request) or add diagnostic stores: they are accepted only in a build that says it is
// one (-DMDL_PROFILING_BUILD), never in the product library.
#if !defined(MDL_PROFILING_BUILD) && \
    (defined(MDL_EXP_NOWAIT) || defined(MDL_EXP_NOTUPLES) || defined(MDL_EXP_NOLDS) || defined(MDL_ABLATE) || \
     defined(MDL_STAMPS))
#error "MDL_EXP_NOWAIT / MDL_EXP_NOTUPLES / MDL_EXP_NOLDS / MDL_ABLATE / MDL_STAMPS need -DMDL_PROFILING_BUILD"
#endif
// Profiling-only ablation builds (MDL_PROFILING_BUILD, scripts/ablate.sh): bit 1 skips the shaped
// reward, 2 the tracker update, 4 movement, 8 package actions, 16 the move-validity reload, 32 the
// shaping agent loops, 64 the carried-package gather; in the small observation builder 128 the
// actor vectors' computation, 256 the critic vector's, 512 the map planes' (their bytes are still
// written).  0 in the product.
#ifndef MDL_ABLATE
#define MDL_ABLATE 0
#endif

namespace mdl {

constexpr int WAVE = 64;
constexpr int MT_N = 624;
constexpr int MT_M = 397;
constexpr int MAX_MAPS = 8;

enum : int { ST_NONE = 0, ST_WAITING = 1, ST_IN_TRANSIT = 2, ST_DELIVERED = 3 };
enum : int { MV_S = 0, MV_L = 1, MV_R = 2, MV_U = 3, MV_D = 4, MV_OTHER = 5 };
// shaping constant slots (MAPPO/helper.py:271-279 order of use)
enum : int { SH_PICK = 0, SH_ONTIME, SH_LATE, SH_CLOSER, SH_WPICK, SH_WDROP, SH_STUCK, SH_IDLE, SH_AWAY };

struct MapDesc {
    int H, W, nfree;
    int grid_off;   // into grids (bytes)
    int free_off;   // into free_cells (u16 packed r | c<<8, row-major)
    int rank_off;   // into rank (u16) table [(2H-1)][(2W-1)]
    float inv_hw;   // 1/(H*W) for fast divmod
    int bits_off;   // into gridbits (u32 words, ceil(H*W/32) per map)
    int mvc_off;    // into movevalid_cell (256*W bytes per map, indexed by the packed cell r | c<<8)
};

// Per-env scalars, one 16-byte record (one load / one store per step).
struct __align__(16) EnvScalars {
    int32_t t;       // Environment.t
    uint32_t ctr;    // RT_* bits: the reward terms the last step added (0 after a reset)
    double total;    // Environment.total_reward (fp64, as the reference's Python float)
};
// env.py's step reward starts as the int 0 (env.py:181) and takes the type of what is added to
// it: move costs (:256), on-time (:288) / late (:291) delivery rewards
enum : uint32_t { RT_MOVE = 1u, RT_ONTIME = 2u, RT_LATE = 4u };

// Per-package state word (u16): bits 0-1 env status (ST_*), then the persistent
// tracker's view of the same id (stale mode): present, in_transit, survivor
// (inserted in an earlier episode -> its data lives in `trk`, not `pkg`).
enum : uint32_t { PS_STATUS = 3u, PS_PRESENT = 4u, PS_TRANSIT = 8u, PS_SURVIVOR = 16u, PS_FLAGS = 31u };
// bits 5-15 of the state word: a survivor's dict-order rank (see ORD_EPISODE)
constexpr int PS_RANK_SHIFT = 5;

// Tracker iteration-order keys (stale mode), all < 0x800: a survivor's key is
// its rank among the entries present at the last reset (pstate bits 5-15), an
// entry of the running episode has ORD_EPISODE + slot (spawn order == id
// order).  Dict order == ascending key.
constexpr uint32_t ORD_EPISODE = 0x400u;

// Everything a kernel needs about the engine, passed by value.
struct DevParams {
    int E, A, P, T;
    double move_cost, delivery_reward, delay_reward;
    double cost_sum[9];  // cost_sum[k] = ((0.0 + move_cost) + move_cost) ... k times: env.py:252-257's fold
    float shaping[9];
    int stale;
    int obsT, MO, MP, MR, MPs;
    int n_maps;
    int key32_dsh;  // > 0: the obs sort keys (dlc, rank, order) fit 32 bits, dlc at this shift
    MapDesc maps[MAX_MAPS];
    const uint8_t* grids;
    const uint8_t* movevalid;  // per map cell: bit m set if move code m (L,R,U,D = 1..4) stays on a free cell
    const uint8_t* movevalid_cell;  // the same bits indexed by the packed cell value (no r*W+c in the step)
    const uint32_t* gridbits;  // per map obstacle bitset
    const uint16_t* free_cells;
    const uint16_t* rank;
    const uint8_t* env_map;    // [E] or null
    // state (SoA, env-major)
    uint32_t* rob;             // [E][A] robot word, see rob_pack()
    uint64_t* pkg;             // [E][P] sr|sc<<8|tr<<16|tc<<24|st<<32|dl<<48 (cells packed r|c<<8)
    uint16_t* pstate;          // [E][P] PS_* bits | survivor rank << PS_RANK_SHIFT
    EnvScalars* es;            // [E]
    uint32_t* mt;              // [E][624]
    int32_t* mt_pos;           // [E]
    uint64_t* trk;             // [E][P] stale mode: a tracker entry's data (written at insertion)
    double* ep_total;          // [E] total_reward of the last finished episode
    int32_t* ep_len;           // [E]
    // observation builders (appended: the step kernel's argument layout stays put)
    const double* obs_recip;   // [2 * n_maps + 2]: 1/H, 1/W of each map, then 1/obsT, 1/(MR-1), fp64 RN
    int obs_plane_words;       // > 0: k_obs stages the map planes as bit words (LDS words reserved per wave)
    int obs_small;             // k_obs_small builds the observations (mdl_obs_small.hpp)
    int key7_dsh;              // > 0: (max(0,dl-t), rank, 7-bit order) fits 32 bits, dlc at this shift
    // cost_fold[k] = the reference's k-fold move-cost sum for every k <= 64 robots (cost_sum's
    // 9 entries, read in the step's first scalar batch, serve A <= 8; the wider kernels index
    // this one instead of adding move_cost n_cost times in a dependent fp64 chain)
    double cost_fold[65];
};

// Robot word: bits 0-15 cell (r | c<<8), bits 16-26 carried package id,
// bits 27-30 valid_position() of the L/R/U/D neighbours of the cell (so the
// step needs no dependent map lookup before resolving moves).
__host__ __device__ __forceinline__ uint32_t rob_pack(int cell, int carry, uint32_t valid_mask /* bits 1..4 */) {
    return (uint32_t)cell | ((uint32_t)carry << 16) | ((valid_mask & 0x1eu) << 26);
}
__host__ __device__ __forceinline__ int rob_cell(uint32_t w) { return (int)(w & 0xffffu); }
__host__ __device__ __forceinline__ int rob_carry(uint32_t w) { return (int)((w >> 16) & 0x7ffu); }
__host__ __device__ __forceinline__ uint32_t rob_valid(uint32_t w) { return (w >> 26) & 0x1eu; }

// ---------------------------------------------------------------- wave utils
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
// wave index in the workgroup as a wave-uniform (SGPR) value, so per-env
// addressing and the map descriptor lookup are scalar
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

// Workgroups are dealt round-robin to the 8 XCDs, each with its own L2: workgroup b of nb runs on
// XCD b % 8.  xcd_block() renumbers them so that each XCD's workgroups take one contiguous range
// of block slots: the envs of an XCD (and so every cache line of their rows, shared with
// neighbours or not) are touched by that XCD alone, launch after launch, and each launch finds
// the rows the previous one wrote in that XCD's L2 (scripts/exp/l2_retain.hip: the state round
// trip 1344 -> 1020 cycles at 4096 envs).  A bijection on [0, nb).
__device__ __forceinline__ int xcd_slot(int b, int nb) { return (b & 7) * (nb >> 3) + min(b & 7, nb & 7) + (b >> 3); }
__device__ __forceinline__ int xcd_block() {
    return xcd_slot((int)blockIdx.x, (int)gridDim.x);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// Global (address space 1) pointer qualifier: keeps loads through pinned
// pointer copies global_load / s_load instead of flat.
#define GLOBAL __attribute__((address_space(1)))
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // POD 16-byte vector

// Materialise a wave-uniform value in SGPRs at this point (the compiler may
// neither sink its load below nor recompute it after).
template <class T>
__device__ __forceinline__ void pin(T& v) { asm volatile("" : "+s"(v)); }

__device__ __forceinline__ int rdl(int v, int j) { return __builtin_amdgcn_readlane(v, j); }
__device__ __forceinline__ float rdlf(float v, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// lmask: a lane predicate as a 0 / ~0 word in a vector register, opaque to the
// optimizer: predicates combined this way stay on the vector ALU.  Combined as
// bools they become scalar lane masks, and every vector-compare -> scalar-op
// hand-off costs ~20 cycles of forwarding latency (scripts/exp/probes.py).
__device__ __forceinline__ uint32_t lmask(bool b) {
    uint32_t x = b ? ~0u : 0u;
    asm("" : "+v"(x));
    return x;
}
__device__ __forceinline__ uint32_t vbit(uint64_t m, int lane) { return 0u - (uint32_t)((m >> lane) & 1ull); }
__device__ __forceinline__ float fmask(uint32_t m, float a) { return __uint_as_float(m & __float_as_uint(a)); }
__device__ __forceinline__ float fpick(uint32_t m, float a, float b) {
    return __uint_as_float((m & __float_as_uint(a)) | (~m & __float_as_uint(b)));
}
__device__ __forceinline__ int ipick(uint32_t m, int a, int b) { return (int)((m & (uint32_t)a) | (~m & (uint32_t)b)); }

__device__ __forceinline__ int popc64(uint64_t m) { return __popcll(m); }
__device__ __forceinline__ int ffs64(uint64_t m) { return __ffsll((long long)m) - 1; }
__device__ __forceinline__ uint64_t lanemask_lt() {
    int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// min over the 64 lanes (identity 0xffffffff): DPP row_shr prefix-min inside
// each 16-lane row, then the four row results by readlane.  Wave-uniform.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    // row_shr 1/2/4/8 leave each row's minimum on its lane 15; row_bcast:15
    // and row_bcast:31 carry it across rows, so lane 63 holds the wave's.
    const int id = (int)0xffffffff;
    uint32_t t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x111, 0xf, 0xf, false); v = t < v ? t : v;  // row_shr:1
    t = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x112, 0xf, 0xf, false); v = t < v ? t : v;  // row_shr:2
    t = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x114, 0xf, 0xf, false); v = t < v ? t : v;  // row_shr:4
    t = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x118, 0xf, 0xf, false); v = t < v ? t : v;  // row_shr:8
    t = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x142, 0xa, 0xf, false); v = t < v ? t : v;  // row_bcast:15
    t = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x143, 0xc, 0xf, false); v = t < v ? t : v;  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Two independent wave minima with their DPP stages interleaved: each stage of
// one chain fills the other's DPP read-after-write wait states.
__device__ __forceinline__ void wave_min_u32x2(uint32_t u, uint32_t v, uint32_t& mu, uint32_t& mv) {
    const int id = (int)0xffffffff;
    uint32_t a, b;
#define MDL_MIN2(ctl, rm)                                                                  \
    a = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)u, ctl, rm, 0xf, false);            \
    b = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, ctl, rm, 0xf, false);            \
    u = a < u ? a : u;                                                                     \
    v = b < v ? b : v;
    MDL_MIN2(0x111, 0xf)  // row_shr:1
    MDL_MIN2(0x112, 0xf)  // row_shr:2
    MDL_MIN2(0x114, 0xf)  // row_shr:4
    MDL_MIN2(0x118, 0xf)  // row_shr:8
    MDL_MIN2(0x142, 0xa)  // row_bcast:15
    MDL_MIN2(0x143, 0xc)  // row_bcast:31
#undef MDL_MIN2
    mu = (uint32_t)__builtin_amdgcn_readlane((int)u, 63);
    mv = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Minima over the wave's 64 lanes of eight keys at once (k[a]: agent a's key on every lane) by a
// halving transpose: v_permlane32_swap pairs agent a's upper half-wave with agent a+4's lower one,
// v_permlane16_swap does the same for rows, then one xor-8 exchange and three in-row DPP stages --
// about 20 VALU for all eight instead of eight 6-stage DPP chains, and one chain's latency.
// Agent a's minimum ends on lanes (a >> 1) * 16 + (a & 1) * 8 + [0, 8) (wave_min8_lane(a)).
__device__ __forceinline__ int wave_min8_lane(int a) { return ((a >> 1) << 4) | ((a & 1) << 3); }
__device__ __forceinline__ uint32_t wave_min8_u32(const uint32_t (&k)[8]) {
    uint32_t m[4], n[2];
#pragma unroll
    for (int i = 0; i < 4; i++) {   // lanes 0-31: agent i over lanes l, l+32; lanes 32-63: agent i+4
        const auto r = __builtin_amdgcn_permlane32_swap(k[i], k[i + 4], false, false);
        m[i] = r[0] < r[1] ? r[0] : r[1];
    }
#pragma unroll
    for (int i = 0; i < 2; i++) {   // rows 0..3: agents i, i+2, i+4, i+6, each over 4 lanes
        const auto r = __builtin_amdgcn_permlane16_swap(m[i], m[i + 2], false, false);
        n[i] = r[0] < r[1] ? r[0] : r[1];
    }
    const bool hi = (lane_id() & 8) != 0;   // half-row: keep agent 2r + 1 (n[1]) or 2r (n[0])
    const uint32_t keep = hi ? n[1] : n[0], send = hi ? n[0] : n[1];
    const int id = (int)0xffffffff;
    uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)send, 0x128, 0xf, 0xf, false);   // row_ror:8
    uint32_t v = t < keep ? t : keep;
    t = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x141, 0xf, 0xf, false);   // row_half_mirror
    v = t < v ? t : v;
    t = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x4E, 0xf, 0xf, false);    // quad_perm 2,3,0,1
    v = t < v ? t : v;
    t = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0xB1, 0xf, 0xf, false);    // quad_perm 1,0,3,2
    return t < v ? t : v;
}

// float32(a / b) for an int a and an int b > 0 whose fp64 reciprocal y = RN(1/b)
// is precomputed: RN_f32(RN_f64(a * y)).  Exact (== qdiv) for |a| < 2^24,
// b < 2^24: a*y is within 2^-52 (relative) of a/b, while a/b is either a float
// or at least 2^-49 (relative) away from every float32 rounding boundary
// (a/b = midpoint would need a 25-bit odd significand from a 24-bit a).
// For |a| >= 2^24 it is float32(float64(a)/b), which is what the reference's
// Python-float division followed by the float32 cast computes.
__device__ __forceinline__ float qdiv_r(int a, double y) { return (float)((double)a * y); }

// Correctly rounded int/int division in float32.  For |a|,|b| < 2^24 this
// equals float32(double(a)/double(b)) (double rounding is innocuous for
// division when 53 >= 2*24+2), i.e. what np.array([a/b], float32) stores.
__device__ __forceinline__ float qdiv(int a, int b) { return (float)a / (float)b; }

// i / d for 0 <= i < 2^23 using a float reciprocal and one correction.
__device__ __forceinline__ int fdivi(int i, int d, float inv) {
    int q = (int)((float)i * inv);
    int r = i - q * d;
    if (r < 0) q -= 1;
    else if (r >= d) q += 1;
    return q;
}

__device__ __forceinline__ int cell_r(int pc) { return pc & 255; }
__device__ __forceinline__ int cell_c(int pc) { return (pc >> 8) & 255; }
__device__ __forceinline__ int manhattan(int a, int b) {
    return abs(cell_r(a) - cell_r(b)) + abs(cell_c(a) - cell_c(b));
}
// The same distance in one v_sad_u8 (sum of |byte differences|): valid for
// packed cells (bits 16..31 zero), which every cell word of the step kernel is.
__device__ __forceinline__ int manhattan_sad(int a, int b) {
    return (int)__builtin_amdgcn_sad_u8((uint32_t)a, (uint32_t)b, 0u);
}

__device__ __forceinline__ int pk_start(uint64_t v) { return (int)(v & 0xffff); }
__device__ __forceinline__ int pk_target(uint64_t v) { return (int)((v >> 16) & 0xffff); }
__device__ __forceinline__ int pk_st(uint64_t v) { return (int)((v >> 32) & 0xffff); }
__device__ __forceinline__ int pk_dl(uint64_t v) { return (int)(v >> 48); }
__device__ __forceinline__ uint64_t pk_make(int start, int target, int st, int dl) {
    return (uint64_t)(uint32_t)start | ((uint64_t)(uint32_t)target << 16) | ((uint64_t)(uint32_t)st << 32) |
           ((uint64_t)(uint32_t)dl << 48);
}

// Action decode.  MDL_ACTION_TRAINER_INT: MAPPO/trainer.py:198-205 with the
// LabelEncoder class order D,L,R,S,U; MDL_ACTION_CODES: move | op<<3.
__device__ __forceinline__ void decode_action(int a, int fmt, int& mv, int& op) {
    if (fmt == 0) {
        const int q = a / 5;
        const int m = a - 5 * q;
        // D,L,R,S,U -> codes 4,1,2,0,3
        mv = (0x30214 >> (4 * m)) & 0xf;
        op = q >= 3 ? 0 : q;
    } else {
        mv = a & 7;
        op = (a >> 3) & 3;
        if (mv > MV_OTHER) mv = MV_OTHER;
    }
}

// ------------------------------------------------- numpy legacy RandomState
// MT19937 state lives in the wave's LDS slice while a reset runs.
// Twist: 64 lanes per round; round-ordered so reads of key[i+1] see old
// values and reads of key[i-227] (i >= 227) see new ones, exactly as the
// sequential mt19937_gen.
__device__ inline void mt_twist(uint32_t* key) {
    const int lane = lane_id();
    for (int base = 0; base < MT_N; base += WAVE) {
        const int i = base + lane;
        uint32_t v = 0;
        if (i < MT_N) {
            const uint32_t y = (key[i] & 0x80000000u) | (key[i + 1 == MT_N ? 0 : i + 1] & 0x7fffffffu);
            const int k = i + MT_M < MT_N ? i + MT_M : i + MT_M - MT_N;
            v = key[k] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        wave_sync();
        if (i < MT_N) key[i] = v;
        wave_sync();
    }
}

struct MTState {
    uint32_t* key;  // LDS
    int pos;        // wave-uniform
};

__device__ inline uint32_t mt_next32(MTState& s) {
    if (s.pos == MT_N) {
        mt_twist(s.key);
        s.pos = 0;
    }
    uint32_t y = s.key[s.pos];
    s.pos++;
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return (uint32_t)uni((int)y);
}

// RandomState.randint(lo, hi): hi exclusive; rng==0 -> lo with NO draw;
// masked rejection on 32-bit draws (numpy distributions.c
// buffered_bounded_masked_uint32).  Caller guarantees lo < hi.
__device__ inline int randint(MTState& s, int lo, int hi) {
    const uint32_t rng = (uint32_t)(hi - 1 - lo);
    if (rng == 0) return lo;
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    do {
        v = mt_next32(s) & mask;
    } while (v > rng);
    return lo + (int)v;
}

// ------------------------------------------------------------------ reset
// Environment.reset() (env.py:81-125) for one env, wave-cooperative.
// Writes robots (lane a: packed cell), the sorted package table into pk[]
// (LDS) and initial statuses into pst[] (LDS).  scratch: LDS u64[P] + u16[64].
struct ResetOut {
    int robot_cell;   // lane a < A
};

__device__ inline int reset_env(MTState& mt, const DevParams& p, const MapDesc& md, uint64_t* pk, uint8_t* pst,
                                uint64_t* scratch, uint16_t* taken) {
    const int lane = lane_id();
    const int A = p.A, P = p.P;
    const uint16_t* fl = p.free_cells + md.free_off;
    const int F = md.nfree;
    // robots: get_random_free_cell(tmp_grid) env.py:161-170 -- the k-th
    // not-yet-taken free cell in row-major order.
    int my_cell = 0;
    int ntk = 0;
    for (int i = 0; i < A; i++) {
        const int k = randint(mt, 0, F - i);
        int idx = k;
        for (int q = 0; q < ntk; q++) {
            const int tq = taken[q];
            if (tq <= idx) idx++;
            else break;
        }
        // insert idx into the sorted taken list (one lane shifts)
        if (lane == 0) {
            int q = ntk;
            while (q > 0 && taken[q - 1] > idx) {
                taken[q] = taken[q - 1];
                q--;
            }
            taken[q] = (uint16_t)idx;
        }
        ntk++;
        wave_sync();
        if (lane == i) my_cell = fl[idx];
    }
    // packages env.py:102-117 (draw order: start, target(s), deadline, start_time)
    const int N = md.H;
    const int lim = A < 20 ? A : 20;
    for (int i = 0; i < P; i++) {
        const int s_idx = randint(mt, 0, F);
        int t_idx;
        do {
            t_idx = randint(mt, 0, F);
        } while (t_idx == s_idx);
        const int to_dl = 10 + randint(mt, N / 2, 3 * N);
        const int st = (i <= lim) ? 0 : randint(mt, 1, p.T);
        if (lane == 0) scratch[i] = pk_make(s_idx, t_idx, st, st + to_dl);
    }
    wave_sync();
    for (int j = lane; j < P; j += WAVE) {
        const uint64_t v = scratch[j];
        scratch[j] = pk_make(fl[pk_start(v)], fl[pk_target(v)], pk_st(v), pk_dl(v));
    }
    wave_sync();
    // stable sort by start_time (env.py:119): rank = #(st_i < st_j) + #(i < j, st_i == st_j)
    for (int j0 = 0; j0 < P; j0 += WAVE) {
        const int j = j0 + lane;
        uint64_t v = 0;
        int sj = 0, rank = 0;
        if (j < P) {
            v = scratch[j];
            sj = pk_st(v);
        }
        for (int i = 0; i < P; i++) {
            const int si = pk_st(scratch[i]);
            rank += (si < sj) || (si == sj && i < j);
        }
        if (j < P) {
            pk[rank] = v;
        }
    }
    wave_sync();
    for (int j = lane; j < P; j += WAVE) pst[j] = pk_st(pk[j]) == 0 ? ST_WAITING : ST_NONE;  // get_state at t=0
    wave_sync();
    return my_cell;
}

// ------------------------------------------------------- tracker accessors
// The persistent-package dict (MAPPO/trainer.py:95-130) seen through one
// interface: slot j -> present / in_transit / start / target / start_time /
// deadline / id / iteration order.
struct TrkFresh {  // == env truth: ids in spawn (= id) order
    static constexpr bool kIdIndexed = true;
    const uint64_t* pk;
    const uint8_t* ps;
    int n;
    __device__ int count() const { return n; }
    __device__ bool present(int j) const { const int s = ps[j] & PS_STATUS; return s == ST_WAITING || s == ST_IN_TRANSIT; }
    __device__ bool in_transit(int j) const { return (ps[j] & PS_STATUS) == ST_IN_TRANSIT; }
    __device__ uint64_t data(int j) const { return pk[j]; }
    __device__ int id(int j) const { return j + 1; }
    __device__ uint32_t order(int j) const { return (uint32_t)j; }
    __device__ int slot_of(int id) const { return (id >= 1 && id <= n && present(id - 1)) ? id - 1 : -1; }
};

// Explicit per-id slots, never cleared on auto-reset.  Iteration order:
// survivors of earlier episodes by their rank, then this episode's
// insertions, which happen in id order (spawn order == id order).
struct TrkStale {
    static constexpr bool kIdIndexed = true;
    const uint8_t* ps;
    const uint64_t* td;   // survivor ? trk data : pkg
    const uint32_t* tq;   // survivor ? rank : ORD_EPISODE + slot
    int n;
    __device__ int count() const { return n; }
    __device__ bool present(int j) const { return (ps[j] & PS_PRESENT) != 0; }
    __device__ bool in_transit(int j) const { return (ps[j] & PS_TRANSIT) != 0; }
    __device__ uint64_t data(int j) const { return td[j]; }
    __device__ int id(int j) const { return j + 1; }
    __device__ uint32_t order(int j) const { return tq[j]; }
    __device__ int slot_of(int id) const { return (id >= 1 && id <= n && present(id - 1)) ? id - 1 : -1; }
};

struct TrkView {  // arbitrary dict from a packed view record (dict order)
    static constexpr bool kIdIndexed = false;
    const int32_t* ids;
    const uint8_t* flag;
    const uint64_t* pk;
    int n;
    __device__ int count() const { return n; }
    __device__ bool present(int j) const { return flag[j] & 1; }
    __device__ bool in_transit(int j) const { return (flag[j] & 2) != 0; }
    __device__ uint64_t data(int j) const { return pk[j]; }
    __device__ int id(int j) const { return ids[j]; }
    __device__ uint32_t order(int j) const { return (uint32_t)j; }
    __device__ int slot_of(int id) const {
        for (int j = 0; j < n; j++)
            if (ids[j] == id) return j;
        return -1;
    }
};

// ----------------------------------------------------------- shaped reward
// compute_shaped_rewards (MAPPO/helper.py:257-369) for the agent on this lane.
// float32 accumulation in the reference's order (NEP 50: each constant is
// rounded to float32 first).  Returns this lane's shaped_rewards[a].
template <class Trk>
__device__ inline float shaped_agent(const Trk& trk, const float* C, bool active, int prev_cell, int prev_carry,
                                     int cur_cell, int cur_carry, int mv, int op, int t_prev, int t_cur) {
    float s = 0.0f;
    const int pslot = (active && prev_carry != 0) ? trk.slot_of(prev_carry) : -1;
    // 1. pickup / delivery
    if (prev_carry == 0 && cur_carry != 0) {
        s = s + C[SH_PICK];
    } else if (prev_carry != 0 && cur_carry == 0) {
        if (pslot >= 0) {
            const uint64_t d = trk.data(pslot);
            if (cur_cell == pk_target(d)) s = s + ((t_cur <= pk_dl(d)) ? C[SH_ONTIME] : C[SH_LATE]);
        }
    }
    const bool moved = prev_cell != cur_cell;
    // scan of waiting (st <= t_prev) entries: can_pickup / nearest / idle
    const bool need_can = active && op == 1 && prev_carry == 0 && cur_carry == 0;
    const bool need_near = active && moved && !(prev_carry != 0 && pslot >= 0);
    const bool need_idle = active && !moved && mv == MV_S && prev_carry == 0;
    bool can = false, idle = false;
    int best_d = 0x7fffffff;
    uint32_t best_o = 0xffffffffu;
    int best_cell = -1;
    if (__ballot(need_can || need_near || need_idle)) {
        const int n = trk.count();
        for (int j = 0; j < n; j++) {
            if (!trk.present(j) || trk.in_transit(j)) continue;
            const uint64_t d = trk.data(j);
            if (pk_st(d) > t_prev) continue;
            const int sc = pk_start(d);
            can |= sc == cur_cell;
            const int md = manhattan(prev_cell, sc);
            idle |= md <= 3;
            const uint32_t o = trk.order(j);
            if (md < best_d || (md == best_d && o < best_o)) {
                best_d = md;
                best_o = o;
                best_cell = sc;
            }
        }
    }
    // 2. wasted operations
    if (op == 1) {
        if (prev_carry != 0) s = s + C[SH_WPICK];
        else if (cur_carry == 0 && !can) s = s + C[SH_WPICK];
    } else if (op == 2) {
        if (prev_carry == 0) s = s + C[SH_WDROP];
        else if (cur_carry != 0 && pslot >= 0 && cur_cell != pk_target(trk.data(pslot))) s = s + C[SH_WDROP];
    }
    // 3. movement
    if (mv != MV_S && !moved) s = s + C[SH_STUCK];
    int target = -1;
    if (prev_carry != 0 && pslot >= 0) target = pk_target(trk.data(pslot));
    else target = best_cell;
    if (target >= 0 && moved) {
        const int db = manhattan(prev_cell, target), da = manhattan(cur_cell, target);
        if (da < db) s = s + C[SH_CLOSER];
        else if (da > db) s = s + C[SH_AWAY];
    }
    // 4. idle near an available package
    if (!moved && mv == MV_S && prev_carry == 0 && idle) s = s + C[SH_IDLE];
    return active ? s : 0.0f;
}

// np_sum_lanes for n <= AU (the sequential n < 8 branch, and the 8-partial form at n == 8),
// with the readlanes issued up front.  Lanes n..AU-1 must hold +0.0f.
template <int AU>
__device__ inline float np_sum_lanes8(float v, int n) {
    static_assert(AU >= 1 && AU <= 8, "np_sum_lanes8: 1 <= AU <= 8");
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = i < AU ? rdlf(v, i) : 0.0f;
    float res;
    if (AU == 8 && n == 8) {
        res = ((x[0] + x[1]) + (x[2] + x[3])) + ((x[4] + x[5]) + (x[6] + x[7]));
    } else {
        // lanes n..6 hold +0.0f, and adding +0.0f is exact here (no partial sum
        // is ever -0.0f), so the n-term sequential sum needs no selects
        res = 0.0f;
#pragma unroll
        for (int i = 0; i < (AU < 7 ? AU : 7); i++) res = res + x[i];
    }
    return 0.0f + res;
}

// numpy float32 add.reduce over lanes 0..n-1 (n <= 64): 0 + pairwise_sum
// (8 running partials for n >= 8, sequential tail).  Wave-uniform result.
__device__ inline float np_sum_lanes(float v, int n) {
    float res;
    if (n < 8) {
        res = 0.0f;
        for (int i = 0; i < n; i++) res = res + rdlf(v, i);
    } else {
        float r0 = rdlf(v, 0), r1 = rdlf(v, 1), r2 = rdlf(v, 2), r3 = rdlf(v, 3);
        float r4 = rdlf(v, 4), r5 = rdlf(v, 5), r6 = rdlf(v, 6), r7 = rdlf(v, 7);
        int i;
        for (i = 8; i < n - (n % 8); i += 8) {
            r0 = r0 + rdlf(v, i + 0); r1 = r1 + rdlf(v, i + 1); r2 = r2 + rdlf(v, i + 2); r3 = r3 + rdlf(v, i + 3);
            r4 = r4 + rdlf(v, i + 4); r5 = r5 + rdlf(v, i + 5); r6 = r6 + rdlf(v, i + 6); r7 = r7 + rdlf(v, i + 7);
        }
        res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
        for (; i < n; i++) res = res + rdlf(v, i);
    }
    return 0.0f + res;
}

// np_sum_lanes for n <= AU <= 7 as a DPP chain: lane i adds lane i-1's running sum
// (row_shr:1) to its own value, so lane AU-1 ends with (((0 + x0) + x1) + ...) + x[AU-1]
// in the reference's order (x + y == y + x exactly).  Lanes n..AU-1 must hold +0.0f
// (exact: no partial sum is -0.0f), and no lane may hold -0.0f: then the reference's
// leading and trailing 0.0f + x are identities and are left out.  No readlanes, no
// SGPRs held.
template <int AU>
__device__ inline float np_sum_lanes_dpp(float v) {
    static_assert(AU >= 1 && AU <= 7, "np_sum_lanes_dpp: 1 <= AU <= 7");
    float t = v;
#pragma unroll
    for (int i = 1; i < AU; i++) {
        const float prev = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(t), 0x111, 0xf, 0xf, true));
        t = v + prev;
    }
    return rdlf(t, AU - 1);
}

// np_sum_lanes for exactly 16 values on lanes 0..15 as four DPP adds in numpy's pairwise
// order (n = 16: r_j = x_j + x_{j+8}, then ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), no tail;
// x + y == y + x exactly): row_ror:8, quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_ror:4.
template <int CTL>
__device__ __forceinline__ float dppf(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTL, 0xf, 0xf, true));
}
__device__ inline float np_sum16_dpp(float v) {
    const float r = v + dppf<0x128>(v);   // lane j < 8: x_j + x_{j+8}
    const float s = r + dppf<0xB1>(r);    // even lanes: r_j + r_{j+1}
    const float c = s + dppf<0x4E>(s);    // lanes 0, 4: (r0+r1)+(r2+r3), (r4+r5)+(r6+r7)
    const float d = c + dppf<0x124>(c);   // lane 0: the two halves
    return 0.0f + rdlf(d, 0);
}

// the step kernel's sum: unrolled form for AU > 0 robots, the general one otherwise
// (the step kernel's lane values are sums or masked +0.0f: never -0.0f)
template <int AU>
__device__ inline float np_sum_step(float v, int n) {
    if constexpr (AU > 0 && AU <= 7) return np_sum_lanes_dpp<AU>(v);
    else if constexpr (AU == 16) return np_sum16_dpp(v);   // the exact-A kernel: n == 16
    else if constexpr (AU == 8) return np_sum_lanes8<AU>(v, n);
    else return np_sum_lanes(v, n);
}

}  // namespace mdl
