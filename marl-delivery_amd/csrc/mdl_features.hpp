// mdl_features.hpp -- actor/critic observation builders (MAPPO/helper.py:6-255)
// as wave-cooperative device code shared by the engine's obs kernel and the
// helper-compatible view kernel.
//
// Layout per wave (LDS, carved by feat_carve):
//   robots  rr/rcol/rcarry/rcslot/rcell/rtgt  int32[64] each
//   bits    uint32[5][NW] cell bitsets (NW = ceil(HW/32)): grid, robot, >=2 robots,
//                          waiting start (ch3), active target (ch4)
//   inv_o   uint8 [A][64]   agent a: sorted-other slot -> robot
//   inv_p   uint16[A][MPc]  agent a: sorted-package slot -> tracker slot
//   inv_c   uint16[MPsc]    critic: id-sorted slot -> tracker slot
//   keys    uint64[NS]      per-agent package sort keys
//   scar    int8 [NS]       carrier robot of each slot (-1 none)
//   cnt     int32[A+2]      n_other / n_pkg per agent, n_active
// Values are 0/1 or single int/int divisions, so every output is exact.
#pragma once
#include "mdl_device.hpp"

namespace mdl {

struct FeatDims {
    int A, NS, HW, MPc, MPsc, stage;  // stage: floats of the vector staging slice
};

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

__host__ __device__ inline size_t feat_lds_bytes(const FeatDims& d) {
    size_t s = 0;
    s += align16(sizeof(int32_t) * 64 * 6);
    s += align16(sizeof(uint32_t) * 5 * (size_t)((d.HW + 31) / 32));
    s += align16((size_t)d.A * 64);
    s += align16(sizeof(uint16_t) * (size_t)d.A * (d.MPc > 0 ? d.MPc : 1));
    s += align16(sizeof(uint16_t) * (size_t)(d.MPsc > 0 ? d.MPsc : 1));
    s += align16(sizeof(uint64_t) * (size_t)(d.NS > 0 ? d.NS : 1));
    s += align16((size_t)(d.NS > 0 ? d.NS : 1));
    s += align16(sizeof(int32_t) * (size_t)(d.A + 2));
    s += align16(sizeof(float) * (size_t)(d.stage > 0 ? d.stage : 1));
    return s;
}

struct FeatLds {
    int32_t *rr, *rcol, *rcarry, *rcslot, *rcell, *rtgt;
    uint32_t* bits;   // [5][NW]
    uint8_t* inv_o;
    uint16_t* inv_p;
    uint16_t* inv_c;
    uint64_t* keys;
    int8_t* scar;
    int32_t* cnt;
    float* stage;
};

__device__ inline FeatLds feat_carve(unsigned char* base, const FeatDims& d) {
    FeatLds L;
    size_t o = 0;
    int32_t* r = (int32_t*)(base + o);
    L.rr = r; L.rcol = r + 64; L.rcarry = r + 128; L.rcslot = r + 192; L.rcell = r + 256; L.rtgt = r + 320;
    o += align16(sizeof(int32_t) * 64 * 6);
    L.bits = (uint32_t*)(base + o); o += align16(sizeof(uint32_t) * 5 * (size_t)((d.HW + 31) / 32));
    L.inv_o = (uint8_t*)(base + o); o += align16((size_t)d.A * 64);
    L.inv_p = (uint16_t*)(base + o); o += align16(sizeof(uint16_t) * (size_t)d.A * (d.MPc > 0 ? d.MPc : 1));
    L.inv_c = (uint16_t*)(base + o); o += align16(sizeof(uint16_t) * (size_t)(d.MPsc > 0 ? d.MPsc : 1));
    L.keys = (uint64_t*)(base + o); o += align16(sizeof(uint64_t) * (size_t)(d.NS > 0 ? d.NS : 1));
    L.scar = (int8_t*)(base + o); o += align16((size_t)(d.NS > 0 ? d.NS : 1));
    L.cnt = (int32_t*)(base + o); o += align16(sizeof(int32_t) * (size_t)(d.A + 2));
    L.stage = (float*)(base + o);
    return L;
}

// bitsets 0..3 are the critic map's planes in order (convert_global_state channels)
enum : int { BS_GRID = 0, BS_ROBOT = 1, BS_WSTART = 2, BS_ATARGET = 3, BS_MULTI = 4 };

struct FeatCtx {
    int A, NS, H, W, HW, NW, t, T, MO, MP, MR, MPs, MPc, MPsc;
    const uint32_t* gridbits;  // [NW] obstacle bitset of the map
    const uint16_t* rank;      // [(2H-1)][(2W-1)]
    float inv_hw;
};

__device__ __forceinline__ int rank_of(const FeatCtx& c, int dr, int dc) {
    return c.rank[(dr + c.H - 1) * (2 * c.W - 1) + (dc + c.W - 1)];
}

// Writes n floats value(i) to dst: scalar head to 16-B alignment, float4 body,
// scalar tail; lanes stride the chunks (1 KiB per wave-instruction).
template <class F>
__device__ inline void emit(float* dst, int n, const F& value) {
    const int lane = lane_id();
    const uintptr_t addr = (uintptr_t)dst;
    int head = (int)(((16 - (addr & 15)) & 15) >> 2);
    if (head > n) head = n;
    if (lane < head) dst[lane] = value(lane);
    const int nb = (n - head) >> 2;
    float4* d4 = reinterpret_cast<float4*>(dst + head);
    for (int q = lane; q < nb; q += WAVE) {
        const int i0 = head + 4 * q;
        float4 v;
        v.x = value(i0);
        v.y = value(i0 + 1);
        v.z = value(i0 + 2);
        v.w = value(i0 + 3);
        d4[q] = v;
    }
    const int tail = head + 4 * nb;
    if (tail + lane < n) dst[tail + lane] = value(tail + lane);
}

// Stage robots / cell flags / carriers / critic id order.  Robots come in on
// lanes (lane a < A): cell packed r|c<<8, carry id.
template <class Trk>
__device__ inline void feat_prepare(const Trk& trk, const FeatCtx& c, FeatLds& L, int cell, int carry) {
    const int lane = lane_id();
    const int A = c.A, NS = c.NS, W = c.W, t = c.t;
    if (lane < A) {
        const int r = cell_r(cell), col = cell_c(cell);
        L.rr[lane] = r;
        L.rcol[lane] = col;
        L.rcarry[lane] = carry;
        L.rcell[lane] = r * W + col;
        const int cs = carry != 0 ? trk.slot_of(carry) : -1;
        L.rcslot[lane] = cs;
        int tg = -1;
        if (cs >= 0 && trk.in_transit(cs)) {
            const int tc = pk_target(trk.data(cs));
            tg = cell_r(tc) * W + cell_c(tc);
        }
        L.rtgt[lane] = tg;   // convert_observation channel 5 (MAPPO/helper.py:59-64)
    }
    const int NW = c.NW;
    for (int w = lane; w < NW; w += WAVE) {
        L.bits[BS_GRID * NW + w] = c.gridbits[w];   // host-built obstacle bitset of the map
        L.bits[BS_ROBOT * NW + w] = 0;
        L.bits[BS_MULTI * NW + w] = 0;
        L.bits[BS_WSTART * NW + w] = 0;
        L.bits[BS_ATARGET * NW + w] = 0;
    }
    wave_sync();
    if (lane < A) {
        const int rc = L.rcell[lane];
        const uint32_t m = 1u << (rc & 31);
        const uint32_t old = atomicOr(&L.bits[BS_ROBOT * NW + (rc >> 5)], m);
        if (old & m) atomicOr(&L.bits[BS_MULTI * NW + (rc >> 5)], m);   // a second robot on the cell
    }
    for (int j0 = 0; j0 < NS; j0 += WAVE) {
        const int j = j0 + lane;
        if (j < NS && trk.present(j)) {
            const uint64_t d = trk.data(j);
            const bool it = trk.in_transit(j);
            const bool wt = !it && pk_st(d) <= t;
            const int tg = pk_target(d), sc = pk_start(d);
            if (wt) {
                const int ci = cell_r(sc) * W + cell_c(sc);
                atomicOr(&L.bits[BS_WSTART * NW + (ci >> 5)], 1u << (ci & 31));
            }
            if (wt || it) {
                const int ci = cell_r(tg) * W + cell_c(tg);
                atomicOr(&L.bits[BS_ATARGET * NW + (ci >> 5)], 1u << (ci & 31));
            }
        }
    }
    // carrier of each slot: first robot (index order) carrying its id
    for (int j0 = 0; j0 < NS; j0 += WAVE) {
        const int j = j0 + lane;
        const int idj = j < NS ? trk.id(j) : 0x7fffffff;
        int car = -1;
        for (int i = A - 1; i >= 0; i--)
            if (rdl(carry, i) == idj) car = i;
        if (j < NS) L.scar[j] = (int8_t)car;
    }
    // critic: active slots sorted by id (MAPPO/helper.py:222-227)
    int nact = 0;
    for (int j0 = 0; j0 < NS; j0 += WAVE) {
        const int j = j0 + lane;
        bool act = false;
        int idj = 0;
        if (j < NS && trk.present(j)) {
            const bool it = trk.in_transit(j);
            act = it || pk_st(trk.data(j)) <= t;
            idj = trk.id(j);
        }
        const uint64_t b = ballot(act);
        int pos;
        if (Trk::kIdIndexed) {  // slot j holds id j+1: id order == slot order
            pos = nact + popc64(b & lanemask_lt());
        } else {
            pos = 0;
            for (int k = 0; k < NS; k++) {
                const bool ak = trk.present(k) && (trk.in_transit(k) || pk_st(trk.data(k)) <= t);
                pos += ak && trk.id(k) < idj;
            }
        }
        if (act && pos < c.MPsc) L.inv_c[pos] = (uint16_t)j;
        nact += popc64(b);
    }
    if (lane == 0) L.cnt[A + 1] = nact;
    wave_sync();
}

// Per-agent sort of the other robots (key: fp64 (dr/H)^2+(dc/W)^2 rank, then
// robot order) and of the waiting packages (key: max(0,dl-t), distance rank,
// tracker order) -- the two stable sorts of MAPPO/helper.py:139,158.
template <class Trk>
__device__ inline void feat_sort_agent(const Trk& trk, const FeatCtx& c, FeatLds& L, int a, int cell) {
    const int lane = lane_id();
    const int A = c.A, NS = c.NS, t = c.t;
    const int ra = L.rr[a], ca = L.rcol[a];
    // others: lane o
    {
        const bool valid = lane < A && lane != a;
        int key = 0x7fffffff;
        if (valid) key = (rank_of(c, cell_r(cell) - ra, cell_c(cell) - ca) << 8) | lane;
        int pos = 0;
        for (int o = 0; o < A; o++) pos += rdl(key, o) < key;
        if (valid && pos < c.MO) L.inv_o[a * 64 + pos] = (uint8_t)lane;
        if (lane == 0) L.cnt[a] = A - 1;
    }
    // packages: lanes over slots
    int np = 0;
    for (int j0 = 0; j0 < NS; j0 += WAVE) {
        const int j = j0 + lane;
        uint64_t key = ~0ull;
        if (j < NS && trk.present(j) && !trk.in_transit(j)) {
            const uint64_t d = trk.data(j);
            if (pk_st(d) <= t) {
                int dlc = pk_dl(d) - t;
                if (dlc < 0) dlc = 0;
                if (c.T <= 0) dlc = 0;
                const int sc = pk_start(d);
                key = ((uint64_t)dlc << 48) | ((uint64_t)rank_of(c, cell_r(sc) - ra, cell_c(sc) - ca) << 32) |
                      (uint64_t)trk.order(j);
            }
        }
        if (j < NS) L.keys[j] = key;
        np += popc64(ballot(key != ~0ull));
    }
    wave_sync();
    if (NS <= WAVE) {
        // one chunk: keys stay in registers (lane j)
        uint64_t key = lane < NS ? L.keys[lane] : ~0ull;
        const int want = np < c.MPc ? np : c.MPc;
        if (want <= 8) {
            // selection: the `want` smallest keys by repeated wave minima (keys are unique)
            for (int s = 0; s < want; s++) {
                const uint32_t hi = wave_min_u32((uint32_t)(key >> 32));
                const uint32_t lo = wave_min_u32((uint32_t)(key >> 32) == hi ? (uint32_t)key : 0xffffffffu);
                const bool me = key == (((uint64_t)hi << 32) | lo);
                if (me) {
                    L.inv_p[a * c.MPc + s] = (uint16_t)lane;
                    key = ~0ull;
                }
            }
        } else {
            // counting rank against every other key via readlane
            int pos = 0;
            for (int k = 0; k < NS; k++) {
                const uint64_t kk = (uint64_t)(uint32_t)rdl((int)(uint32_t)key, k) |
                                    ((uint64_t)(uint32_t)rdl((int)(uint32_t)(key >> 32), k) << 32);
                pos += kk < key;
            }
            if (key != ~0ull && pos < c.MPc) L.inv_p[a * c.MPc + pos] = (uint16_t)lane;
        }
    } else {
        for (int j0 = 0; j0 < NS; j0 += WAVE) {
            const int j = j0 + lane;
            const uint64_t key = j < NS ? L.keys[j] : ~0ull;
            int pos = 0;
            for (int k = 0; k < NS; k++) pos += L.keys[k] < key;
            if (key != ~0ull && pos < c.MPc) L.inv_p[a * c.MPc + pos] = (uint16_t)j;
        }
    }
    if (lane == 0) L.cnt[a] = (A - 1) | (np << 8);  // n_other | n_pkg << 8 (np <= 1024 -> use 16 bits)
    wave_sync();
}

// All agents' waiting-package selections at once (engine path: NS <= 64 slots,
// A <= AMAX, and (dlc, rank, order) packed into 32 bits -- the host checks the
// bit budget, DevParams::key32_dsh): the per-slot fields are computed once, the
// A rank-table gathers issue together, and the A selection chains (one wave
// minimum per wanted slot) interleave.  Same order as feat_sort_agent's
// (dlc, rank, order) 64-bit keys.
template <class Trk, int AMAX>
__device__ inline void feat_sort_pkgs_fast(const Trk& trk, const FeatCtx& c, FeatLds& L, int dsh) {
    const int lane = lane_id();
    const int A = c.A, t = c.t;
    bool wv = false;
    int dlc = 0, sr = 0, scc = 0;
    uint32_t ord = 0;
    if (lane < c.NS && trk.present(lane) && !trk.in_transit(lane)) {
        const uint64_t d = trk.data(lane);
        if (pk_st(d) <= t) {
            wv = true;
            dlc = pk_dl(d) - t;
            if (dlc < 0 || c.T <= 0) dlc = 0;
            sr = cell_r(pk_start(d));
            scc = cell_c(pk_start(d));
            ord = trk.order(lane);
        }
    }
    const int np = popc64(ballot(wv));
    const int want = np < c.MPc ? np : c.MPc;
    uint32_t key[AMAX];
#pragma unroll
    for (int a = 0; a < AMAX; a++) {
        const int aa = a < A ? a : 0;
        const int ra = L.rr[aa], ca = L.rcol[aa];
        key[a] = (wv && a < A) ? ((uint32_t)dlc << dsh) | ((uint32_t)rank_of(c, sr - ra, scc - ca) << 11) | ord
                               : 0xffffffffu;
    }
    for (int s = 0; s < want; s++) {
#pragma unroll
        for (int a = 0; a < AMAX; a++) {
            if (a < A) {
                const uint32_t m = wave_min_u32(key[a]);
                if (key[a] == m) {
                    L.inv_p[a * c.MPc + s] = (uint16_t)lane;
                    key[a] = 0xffffffffu;
                }
            }
        }
    }
    if (lane < A) L.cnt[lane] = (A - 1) | (np << 8);
    wave_sync();
}

// The other-robot half of feat_sort_agent (for use beside feat_sort_pkgs_fast).
__device__ inline void feat_sort_others(const FeatCtx& c, FeatLds& L, int a, int cell) {
    const int lane = lane_id();
    const int A = c.A;
    const int ra = L.rr[a], ca = L.rcol[a];
    const bool valid = lane < A && lane != a;
    int key = 0x7fffffff;
    if (valid) key = (rank_of(c, cell_r(cell) - ra, cell_c(cell) - ca) << 8) | lane;
    int pos = 0;
    for (int o = 0; o < A; o++) pos += rdl(key, o) < key;
    if (valid && pos < c.MO) L.inv_o[a * 64 + pos] = (uint8_t)lane;
}

__device__ __forceinline__ float dlc_over_T(int dl, int t, int T) {
    if (T <= 0) return 0.0f;
    int d = dl - t;
    if (d < 0) d = 0;
    return qdiv(d, T);
}

__device__ __forceinline__ uint32_t bits_at(const FeatLds& L, int NW, int set, int cell) {
    return (L.bits[set * NW + (cell >> 5)] >> (cell & 31)) & 1u;
}

__device__ __forceinline__ float4 float4_of_bits(uint32_t b) {
    return make_float4((b & 1u) ? 1.0f : 0.0f, (b & 2u) ? 1.0f : 0.0f, (b & 4u) ? 1.0f : 0.0f,
                       (b & 8u) ? 1.0f : 0.0f);
}

// one-hot of `cell` within the 4 cells starting at c0
__device__ __forceinline__ uint32_t onehot4(int cell, int c0) {
    const unsigned d = (unsigned)(cell - c0);
    return d < 4u ? (1u << d) : 0u;
}

// The 4 actor-map values of plane (agent a, channel ch) at cells c0..c0+3.
__device__ __forceinline__ uint32_t actor_bits4(const FeatLds& L, int NW, int a, int ch, int c0, bool a_valid) {
    const int w = c0 >> 5, sh = c0 & 31;
    const int set = ch == 0 ? BS_GRID : ch == 2 ? BS_ROBOT : ch == 3 ? BS_WSTART : BS_ATARGET;
    const uint32_t wb = (L.bits[set * NW + w] >> sh) & 15u;
    if (ch == 0) return wb;
    if (!a_valid) return 0u;
    const uint32_t own = onehot4(L.rcell[a], c0);
    if (ch == 1) return own;
    if (ch == 2) return (wb & ~own) | ((L.bits[BS_MULTI * NW + w] >> sh) & 15u);
    if (ch == 5) return onehot4(L.rtgt[a], c0);
    return wb;
}

// ---- map outputs from plane words (engine path) ----
// Every output map plane as bit words in LDS: actor plane (a, ch) at word
// (6a + ch) * NW, critic plane ch at (6A + ch) * NW.  Each float4 of the
// outputs is then one LDS word, a shift and four selects.
__host__ __device__ inline int plane_words(int A, int HW) { return (6 * A + 4) * ((HW + 31) / 32); }

__device__ inline void feat_build_planes(const FeatCtx& c, const FeatLds& L, uint32_t* pl) {
    const int lane = lane_id();
    const int NW = c.NW, A = c.A, n = (6 * A + 4) * NW;
    const float inv_nw = 1.0f / (float)NW;
    for (int k = lane; k < n; k += WAVE) {
        const int p = fdivi(k, NW, inv_nw);
        const int w = k - p * NW;
        const int base = w << 5;
        const uint32_t g = L.bits[BS_GRID * NW + w], rb = L.bits[BS_ROBOT * NW + w];
        const uint32_t ws = L.bits[BS_WSTART * NW + w], at = L.bits[BS_ATARGET * NW + w];
        uint32_t v;
        if (p < 6 * A) {
            const int a = p / 6, ch = p - 6 * a;
            const unsigned od = (unsigned)(L.rcell[a] - base), td = (unsigned)(L.rtgt[a] - base);
            const uint32_t ow = od < 32u ? 1u << od : 0u;
            const uint32_t tw = td < 32u ? 1u << td : 0u;   // rtgt = -1: no bit
            const uint32_t oth = (rb & ~ow) | L.bits[BS_MULTI * NW + w];
            v = ch == 0 ? g : ch == 1 ? ow : ch == 2 ? oth : ch == 3 ? ws : ch == 4 ? at : tw;
        } else {
            const int ch = p - 6 * A;
            v = ch == 0 ? g : ch == 1 ? rb : ch == 2 ? ws : at;
        }
        pl[k] = v;
    }
    wave_sync();
}

// Planes [0, np) of pl (HW cells each, HW % 4 == 0) as float4 rows into dst
// (16-B aligned).  The (plane, float4-in-plane) pair of each lane advances by
// a constant per iteration: no division in the loop.
__device__ inline void emit_planes(const uint32_t* pl, int NW, int np, int HW, float* dst) {
    const int lane = lane_id();
    const int qpp = HW >> 2, nq = np * qpp;
    const int dp = WAVE / qpp, dr = WAVE - dp * qpp;
    int p = lane / qpp;
    int r = lane - p * qpp;
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int q = lane; q < nq; q += WAVE) {
        const int c0 = r << 2;
        d4[q] = float4_of_bits((pl[p * NW + (c0 >> 5)] >> (c0 & 31)) & 15u);
        p += dp;
        r += dr;
        if (r >= qpp) {
            r -= qpp;
            p += 1;
        }
    }
}

// All 6A actor planes and the 4 critic planes straight from the five cell bitsets (maps too
// large for prebuilt plane words, e.g. 64x64 with 16 agents): plane by plane (uniform loop),
// float4 q of a plane is the 4 bits at bit 4q of its bit row -- word q/8 at shift 4(q%8), so with
// q = lane + 64k the word is lane/8 + 8k and the shift is fixed per lane (no division per
// float4).  The 4 bits are spread to bytes by one multiply and converted by v_cvt_f32_ubyteN.
// Needs HW % 4 == 0 and 16-B aligned outputs (am / cm may be null).
template <int B>
__device__ __forceinline__ float cvt_ub(uint32_t y) {
    float f;
    if constexpr (B == 0) asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(f) : "v"(y));
    else if constexpr (B == 1) asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(f) : "v"(y));
    else if constexpr (B == 2) asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(f) : "v"(y));
    else asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(f) : "v"(y));
    return f;
}

// One plane of emit_maps_bitrows, its kind fixed at compile time (0 a bit row as is, 1 a one-hot
// of cell `own`, 2 the bit row less `own` plus the multi-robot row), the float4 loop unrolled by
// BITROWS_U: the unrolled group's LDS words are all read before the first is used and its stores
// issue back to back (one kind branch per plane instead of per float4, one LDS wait per group).
template <int KIND>
__device__ __forceinline__ void bitrow_plane(GLOBAL char* base, const uint32_t* row, const uint32_t* mrow, int own,
                                             int qpp, int lane, uint32_t sh) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    constexpr int U = 4;   // float4 stores per unrolled group
    auto put = [&](int q, uint32_t b) {
        const uint32_t y = (b * 0x204081u) & 0x01010101u;   // bit i -> byte i (b < 16: no carries)
        *(GLOBAL f32x4*)(base + ((uint32_t)q << 4)) = f32x4{cvt_ub<0>(y), cvt_ub<1>(y), cvt_ub<2>(y), cvt_ub<3>(y)};
    };
    auto bits = [&](int q, uint32_t r, uint32_t m) -> uint32_t {
        if constexpr (KIND == 1) return onehot4(own, q << 2);
        else if constexpr (KIND == 2) return (__builtin_amdgcn_ubfe(r, sh, 4u) & ~onehot4(own, q << 2)) |
                                             __builtin_amdgcn_ubfe(m, sh, 4u);
        else return __builtin_amdgcn_ubfe(r, sh, 4u);
    };
    int q = lane, k = 0;
    for (; q + (U - 1) * WAVE < qpp; q += U * WAVE, k += 8 * U) {   // uniform (qpp % 64 == 0 for the maps here)
        uint32_t r[U], m[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            r[u] = KIND != 1 ? row[k + 8 * u] : 0u;
            m[u] = KIND == 2 ? mrow[k + 8 * u] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; u++) put(q + u * WAVE, bits(q + u * WAVE, r[u], m[u]));
    }
    for (; q < qpp; q += WAVE, k += 8)
        put(q, bits(q, KIND != 1 ? row[k] : 0u, KIND == 2 ? mrow[k] : 0u));
}

__device__ inline void emit_maps_bitrows(const FeatLds& L, int NW, int HW, int A, float* am, float* cm) {
    const int lane = lane_id();
    const int qpp = HW >> 2;
    const uint32_t sh = (uint32_t)(lane & 7) << 2;
    const int np = 6 * A + 4;
    for (int pl = 0; pl < np; pl++) {   // uniform
        const bool actor = pl < 6 * A;
        const int a = actor ? pl / 6 : 0, ch = actor ? pl - 6 * a : pl - 6 * A;
        float* dst = actor ? (am ? am + (size_t)pl * HW : nullptr) : (cm ? cm + (size_t)ch * HW : nullptr);
        if (!dst) continue;
        // kind: 0 a bit row as is, 1 own-cell one-hot, 2 other robots, 5 carried-target one-hot
        const int kind = actor ? (ch == 1 ? 1 : ch == 2 ? 2 : ch == 5 ? 5 : 0) : 0;
        const int set = actor ? (ch == 0 ? BS_GRID : ch == 2 ? BS_ROBOT : ch == 3 ? BS_WSTART : BS_ATARGET)
                              : (ch == 0 ? BS_GRID : ch == 1 ? BS_ROBOT : ch == 2 ? BS_WSTART : BS_ATARGET);
        const uint32_t* row = L.bits + set * NW + (lane >> 3);
        const uint32_t* mrow = L.bits + BS_MULTI * NW + (lane >> 3);
        GLOBAL char* base = (GLOBAL char*)dst;
        if (kind == 0) bitrow_plane<0>(base, row, mrow, 0, qpp, lane, sh);
        else if (kind == 2) bitrow_plane<2>(base, row, mrow, L.rcell[a], qpp, lane, sh);
        else bitrow_plane<1>(base, row, mrow, kind == 1 ? L.rcell[a] : L.rtgt[a], qpp, lane, sh);
    }
}

// convert_observation for agents [a0, a0+na): dst [na][6][H][W].
// a_valid=false reproduces the early return (channel 0 only).
__device__ inline void emit_actor_maps(const FeatCtx& c, const FeatLds& L, int a0, int na, bool a_valid, float* dst) {
    const int HW = c.HW, NW = c.NW;
    const int lane = lane_id();
    if ((HW & 3) == 0 && (((uintptr_t)dst) & 15) == 0) {
        // float4 per lane, never straddling a plane: 1 KiB per wave store
        const int qpp = HW >> 2;
        const float inv_qpp = 1.0f / (float)qpp;
        const int nq = na * 6 * qpp;
        float4* d4 = reinterpret_cast<float4*>(dst);
        for (int q = lane; q < nq; q += WAVE) {
            const int plane = fdivi(q, qpp, inv_qpp);
            const int c0 = (q - plane * qpp) << 2;
            const int al = plane / 6;
            const int ch = plane - 6 * al;
            d4[q] = float4_of_bits(actor_bits4(L, NW, a0 + al, ch, c0, a_valid));
        }
        return;
    }
    const float inv_hw = c.inv_hw;
    emit(dst, na * 6 * HW, [&](int i) -> float {
        const int plane = fdivi(i, HW, inv_hw);
        const int cell = i - plane * HW;
        const int al = plane / 6;
        const int ch = plane - 6 * al;
        if (ch == 0) return bits_at(L, NW, BS_GRID, cell) ? 1.0f : 0.0f;
        if (!a_valid) return 0.0f;
        const int a = a0 + al;
        const int own = L.rcell[a];
        switch (ch) {
            case 1: return cell == own ? 1.0f : 0.0f;
            case 2: return ((bits_at(L, NW, BS_ROBOT, cell) && cell != own) || bits_at(L, NW, BS_MULTI, cell)) ? 1.0f
                                                                                                                : 0.0f;
            case 3: return bits_at(L, NW, BS_WSTART, cell) ? 1.0f : 0.0f;
            case 4: return bits_at(L, NW, BS_ATARGET, cell) ? 1.0f : 0.0f;
            default: return cell == L.rtgt[a] ? 1.0f : 0.0f;
        }
    });
}

// convert_global_state map: dst [4][H][W] (grid, robots, waiting starts, active targets)
__device__ inline void emit_critic_map(const FeatCtx& c, const FeatLds& L, float* dst) {
    const int HW = c.HW, NW = c.NW;
    const int lane = lane_id();
    if ((HW & 3) == 0 && (((uintptr_t)dst) & 15) == 0) {
        const int qpp = HW >> 2;
        const float inv_qpp = 1.0f / (float)qpp;
        float4* d4 = reinterpret_cast<float4*>(dst);
        for (int q = lane; q < 4 * qpp; q += WAVE) {
            const int ch = fdivi(q, qpp, inv_qpp);
            const int c0 = (q - ch * qpp) << 2;
            const int set = ch == 0 ? BS_GRID : ch == 1 ? BS_ROBOT : ch == 2 ? BS_WSTART : BS_ATARGET;
            d4[q] = float4_of_bits((L.bits[set * NW + (c0 >> 5)] >> (c0 & 31)) & 15u);
        }
        return;
    }
    const float inv_hw = c.inv_hw;
    emit(dst, 4 * HW, [&](int i) -> float {
        const int ch = fdivi(i, HW, inv_hw);
        const int cell = i - ch * HW;
        const int set = ch == 0 ? BS_GRID : ch == 1 ? BS_ROBOT : ch == 2 ? BS_WSTART : BS_ATARGET;
        return bits_at(L, NW, set, cell) ? 1.0f : 0.0f;
    });
}

// Vector outputs are mostly padding.  Every tuple that can be non-zero is
// computed by one lane into a compact staging slice (one lane per robot /
// other-robot slot / package slot, so each value's division runs once and
// lanes do the same kind of work), then the full row is streamed: padding as
// literal zeros, the rest read back from the staging slice.
__host__ __device__ inline int actor_compact_dim(int A, int MO, int MPc) {
    const int MOc = MO < A - 1 ? MO : (A - 1 > 0 ? A - 1 : 0);
    return 6 + 5 * MOc + 5 * MPc + 1;
}
__host__ __device__ inline int critic_compact_dim(int A, int MR, int MPsc) {
    return 6 * (A < MR ? A : MR) + 7 * MPsc + 1;
}
// agents whose compact actor rows are staged together (<= STAGE_FLOATS floats, >= 1 agent).
// The staging slice is most of the general builder's LDS per wave (config 5: 16 agents x 182 floats),
// and that LDS sets its occupancy: 512 floats (2 agents there) leave the critic row as the largest
// staged item (797 floats) and take the slice from 17.1 to 12.3 KB per wave.
constexpr int STAGE_FLOATS = 512;
__host__ __device__ inline int actor_group(int na, int Dc) {
    const int g = STAGE_FLOATS / Dc;
    return g < 1 ? 1 : (g < na ? g : na);
}

// generate_vector_features (MAPPO/helper.py:68-165): tuple `slot` of agent a
// into out (compact layout [6 self][5*MOc others][5*MPc packages][1 time]).
template <class Trk>
__device__ inline void actor_tuple(const Trk& trk, const FeatCtx& c, const FeatLds& L, int a, int kind, int s,
                                   int MOc, float* out) {
    const int H = c.H, W = c.W, t = c.t, T = c.T;
    const int ra = L.rr[a], ca = L.rcol[a];
    if (kind == 0) {  // self: my_r/H, my_c/W, carrying, (tr-my_r)/H, (tc-my_c)/W, max(0,dl-t)/T ; and t/T
        const int cy = L.rcarry[a], cs = L.rcslot[a];
        float v3 = 0.0f, v4 = 0.0f, v5 = 0.0f;
        if (cy != 0 && cs >= 0 && trk.in_transit(cs)) {
            const uint64_t d = trk.data(cs);
            const int tg = pk_target(d);
            v3 = qdiv(cell_r(tg) - ra, H);
            v4 = qdiv(cell_c(tg) - ca, W);
            v5 = dlc_over_T(pk_dl(d), t, T);
        }
        out[0] = qdiv(ra, H);
        out[1] = qdiv(ca, W);
        out[2] = cy != 0 ? 1.0f : 0.0f;
        out[3] = v3;
        out[4] = v4;
        out[5] = v5;
        out[6 + 5 * MOc + 5 * c.MPc] = T > 0 ? qdiv(t, T) : 0.0f;
    } else if (kind == 1) {  // s-th nearest other robot
        float* o5 = out + 6 + 5 * s;
        if (s >= (L.cnt[a] & 0xff)) {
            o5[0] = o5[1] = o5[2] = o5[3] = o5[4] = 0.0f;
            return;
        }
        const int o = L.inv_o[a * 64 + s];
        const int ro = L.rr[o], co = L.rcol[o];
        const int cy = L.rcarry[o], cs = L.rcslot[o];
        float v3 = 0.0f, v4 = 0.0f;
        if (cy != 0 && cs >= 0 && trk.in_transit(cs)) {
            const int tg = pk_target(trk.data(cs));
            v3 = qdiv(cell_r(tg) - ro, H);
            v4 = qdiv(cell_c(tg) - co, W);
        }
        o5[0] = qdiv(ro - ra, H);
        o5[1] = qdiv(co - ca, W);
        o5[2] = cy != 0 ? 1.0f : 0.0f;
        o5[3] = v3;
        o5[4] = v4;
    } else {  // s-th waiting package in (deadline, distance, order) order
        float* o5 = out + 6 + 5 * MOc + 5 * s;
        if (s >= (L.cnt[a] >> 8)) {
            o5[0] = o5[1] = o5[2] = o5[3] = o5[4] = 0.0f;
            return;
        }
        const uint64_t d = trk.data(L.inv_p[a * c.MPc + s]);
        const int sc = pk_start(d), tg = pk_target(d);
        o5[0] = qdiv(cell_r(sc) - ra, H);
        o5[1] = qdiv(cell_c(sc) - ca, W);
        o5[2] = qdiv(cell_r(tg) - ra, H);
        o5[3] = qdiv(cell_c(tg) - ca, W);
        o5[4] = dlc_over_T(pk_dl(d), t, T);
    }
}

// generate_vector_features for agents [a0, a0+na): dst [na][6+5MO+5MP+1]
template <class Trk>
__device__ inline void emit_actor_vecs(const Trk& trk, const FeatCtx& c, const FeatLds& L, int a0, int na,
                                       bool a_valid, float* dst) {
    const int lane = lane_id();
    const int Dv = 6 + 5 * c.MO + 5 * c.MP + 1;
    if (!a_valid) {
        emit(dst, na * Dv, [](int) -> float { return 0.0f; });
        return;
    }
    const int MOc = c.MO < c.A - 1 ? c.MO : (c.A - 1 > 0 ? c.A - 1 : 0);
    const int o_c = 6 + 5 * MOc, p_c = o_c + 5 * c.MPc;   // compact section ends
    const int Dc = p_c + 1;
    const int o_end = 6 + 5 * c.MO, p_end = o_end + 5 * c.MP;
    const int tpa = 1 + MOc + c.MPc;                        // tuples per agent
    const float inv_tpa = 1.0f / (float)tpa, inv_dv = 1.0f / (float)Dv;
    const int G = actor_group(na, Dc);
    for (int g0 = 0; g0 < na; g0 += G) {
        const int ng = na - g0 < G ? na - g0 : G;
        for (int ti = lane; ti < ng * tpa; ti += WAVE) {
            const int al = fdivi(ti, tpa, inv_tpa);
            const int k = ti - al * tpa;
            const int kind = k == 0 ? 0 : (k <= MOc ? 1 : 2);
            const int slot = kind == 1 ? k - 1 : k - 1 - MOc;
            actor_tuple(trk, c, L, a0 + g0 + al, kind, slot, MOc, L.stage + al * Dc);
        }
        wave_sync();
        emit(dst + (size_t)g0 * Dv, ng * Dv, [&](int i) -> float {
            const int al = fdivi(i, Dv, inv_dv);
            const int f = i - al * Dv;
            int cf;
            if (f < o_c) cf = f;
            else if (f < o_end) return 0.0f;
            else if (f < o_end + 5 * c.MPc) cf = o_c + (f - o_end);
            else if (f < p_end) return 0.0f;
            else cf = Dc - 1;
            return L.stage[al * Dc + cf];
        });
        wave_sync();
    }
}

// convert_global_state vector: dst [6MR+7MPs+1] (MAPPO/helper.py:199-255)
template <class Trk>
__device__ inline void emit_critic_vec(const Trk& trk, const FeatCtx& c, const FeatLds& L, float* dst) {
    const int lane = lane_id();
    const int H = c.H, W = c.W, t = c.t, T = c.T, MR = c.MR;
    const int Dg = 6 * MR + 7 * c.MPs + 1;
    const int r_end = 6 * MR, p_end = r_end + 7 * c.MPs;
    const int nact = L.cnt[c.A + 1];
    const int nr = c.A < MR ? c.A : MR;                 // robot rows present
    const int np = nact < c.MPsc ? nact : c.MPsc;       // package rows present
    const int r_c = 6 * nr, p_c = r_c + 7 * np;
    for (int ti = lane; ti < nr + np + 1; ti += WAVE) {
        if (ti < nr) {  // robot row: r/H, c/W, carrying, tr/H, tc/W, max(0,dl-t)/T
            const int cy = L.rcarry[ti], cs = L.rcslot[ti];
            float v3 = 0.0f, v4 = 0.0f, v5 = 0.0f;
            if (cy != 0 && cs >= 0 && trk.in_transit(cs)) {
                const uint64_t d = trk.data(cs);
                const int tg = pk_target(d);
                v3 = qdiv(cell_r(tg), H);
                v4 = qdiv(cell_c(tg), W);
                v5 = dlc_over_T(pk_dl(d), t, T);
            }
            float* o = L.stage + 6 * ti;
            o[0] = qdiv(L.rr[ti], H);
            o[1] = qdiv(L.rcol[ti], W);
            o[2] = cy != 0 ? 1.0f : 0.0f;
            o[3] = v3;
            o[4] = v4;
            o[5] = v5;
        } else if (ti < nr + np) {  // active package row (id order)
            const int s = ti - nr;
            const int j = L.inv_c[s];
            const uint64_t d = trk.data(j);
            const bool waiting = !trk.in_transit(j);
            const int sc = pk_start(d), tg = pk_target(d);
            float carrier = -1.0f;
            if (!waiting) {
                const int car = L.scar[j];
                if (car >= 0) carrier = MR > 1 ? qdiv(car, MR - 1) : 0.0f;
            }
            float* o = L.stage + r_c + 7 * s;
            o[0] = waiting ? qdiv(cell_r(sc), H) : 0.0f;
            o[1] = waiting ? qdiv(cell_c(sc), W) : 0.0f;
            o[2] = qdiv(cell_r(tg), H);
            o[3] = qdiv(cell_c(tg), W);
            o[4] = dlc_over_T(pk_dl(d), t, T);
            o[5] = waiting ? 0.0f : 1.0f;
            o[6] = carrier;
        } else {
            L.stage[p_c] = T > 0 ? qdiv(t, T) : 0.0f;
        }
    }
    wave_sync();
    emit(dst, Dg, [&](int f) -> float {
        int cf;
        if (f < r_c) cf = f;
        else if (f < r_end) return 0.0f;
        else if (f < r_end + 7 * np) cf = r_c + (f - r_end);
        else if (f < p_end) return 0.0f;
        else cf = p_c;
        return L.stage[cf];
    });
    wave_sync();
}

}  // namespace mdl
