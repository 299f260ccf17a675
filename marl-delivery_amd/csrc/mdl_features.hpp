// mdl_features.hpp -- actor/critic observation builders (MAPPO/helper.py:6-255)
// as wave-cooperative device code shared by the engine's obs kernel and the
// helper-compatible view kernel.
//
// Layout per wave (LDS, carved by feat_carve):
//   robots  rr/rcol/rcarry/rcslot/rcell/rtgt  int32[64] each
//   cellf   uint32[HW]   bit0 grid, bit1 wstart, bit2 atarget, bits 8.. robot count
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
    int A, NS, HW, MPc, MPsc;
};

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

__host__ __device__ inline size_t feat_lds_bytes(const FeatDims& d) {
    size_t s = 0;
    s += align16(sizeof(int32_t) * 64 * 6);
    s += align16(sizeof(uint32_t) * (size_t)d.HW);
    s += align16((size_t)d.A * 64);
    s += align16(sizeof(uint16_t) * (size_t)d.A * (d.MPc > 0 ? d.MPc : 1));
    s += align16(sizeof(uint16_t) * (size_t)(d.MPsc > 0 ? d.MPsc : 1));
    s += align16(sizeof(uint64_t) * (size_t)(d.NS > 0 ? d.NS : 1));
    s += align16((size_t)(d.NS > 0 ? d.NS : 1));
    s += align16(sizeof(int32_t) * (size_t)(d.A + 2));
    return s;
}

struct FeatLds {
    int32_t *rr, *rcol, *rcarry, *rcslot, *rcell, *rtgt;
    uint32_t* cellf;
    uint8_t* inv_o;
    uint16_t* inv_p;
    uint16_t* inv_c;
    uint64_t* keys;
    int8_t* scar;
    int32_t* cnt;
};

__device__ inline FeatLds feat_carve(unsigned char* base, const FeatDims& d) {
    FeatLds L;
    size_t o = 0;
    int32_t* r = (int32_t*)(base + o);
    L.rr = r; L.rcol = r + 64; L.rcarry = r + 128; L.rcslot = r + 192; L.rcell = r + 256; L.rtgt = r + 320;
    o += align16(sizeof(int32_t) * 64 * 6);
    L.cellf = (uint32_t*)(base + o); o += align16(sizeof(uint32_t) * (size_t)d.HW);
    L.inv_o = (uint8_t*)(base + o); o += align16((size_t)d.A * 64);
    L.inv_p = (uint16_t*)(base + o); o += align16(sizeof(uint16_t) * (size_t)d.A * (d.MPc > 0 ? d.MPc : 1));
    L.inv_c = (uint16_t*)(base + o); o += align16(sizeof(uint16_t) * (size_t)(d.MPsc > 0 ? d.MPsc : 1));
    L.keys = (uint64_t*)(base + o); o += align16(sizeof(uint64_t) * (size_t)(d.NS > 0 ? d.NS : 1));
    L.scar = (int8_t*)(base + o); o += align16((size_t)(d.NS > 0 ? d.NS : 1));
    L.cnt = (int32_t*)(base + o);
    return L;
}

struct FeatCtx {
    int A, NS, H, W, HW, t, T, MO, MP, MR, MPs, MPc, MPsc;
    const uint8_t* grid;
    const uint16_t* rank;   // [(2H-1)][(2W-1)]
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
    const int A = c.A, NS = c.NS, HW = c.HW, W = c.W, t = c.t;
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
    for (int i = lane; i < HW; i += WAVE) L.cellf[i] = c.grid[i] ? 1u : 0u;
    wave_sync();
    if (lane < A) atomicAdd(&L.cellf[L.rcell[lane]], 256u);
    for (int j0 = 0; j0 < NS; j0 += WAVE) {
        const int j = j0 + lane;
        if (j < NS && trk.present(j)) {
            const uint64_t d = trk.data(j);
            const bool it = trk.in_transit(j);
            const bool wt = !it && pk_st(d) <= t;
            const int tg = pk_target(d), sc = pk_start(d);
            if (wt) atomicOr(&L.cellf[cell_r(sc) * W + cell_c(sc)], 2u);
            if (wt || it) atomicOr(&L.cellf[cell_r(tg) * W + cell_c(tg)], 4u);
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
        int pos = 0;
        for (int k = 0; k < NS; k++) {
            const bool ak = trk.present(k) && (trk.in_transit(k) || pk_st(trk.data(k)) <= t);
            pos += ak && trk.id(k) < idj;
        }
        if (act && pos < c.MPsc) L.inv_c[pos] = (uint16_t)j;
        nact += popc64(ballot(act));
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
    for (int j0 = 0; j0 < NS; j0 += WAVE) {
        const int j = j0 + lane;
        const uint64_t key = j < NS ? L.keys[j] : ~0ull;
        int pos = 0;
        for (int k = 0; k < NS; k++) pos += L.keys[k] < key;
        if (key != ~0ull && pos < c.MPc) L.inv_p[a * c.MPc + pos] = (uint16_t)j;
    }
    if (lane == 0) L.cnt[a] = (A - 1) | (np << 8);  // n_other | n_pkg << 8 (np <= 1024 -> use 16 bits)
    wave_sync();
}

__device__ __forceinline__ float dlc_over_T(int dl, int t, int T) {
    if (T <= 0) return 0.0f;
    int d = dl - t;
    if (d < 0) d = 0;
    return qdiv(d, T);
}

// convert_observation for agents [a0, a0+na): dst [na][6][H][W].
// a_valid=false reproduces the early return (channel 0 only).
__device__ inline void emit_actor_maps(const FeatCtx& c, const FeatLds& L, int a0, int na,
                                       bool a_valid, float* dst) {
    const int HW = c.HW;
    const float inv_hw = c.inv_hw;
    emit(dst, na * 6 * HW, [&](int i) -> float {
        const int plane = fdivi(i, HW, inv_hw);
        const int cell = i - plane * HW;
        const int al = plane / 6;
        const int ch = plane - 6 * al;
        const uint32_t f = L.cellf[cell];
        if (ch == 0) return (f & 1u) ? 1.0f : 0.0f;
        if (!a_valid) return 0.0f;
        const int a = a0 + al;
        const int own = L.rcell[a];
        switch (ch) {
            case 1: return cell == own ? 1.0f : 0.0f;
            case 2: return ((f >> 8) - (cell == own ? 1u : 0u)) > 0u ? 1.0f : 0.0f;
            case 3: return (f & 2u) ? 1.0f : 0.0f;
            case 4: return (f & 4u) ? 1.0f : 0.0f;
            default: return cell == L.rtgt[a] ? 1.0f : 0.0f;
        }
    });
}

// convert_global_state map: dst [4][H][W]
__device__ inline void emit_critic_map(const FeatCtx& c, const FeatLds& L, float* dst) {
    const int HW = c.HW;
    const float inv_hw = c.inv_hw;
    emit(dst, 4 * HW, [&](int i) -> float {
        const int ch = fdivi(i, HW, inv_hw);
        const uint32_t f = L.cellf[i - ch * HW];
        switch (ch) {
            case 0: return (f & 1u) ? 1.0f : 0.0f;
            case 1: return (f >> 8) ? 1.0f : 0.0f;
            case 2: return (f & 2u) ? 1.0f : 0.0f;
            default: return (f & 4u) ? 1.0f : 0.0f;
        }
    });
}

// generate_vector_features for agents [a0, a0+na): dst [na][6+5MO+5MP+1]
template <class Trk>
__device__ inline void emit_actor_vecs(const Trk& trk, const FeatCtx& c, const FeatLds& L, int a0, int na,
                                       bool a_valid, float* dst) {
    const int Dv = 6 + 5 * c.MO + 5 * c.MP + 1;
    const float inv_dv = 1.0f / (float)Dv;
    const int H = c.H, W = c.W, t = c.t, T = c.T;
    const int o_end = 6 + 5 * c.MO, p_end = o_end + 5 * c.MP;
    emit(dst, na * Dv, [&](int i) -> float {
        if (!a_valid) return 0.0f;
        const int al = fdivi(i, Dv, inv_dv);
        const int f = i - al * Dv;
        const int a = a0 + al;
        const int ra = L.rr[a], ca = L.rcol[a];
        if (f < 6) {
            if (f == 0) return qdiv(ra, H);
            if (f == 1) return qdiv(ca, W);
            const int cy = L.rcarry[a];
            if (f == 2) return cy != 0 ? 1.0f : 0.0f;
            const int cs = L.rcslot[a];
            if (cy == 0 || cs < 0 || !trk.in_transit(cs)) return 0.0f;
            const uint64_t d = trk.data(cs);
            const int tg = pk_target(d);
            if (f == 3) return qdiv(cell_r(tg) - ra, H);
            if (f == 4) return qdiv(cell_c(tg) - ca, W);
            return dlc_over_T(pk_dl(d), t, T);
        }
        if (f < o_end) {
            const int s = fdivi(f - 6, 5, 0.2f);
            const int k = f - 6 - 5 * s;
            const int cnt = L.cnt[a];
            if (s >= (cnt & 0xff)) return 0.0f;
            const int o = L.inv_o[a * 64 + s];
            const int ro = L.rr[o], co = L.rcol[o];
            if (k == 0) return qdiv(ro - ra, H);
            if (k == 1) return qdiv(co - ca, W);
            const int cy = L.rcarry[o];
            if (k == 2) return cy != 0 ? 1.0f : 0.0f;
            const int cs = L.rcslot[o];
            if (cy == 0 || cs < 0 || !trk.in_transit(cs)) return 0.0f;
            const int tg = pk_target(trk.data(cs));
            if (k == 3) return qdiv(cell_r(tg) - ro, H);
            return qdiv(cell_c(tg) - co, W);
        }
        if (f < p_end) {
            const int s = fdivi(f - o_end, 5, 0.2f);
            const int k = f - o_end - 5 * s;
            const int npk = L.cnt[a] >> 8;
            if (s >= npk || s >= c.MPc) return 0.0f;
            const int j = L.inv_p[a * c.MPc + s];
            const uint64_t d = trk.data(j);
            const int sc = pk_start(d), tg = pk_target(d);
            switch (k) {
                case 0: return qdiv(cell_r(sc) - ra, H);
                case 1: return qdiv(cell_c(sc) - ca, W);
                case 2: return qdiv(cell_r(tg) - ra, H);
                case 3: return qdiv(cell_c(tg) - ca, W);
                default: return dlc_over_T(pk_dl(d), t, T);
            }
        }
        return T > 0 ? qdiv(t, T) : 0.0f;
    });
}

// convert_global_state vector: dst [6MR+7MPs+1]
template <class Trk>
__device__ inline void emit_critic_vec(const Trk& trk, const FeatCtx& c, const FeatLds& L, float* dst) {
    const int Dg = 6 * c.MR + 7 * c.MPs + 1;
    const int H = c.H, W = c.W, t = c.t, T = c.T, A = c.A, MR = c.MR;
    const int r_end = 6 * MR, p_end = r_end + 7 * c.MPs;
    const int nact = L.cnt[A + 1];
    emit(dst, Dg, [&](int f) -> float {
        if (f < r_end) {
            const int i = fdivi(f, 6, 1.0f / 6.0f);
            const int k = f - 6 * i;
            if (i >= A) return 0.0f;
            if (k == 0) return qdiv(L.rr[i], H);
            if (k == 1) return qdiv(L.rcol[i], W);
            const int cy = L.rcarry[i];
            if (k == 2) return cy != 0 ? 1.0f : 0.0f;
            const int cs = L.rcslot[i];
            if (cy == 0 || cs < 0 || !trk.in_transit(cs)) return 0.0f;
            const uint64_t d = trk.data(cs);
            const int tg = pk_target(d);
            if (k == 3) return qdiv(cell_r(tg), H);
            if (k == 4) return qdiv(cell_c(tg), W);
            return dlc_over_T(pk_dl(d), t, T);
        }
        if (f < p_end) {
            const int s = fdivi(f - r_end, 7, 1.0f / 7.0f);
            const int k = f - r_end - 7 * s;
            if (s >= nact || s >= c.MPsc) return 0.0f;
            const int j = L.inv_c[s];
            const uint64_t d = trk.data(j);
            const bool waiting = !trk.in_transit(j);
            const int sc = pk_start(d), tg = pk_target(d);
            switch (k) {
                case 0: return waiting ? qdiv(cell_r(sc), H) : 0.0f;
                case 1: return waiting ? qdiv(cell_c(sc), W) : 0.0f;
                case 2: return qdiv(cell_r(tg), H);
                case 3: return qdiv(cell_c(tg), W);
                case 4: return dlc_over_T(pk_dl(d), t, T);
                case 5: return waiting ? 0.0f : 1.0f;
                default: {
                    if (waiting) return -1.0f;
                    const int car = L.scar[j];
                    if (car < 0) return -1.0f;
                    return MR > 1 ? qdiv(car, MR - 1) : 0.0f;
                }
            }
        }
        return T > 0 ? qdiv(t, T) : 0.0f;
    });
}

}  // namespace mdl
