// mdl_altfeat.hpp -- the IDQ / qmix featurizers and IDQ's per-agent reward
// shaping, device side:
//   alt_emit_idq    convert_state              IDQ/networks.py:112-217 (qmix/networks.py:243-348 is the same code)
//   alt_emit_qmix   convert_global_state_to_tensor           qmix/networks.py:350-468
//   idq_reward      reward_shaping                           IDQ/networks.py:228-349
// One wave per state; per-cell scratch in the wave's LDS slice.
#pragma once
#include "mdl_features.hpp"

namespace mdl {

struct AltLds {
    uint8_t* rob;    // [HW] robot index | 0x40 if carrying; 0xff = none (robots stand on distinct cells)
    float* urg;      // [HW] max urgency of waiting, started packages whose start is here; -1 = none
    uint8_t* wt;     // [HW] a waiting, started package targets this cell
    uint8_t* tt;     // [HW] an in-transit, started package targets this cell
    uint32_t* bits;  // [ALT_NBS][NW] the same cell sets as bitsets (alt_emit_fast)
};

// bitsets of alt_emit_fast: obstacles, robots, carrying robots, waiting starts (urgency
// >= 0), waiting targets, in-transit targets
enum : int { ABS_GRID = 0, ABS_ROB, ABS_CARRY, ABS_START, ABS_WT, ABS_TT, ALT_NBS };

__host__ __device__ inline size_t alt_lds_bytes(int HW) {
    const size_t NW = ((size_t)HW + 31) / 32;
    return align16((size_t)HW) + align16(4 * (size_t)HW) + 2 * align16((size_t)HW) + align16(4 * ALT_NBS * NW);
}

__device__ inline AltLds alt_carve(unsigned char* b, int HW) {
    AltLds L;
    size_t o = 0;
    L.rob = b + o; o += align16((size_t)HW);
    L.urg = (float*)(b + o); o += align16(4 * (size_t)HW);
    L.wt = b + o; o += align16((size_t)HW);
    L.tt = b + o; o += align16((size_t)HW);
    L.bits = (uint32_t*)(b + o);
    return L;
}

// urgency = min(1, max(0, (t-st)/(dl-st))) if dl > st; 1 if dl == st (t >= st holds here); else 0.
// The reference divides in double and stores the max into a float32 array: float32 rounding is
// monotone, so the max of correctly rounded float32 quotients is the same value.
__device__ __forceinline__ float alt_urgency(int t, int st, int dl) {
    if (dl > st) {
        const float u = qdiv(t - st, dl - st);
        return u > 1.0f ? 1.0f : (u < 0.0f ? 0.0f : u);
    }
    return dl == st ? 1.0f : 0.0f;
}

template <class Trk>
__device__ inline void alt_prepare(const Trk& trk, int HW, int W, int A, int t, int cell, int carry, AltLds L) {
    const int lane = lane_id();
    for (int i = lane; i < HW; i += WAVE) {
        L.rob[i] = 0xff;
        L.urg[i] = -1.0f;
        L.wt[i] = 0;
        L.tt[i] = 0;
    }
    wave_sync();
    if (lane < A) L.rob[cell_r(cell) * W + cell_c(cell)] = (uint8_t)(lane | (carry ? 0x40 : 0));
    for (int j = lane; j < trk.count(); j += WAVE) {
        if (!trk.present(j)) continue;
        const uint64_t d = trk.data(j);
        const int st = pk_st(d);
        if (!(t >= st)) continue;
        const int sc = pk_start(d), tg = pk_target(d);
        const int si = cell_r(sc) * W + cell_c(sc), ti = cell_r(tg) * W + cell_c(tg);
        if (!trk.in_transit(j)) {
            // urgencies are >= 0, so their float bits order like ints (above -1.0f's)
            atomicMax((int*)&L.urg[si], __float_as_int(alt_urgency(t, st, pk_dl(d))));
            L.wt[ti] = 1;
        } else {
            L.tt[ti] = 1;
        }
    }
    wave_sync();
}

// The cell sets of alt_prepare as bitsets (two words per 64 cells, by ballot).
__device__ inline void alt_bits(const uint32_t* gridbits, int HW, const AltLds& L) {
    const int lane = lane_id();
    const int NW = (HW + 31) >> 5;
    for (int c0 = 0; c0 < HW; c0 += WAVE) {
        const int c = c0 + lane;
        const bool in = c < HW;
        const uint32_t rb = in ? L.rob[c] : 0xffu;
        const float u = in ? L.urg[c] : -1.0f;
        const uint64_t b[ALT_NBS - 1] = {ballot(rb != 0xffu), ballot(rb != 0xffu && (rb & 0x40u)), ballot(u >= 0.0f),
                                         ballot(in && L.wt[c]), ballot(in && L.tt[c])};
        const int wd = c0 >> 5;
#pragma unroll
        for (int k = 0; k < ALT_NBS - 1; k++) {
            // lane 2k / 2k+1 store the low / high word of set k
            const uint32_t v = (lane & 1) ? (uint32_t)(b[k] >> 32) : (uint32_t)b[k];
            if ((lane >> 1) == k && wd + (lane & 1) < NW) L.bits[(k + 1) * NW + wd + (lane & 1)] = v;
        }
    }
    for (int k = lane; k < NW; k += WAVE) L.bits[ABS_GRID * NW + k] = gridbits[k];
    wave_sync();
}

// Fast emission (HW % 4 == 0, 16-B aligned outputs, qmix state shape == map shape): every
// output plane is written as float4s, float4 q of a plane being the 4 cells at 4q -- with
// q = lane + 64k the bitset word is lane/8 + 8k at the fixed shift (lane%8)*4 -- so an
// element costs a shift, a mask and a convert instead of a division and a branch.
__device__ __forceinline__ float4 nib4(uint32_t nib) {
    return make_float4((float)(nib & 1u), (float)((nib >> 1) & 1u), (float)((nib >> 2) & 1u), (float)(nib >> 3));
}
__device__ __forceinline__ uint32_t onehot_nib(int idx, int c0) {
    const unsigned d = (unsigned)(idx - c0);
    return d < 4u ? 1u << d : 0u;
}

// plane kinds: a bitset (or an agent-relative set), or the urgency floats
enum : int { AP_GRID, AP_URG, AP_START, AP_OTHERS, AP_SELF, AP_TGT, AP_ROB, AP_CARRY, AP_WT, AP_TT, AP_ZERO };

__device__ inline void alt_emit_plane(const AltLds& L, int NW, int HW, int kind, int self, int tgt, float* dst) {
    const int lane = lane_id();
    const int nq = HW >> 2;
    const uint32_t sh = (uint32_t)(lane & 7) << 2;
    float4* d4 = reinterpret_cast<float4*>(dst);
    if (kind == AP_URG) {
        const float4* u4 = reinterpret_cast<const float4*>(L.urg);
        for (int q = lane; q < nq; q += WAVE) {
            const float4 u = u4[q];   // -1 = no package: 0
            d4[q] = make_float4(fmaxf(u.x, 0.0f), fmaxf(u.y, 0.0f), fmaxf(u.z, 0.0f), fmaxf(u.w, 0.0f));
        }
        return;
    }
    const int bs = kind == AP_GRID ? ABS_GRID : kind == AP_START ? ABS_START : kind == AP_CARRY ? ABS_CARRY
                 : kind == AP_WT ? ABS_WT : kind == AP_TT ? ABS_TT : ABS_ROB;
    const uint32_t* src = L.bits + bs * NW + (lane >> 3);
    for (int q = lane; q < nq; q += WAVE, src += 8) {
        const int c0 = q << 2;
        uint32_t nib = (*src >> sh) & 15u;
        const uint32_t so = onehot_nib(self, c0);
        nib = kind == AP_OTHERS ? nib & ~so : kind == AP_SELF ? so : kind == AP_TGT ? onehot_nib(tgt, c0)
            : kind == AP_ZERO ? 0u : nib;
        d4[q] = nib4(nib);
    }
}

template <class Trk>
__device__ inline void alt_emit_fast(const Trk& trk, int H, int W, const AltLds& L, int cell, int carry, int A,
                                     float* idq, float* qst) {
    const int HW = H * W, NW = (HW + 31) >> 5;
    if (idq) {
        for (int a = 0; a < A; a++) {
            const int ca = rdl(cell, a), ka = rdl(carry, a);
            const int self = cell_r(ca) * W + cell_c(ca);
            int tgt5 = -1;  // carried package's target, when the id is in the tracker
            if (ka != 0) {
                const int sl = trk.slot_of(ka);
                if (sl >= 0) {
                    const int tg = pk_target(trk.data(sl));
                    tgt5 = cell_r(tg) * W + cell_c(tg);
                }
            }
            float* o = idq + (size_t)a * 6 * HW;
            alt_emit_plane(L, NW, HW, AP_GRID, self, tgt5, o);
            alt_emit_plane(L, NW, HW, ka == 0 ? AP_URG : AP_ZERO, self, tgt5, o + HW);
            alt_emit_plane(L, NW, HW, ka == 0 ? AP_START : AP_ZERO, self, tgt5, o + 2 * HW);
            alt_emit_plane(L, NW, HW, AP_OTHERS, self, tgt5, o + 3 * HW);
            alt_emit_plane(L, NW, HW, AP_SELF, self, tgt5, o + 4 * HW);
            alt_emit_plane(L, NW, HW, AP_TGT, self, tgt5, o + 5 * HW);
        }
    }
    if (qst) {
        const int kinds[7] = {AP_GRID, AP_ROB, AP_CARRY, AP_START, AP_WT, AP_TT, AP_URG};
#pragma unroll
        for (int ch = 0; ch < 7; ch++) alt_emit_plane(L, NW, HW, kinds[ch], -1, -1, qst + (size_t)ch * HW);
    }
}

// convert_state for agents [a0, a0+na): dst [na][6][H][W]
template <class Trk>
__device__ inline void alt_emit_idq(const Trk& trk, const uint8_t* grid, int H, int W, const AltLds& L, int cell,
                                    int carry, int a0, int na, bool valid, float* dst) {
    const int HW = H * W;
    for (int k = 0; k < na; k++) {
        const int a = a0 + k;
        float* o = dst + (size_t)k * 6 * HW;
        if (!valid) {  // bad robot index: the map channel only
            emit(o, 6 * HW, [&](int i) -> float { return i < HW ? (float)grid[i] : 0.0f; });
            continue;
        }
        const int ca = rdl(cell, a), ka = rdl(carry, a);
        const int self = cell_r(ca) * W + cell_c(ca);
        int tgt5 = -1;  // carried package's target, when the id is in the tracker
        if (ka != 0) {
            const int sl = trk.slot_of(ka);
            if (sl >= 0) {
                const int tg = pk_target(trk.data(sl));
                tgt5 = cell_r(tg) * W + cell_c(tg);
            }
        }
        emit(o, 6 * HW, [&](int i) -> float {
            const int ch = i / HW, c = i - ch * HW;
            switch (ch) {
                case 0: return (float)grid[c];
                case 1: return (ka == 0 && L.urg[c] >= 0.0f) ? L.urg[c] : 0.0f;
                case 2: return (ka == 0 && L.urg[c] >= 0.0f) ? 1.0f : 0.0f;
                case 3: return (L.rob[c] != 0xff && (L.rob[c] & 63) != a) ? 1.0f : 0.0f;
                case 4: return c == self ? 1.0f : 0.0f;
                default: return c == tgt5 ? 1.0f : 0.0f;
            }
        });
    }
}

// convert_global_state_to_tensor with state_tensor_shape (7, oh, ow): dst [7][oh][ow].
// Only the map channel is centred / cropped; robots and packages keep their raw
// coordinates and are dropped outside (oh, ow), as the reference does.
__device__ inline void alt_emit_qmix(const uint8_t* grid, int H, int W, const AltLds& L, int oh, int ow, float* dst) {
    const int S = oh * ow;
    const int sr0 = H > oh ? (H - oh) / 2 : 0, sc0 = W > ow ? (W - ow) / 2 : 0;
    const int rows = H < oh ? H : oh, cols = W < ow ? W : ow;
    const int tro = (oh - rows) / 2, tco = (ow - cols) / 2;
    emit(dst, 7 * S, [&](int i) -> float {
        const int ch = i / S, q = i - ch * S;
        const int r = q / ow, c = q - r * ow;
        if (ch == 0) {
            const int rr = r - tro, cc = c - tco;
            return (rr >= 0 && rr < rows && cc >= 0 && cc < cols) ? (float)grid[(sr0 + rr) * W + sc0 + cc] : 0.0f;
        }
        if (r >= H || c >= W) return 0.0f;
        const int m = r * W + c;
        switch (ch) {
            case 1: return L.rob[m] != 0xff ? 1.0f : 0.0f;
            case 2: return (L.rob[m] != 0xff && (L.rob[m] & 0x40)) ? 1.0f : 0.0f;
            case 3: return L.urg[m] >= 0.0f ? 1.0f : 0.0f;
            case 4: return L.wt[m] ? 1.0f : 0.0f;
            case 5: return L.tt[m] ? 1.0f : 0.0f;
            default: return L.urg[m] >= 0.0f ? L.urg[m] : 0.0f;
        }
    });
}

// reward_shaping for the agent on this lane (fp64, the reference's accumulation order).
// op < 0 means the reference was handed string ops (IDQ/trainer.py): no op branch fires.
template <class Trk>
__device__ inline double idq_reward(const Trk& trk, int prev_cell, int prev_carry, int cur_cell, int cur_carry, int op,
                                    int t_prev, int t_cur) {
    double r = 0.0;
    if (prev_cell == cur_cell) r = r + -0.1;                           // SHAPING_STAY_PENALTY
    if (op == 1) {
        if (prev_carry == 0 && cur_carry != 0) r = r + 2.0;            // SHAPING_SUCCESSFUL_PICKUP_BONUS
        else if (prev_carry != 0) r = r + -0.1;                        // SHAPING_WASTED_PICKUP_PENALTY
        else {
            bool avail = false;
            for (int j = 0; j < trk.count() && !avail; j++) {
                if (!trk.present(j) || trk.in_transit(j)) continue;
                const uint64_t d = trk.data(j);
                avail = pk_start(d) == prev_cell && pk_st(d) <= t_prev;
            }
            if (!avail) r = r + -0.1;
        }
    } else if (op == 2) {
        if (prev_carry != 0 && cur_carry == 0) {
            const int sl = trk.slot_of(prev_carry);
            if (sl >= 0) {
                const uint64_t d = trk.data(sl);
                if (cur_cell == pk_target(d)) {
                    r = r + 10.0;                                        // SHAPING_SUCCESSFUL_DELIVERY_BONUS
                    if (t_cur > pk_dl(d)) r = r + -5.0;                  // SHAPING_LATE_DELIVERY_PENALTY
                }
            }
        } else if (prev_carry == 0) {
            r = r + 0.0;                                                 // SHAPING_WASTED_DROP_PENALTY
        }
    }
    return r;
}

}  // namespace mdl
