// mdl_obs_expand.hpp -- the flat emission pass of the observation builder.
//
// k_obs_expand turns the per-env records of obs_small_record (mdl_obs_small.hpp) into the four
// float32 output tensors of MAPPO/helper.py:6-255 (actor maps [n][A][6][H][W], actor vectors
// [n][A][6 + 5 MO + 5 MP + 1], critic maps [n][4][H][W], critic vectors [n][6 MR + 7 MPs + 1]).
// Thread i of a segment writes float4 i of its tensor and nothing else; blocks run in address
// order, so at any moment the chip's stores fall in one moving window -- the write shape of a
// fill (6.3+ TB/s on MI355X) instead of one stream per resident wave (5.1-5.3 TB/s,
// profiles/r03/slab_write_shapes*.jsonl).  A thread's float4 may straddle two envs, two planes
// or two agents, and a tensor may start anywhere inside a 16-B line: the first float's
// coordinates come from exact magic-number divisions, the next three by increments; the float4s
// at a tensor's two ends are stored per float.
#pragma once
#include "mdl_obs_small.hpp"

namespace mdl {

// floor(x / d) = umulhi(x, m) >> s for 0 <= x < 2^31 (obs_magic picks m, s on the host)
struct Magic {
    uint32_t m, s;
};
__device__ __forceinline__ uint32_t mdiv(uint32_t x, Magic g) { return __umulhi(x, g.m) >> g.s; }

inline Magic obs_magic(uint32_t d) {
    // s = floor(log2 d), m = ceil(2^(32+s) / d): m < 2^32 unless d is a power of two (then m = 2^31
    // and s - 1), and the error (m d - 2^(32+s)) x / 2^(32+s) < 1/d for every x < 2^31.
    // (d >= 2: the host never asks for d = 1)
    uint32_t s = 0;
    while ((2ull << s) <= d) s++;
    if ((d & (d - 1)) == 0) return Magic{0x80000000u, s - 1};
    const unsigned long long two = 1ull << (32 + s);
    return Magic{(uint32_t)((two + d - 1) / d), s};
}

struct ExpSeg {
    float* out;      // the tensor's first float rounded down to 16 B (nullptr: no segment)
    uint32_t lead;   // floats of the first float4 before the tensor's first float (0..3)
    uint32_t nf;     // floats of the segment: n envs x D
    uint32_t D;      // floats per env
    Magic mD;
    uint32_t blk0;   // first block of the segment in the launch
    uint32_t pad;
};

struct ExpandArgs {
    const uint32_t* rec;   // record of output row 0 (stride L.words)
    ObsRec L;
    int A, HW, np;         // np = 6A (actor map planes per env)
    Magic mHW;
    int Dv, ps0, Dg, MR6;  // actor vector length, first package slot, critic vector length, 6 MR
    Magic mDv;
    ExpSeg seg[4];         // 0 actor maps, 1 critic maps, 2 actor vectors, 3 critic vectors
};

// ---- values: (record, coordinates) -> float ----
// actor plane pp of an env at cell c (MAPPO/helper.py:6-66): grid, self, other robots (robots
// but self, plus cells holding two or more), waiting starts, active targets, carried target
__device__ __forceinline__ uint32_t amap_bit(const uint32_t* __restrict__ r, const ExpandArgs& x, uint32_t pp,
                                             uint32_t c) {
    const uint32_t a = (pp * 43691u) >> 18, ch = pp - 6u * a;   // pp / 6 (exact for pp < 2^16)
    const int set = ch == 0 ? BS_GRID : ch == 3 ? BS_WSTART : ch == 4 ? BS_ATARGET : BS_ROBOT;
    const uint32_t* b = r + x.L.o_bits + (c >> 5);
    const uint32_t sh = c & 31u;
    uint32_t v = (b[set * x.L.NW] >> sh) & 1u;
    const uint32_t own = r[x.L.o_aidx + 2 * a], tgt = r[x.L.o_aidx + 2 * a + 1];
    const uint32_t so = own == c ? 1u : 0u;
    if (ch == 1) v = so;
    else if (ch == 5) v = tgt == c ? 1u : 0u;
    else if (ch == 2) v = (v & ~so) | ((b[BS_MULTI * x.L.NW] >> sh) & 1u);
    return v;
}

// the 4 cells c0..c0+3 of actor plane pp (c0 % 4 == 0: one bitset word)
__device__ __forceinline__ uint32_t amap_bits4(const uint32_t* __restrict__ r, const ExpandArgs& x, uint32_t pp,
                                               uint32_t c0) {
    const uint32_t a = (pp * 43691u) >> 18, ch = pp - 6u * a;
    const int set = ch == 0 ? BS_GRID : ch == 3 ? BS_WSTART : ch == 4 ? BS_ATARGET : BS_ROBOT;
    const uint32_t* b = r + x.L.o_bits + (c0 >> 5);
    const uint32_t sh = c0 & 31u;
    uint32_t v = (b[set * x.L.NW] >> sh) & 15u;
    const uint32_t own = r[x.L.o_aidx + 2 * a], tgt = r[x.L.o_aidx + 2 * a + 1];
    const uint32_t so = own - c0 < 4u ? 1u << (own - c0) : 0u;
    if (ch == 1) v = so;
    else if (ch == 5) v = tgt - c0 < 4u ? 1u << (tgt - c0) : 0u;
    else if (ch == 2) v = (v & ~so) | ((b[BS_MULTI * x.L.NW] >> sh) & 15u);
    return v;
}

// critic plane ch = bitset ch (grid, robots, waiting starts, active targets; helper.py:167-198)
__device__ __forceinline__ uint32_t cmap_bit(const uint32_t* __restrict__ r, const ExpandArgs& x, uint32_t ch,
                                             uint32_t c) {
    return (r[x.L.o_bits + ch * x.L.NW + (c >> 5)] >> (c & 31u)) & 1u;
}

// float o of agent a's vector (helper.py:68-165): self + other-robot tuples, filled package
// slots, t/T last, zeros elsewhere
__device__ __forceinline__ float avec_val(const uint32_t* __restrict__ r, const ExpandArgs& x, uint32_t a,
                                          uint32_t o) {
    const uint32_t want = r[0];
    const uint32_t xe = 6u + 5u * (uint32_t)x.L.MOc, ps0 = (uint32_t)x.ps0;
    uint32_t k = 0xffffffffu;
    if (o < xe) k = o;
    else if (o - ps0 < 5u * want) k = xe + (o - ps0);
    if (o == (uint32_t)x.Dv - 1u) return __uint_as_float(r[2]);
    return k != 0xffffffffu ? __uint_as_float(r[x.L.o_av + a * (uint32_t)x.L.RA + k]) : 0.0f;
}

// float o of the critic vector (helper.py:199-255): nr robot rows, npr package rows, t/T last
__device__ __forceinline__ float cvec_val(const uint32_t* __restrict__ r, const ExpandArgs& x, uint32_t o) {
    const uint32_t npr = r[1], nr6 = 6u * (uint32_t)x.L.nr, MR6 = (uint32_t)x.MR6;
    uint32_t k = 0xffffffffu;
    if (o < nr6) k = o;
    else if (o - MR6 < 7u * npr) k = nr6 + (o - MR6);
    if (o == (uint32_t)x.Dg - 1u) return __uint_as_float(r[2]);
    return k != 0xffffffffu ? __uint_as_float(r[x.L.o_cv + k]) : 0.0f;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// the float4 of 4 bits (bit i -> float i), by one multiply and v_cvt_f32_ubyteN
__device__ __forceinline__ f32x4 f4_of_nibble(uint32_t b) {
    const uint32_t y = (b * 0x204081u) & 0x01010101u;   // bit i -> byte i (b < 16: no carries)
    return f32x4{cvt_ubyte<0>(y), cvt_ubyte<1>(y), cvt_ubyte<2>(y), cvt_ubyte<3>(y)};
}

// float4 q of segment S: v[i] = float 4q + i - lead of the tensor (valid where 0 <= f < nf)
template <int KIND>
__device__ __forceinline__ void expand_one(const ExpandArgs& x, const ExpSeg& S, uint32_t q) {
    const int64_t g0 = 4 * (int64_t)q - (int64_t)S.lead;      // tensor float of v[0]
    const bool full = g0 >= 0 && g0 + 4 <= (int64_t)S.nf;
    const uint32_t f0 = g0 < 0 ? 0u : (uint32_t)g0;            // a head float4 starts at float 0
    const uint32_t sk = (uint32_t)(f0 - g0);                   // v[0..sk) precede the tensor
    const uint32_t nleft = S.nf - f0;                          // >= 1: floats from f0 to the end
    uint32_t e = mdiv(f0, S.mD), off = f0 - e * S.D;
    const uint32_t* r = x.rec + (size_t)e * x.L.words;
    GLOBAL f32x4* dst = (GLOBAL f32x4*)S.out + q;
    if (KIND == 0 && full && (S.D & 3u) == 0 && (x.HW & 3) == 0 && S.lead == 0) {
        // one plane, 4 cells in one bitset word
        const uint32_t pp = mdiv(off, x.mHW), c0 = off - pp * (uint32_t)x.HW;
        *dst = f4_of_nibble(amap_bits4(r, x, pp, c0));
        return;
    }
    if (KIND == 1 && full && (S.D & 3u) == 0 && (x.HW & 3) == 0 && S.lead == 0) {
        const uint32_t ch = mdiv(off, x.mHW), c0 = off - ch * (uint32_t)x.HW;
        *dst = f4_of_nibble((r[x.L.o_bits + ch * x.L.NW + (c0 >> 5)] >> (c0 & 31u)) & 15u);
        return;
    }
    // general: coordinates of float f0, then +1 per float (an env / plane / agent boundary wraps)
    uint32_t u = 0, o = off;   // maps: plane u, cell o; actor vector: agent u, float o
    const uint32_t inner = KIND <= 1 ? (uint32_t)x.HW : KIND == 2 ? (uint32_t)x.Dv : (uint32_t)x.Dg;
    const uint32_t outer = KIND == 0 ? (uint32_t)x.np : KIND == 1 ? 4u : KIND == 2 ? (uint32_t)x.A : 1u;
    if (KIND <= 1) {
        u = mdiv(off, x.mHW);
        o = off - u * inner;
    } else if (KIND == 2) {
        u = mdiv(off, x.mDv);
        o = off - u * inner;
    }
    float vv[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        float val = 0.0f;
        if ((uint32_t)i >= sk && (uint32_t)i - sk < nleft) {   // no record past the last env is read
            if (KIND == 0) val = amap_bit(r, x, u, o) ? 1.0f : 0.0f;
            else if (KIND == 1) val = cmap_bit(r, x, u, o) ? 1.0f : 0.0f;
            else if (KIND == 2) val = avec_val(r, x, u, o);
            else val = cvec_val(r, x, o);
            if (++o == inner) {   // next plane / agent / env
                o = 0;
                if (++u == outer) {
                    u = 0;
                    r += x.L.words;
                }
            }
        }
        vv[i] = val;
    }
    if (full && S.lead == 0) {
        *dst = f32x4{vv[0], vv[1], vv[2], vv[3]};
    } else {
        float* d = (float*)S.out + 4 * (size_t)q;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int64_t f = g0 + i;
            if (f >= 0 && f < (int64_t)S.nf) d[i] = vv[i];
        }
    }
}

// One launch over the four segments (blocks of one segment are contiguous, in address order).
__global__ __launch_bounds__(256) void k_obs_expand(ExpandArgs x) {
    const uint32_t b = blockIdx.x;
    const int k = (b >= x.seg[1].blk0) + (b >= x.seg[2].blk0) + (b >= x.seg[3].blk0);   // uniform
    const uint32_t q = (b - x.seg[k].blk0) * 256u + threadIdx.x;
    switch (k) {
        case 0: {
            const ExpSeg& S = x.seg[0];
            if (4 * (uint64_t)q < (uint64_t)S.lead + S.nf) expand_one<0>(x, S, q);
            break;
        }
        case 1: {
            const ExpSeg& S = x.seg[1];
            if (4 * (uint64_t)q < (uint64_t)S.lead + S.nf) expand_one<1>(x, S, q);
            break;
        }
        case 2: {
            const ExpSeg& S = x.seg[2];
            if (4 * (uint64_t)q < (uint64_t)S.lead + S.nf) expand_one<2>(x, S, q);
            break;
        }
        default: {
            const ExpSeg& S = x.seg[3];
            if (4 * (uint64_t)q < (uint64_t)S.lead + S.nf) expand_one<3>(x, S, q);
            break;
        }
    }
}

}  // namespace mdl
