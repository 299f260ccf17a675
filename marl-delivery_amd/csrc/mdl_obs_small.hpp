// mdl_obs_small.hpp -- the engine's observation builder for small envs:
// A <= 8 robots, P <= 64 packages and 32-bit package sort keys (every trainer
// configuration of the reference: config 3 is map1, A = 5, P = 50, MO = 4,
// MP = 5, MR = MPs = 100; config 3b the helper defaults MO = MP = 100).
// Same outputs as k_obs (MAPPO/helper.py:6-255: convert_observation x A,
// generate_vector_features x A, convert_global_state), built for VALU economy --
// k_obs measured VALU-issue bound (2.6k VALU instructions per env on config 3,
// 4 cycles each on a 16-lane SIMD):
//   * packages on lanes (lane j = slot j), robots on lanes (lane a = robot a);
//     cross-lane data moves by ds_bpermute / DPP, not through per-value tables;
//   * package order per agent: repeated wave minima for a few slots, a bitonic
//     sort of the 64 lanes otherwise;
//   * every vector tuple (self / other robot / package slot of an agent, a
//     critic robot or package row) is computed by ONE lane in uniform passes
//     (the tuple kinds differ only in which operands feed the same divisions,
//     each one fp64 multiply by a precomputed reciprocal) and stored straight to
//     HBM; padding is a separate zero fill;
//   * maps: every output plane as bit words in LDS, one float4 per word nibble.
#pragma once
#include "mdl_features.hpp"

// Early whole-slab zero fill of mostly-padding actor vectors (see k_obs_small).  Measured
// (scripts/exp/earlyfill.sh, 16384 envs): the 1007-dim actor vectors 138-152 -> 122-124 us per
// build; the same early fill of the critic vector was slower (136-169 us), so it has none.
// Single-write actor vectors (mostly-padding vectors, e.g. the 1007-dim one): the tuples are
// assembled in an LDS image of each agent's data slots and the env's whole actor-vector slab
// is then streamed once as aligned float4s -- data float4s from the image, padding float4s as
// zeros -- instead of a zero-filled slab overwritten by the tuples after a vmcnt(0) wait
// (which wrote the tuple bytes twice).  Replaces the early fill when it applies.

namespace mdl {

__device__ __forceinline__ int bperm(int v, int src_lane) { return __builtin_amdgcn_ds_bpermute(src_lane << 2, v); }

// n zeros at dst: dword head to 16-B alignment, float4 body, dword tail.
// (Stores stay default-policy: nontemporal float4 stores measured slower,
// config 3 actor maps alone 34 -> 47 us.)
__device__ inline void zero_fill(float* dst, int n) {
    if (n <= 0) return;
    const int lane = lane_id();
    int head = (int)(((16 - ((uintptr_t)dst & 15)) & 15) >> 2);
    if (head > n) head = n;
    if (lane < head) dst[lane] = 0.0f;
    const int nb = (n - head) >> 2;
    float4* d4 = reinterpret_cast<float4*>(dst + head);
    for (int q = lane; q < nb; q += WAVE) d4[q] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const int tail = head + 4 * nb;
    if (tail + lane < n) dst[tail + lane] = 0.0f;
}

// Flat bit image of np output planes of HW cells each: bit p*HW + cell of FB is
// the value of (plane p, cell), so the planes are packed with no per-plane padding
// and bit i is float i of the [np][H][W] output.  src(p, c0) returns the 32 bits
// of plane p starting at cell c0 (bits past the plane's end are don't-care).
template <class F>
__device__ inline void build_flat(uint32_t* FB, int np, int HW, F src) {
    const int nfw = (np * HW + 31) >> 5;
    const float inv = 1.0f / (float)HW;
    for (int k = lane_id(); k < nfw; k += WAVE) {
        const int g0 = k << 5;   // < 2^23: fdivi is exact
        int p = fdivi(g0, HW, inv);
        int c0 = g0 - p * HW;
        uint32_t out = 0;
        int pos = 0;
        while (pos < 32 && p < np) {
            const int nb = min(32 - pos, HW - c0);
            const uint32_t m = nb >= 32 ? ~0u : ((1u << nb) - 1u);
            out |= (src(p, c0) & m) << pos;
            pos += nb;
            p++;
            c0 = 0;
        }
        FB[k] = out;
    }
}

// The 32 bits of bitset bs (NW words per set, sets back to back) starting at cell c0.
__device__ __forceinline__ uint32_t bits_at(const uint32_t* bits, int NW, int bs, int c0) {
    const uint32_t* w = bits + bs * NW + (c0 >> 5);
    return __builtin_amdgcn_alignbit(w[1], w[0], (uint32_t)(c0 & 31));
}

__device__ __forceinline__ uint32_t onehot32(int idx, int c0) {
    const unsigned d = (unsigned)(idx - c0);
    return d < 32u ? 1u << d : 0u;
}

// n floats of a flat bit image at dst (16-B aligned): one float4 per lane per pass.
// Float q*4..q*4+3 are the 4 bits at bit 4q: word q/8 -- with q = lane + 64k the
// word offset is lane/8 + 8k and the shift (lane%8)*4 is fixed per lane.  The 4
// bits are spread to bytes by one 24-bit multiply and converted by v_cvt_f32_ubyteN.
template <int B>
__device__ __forceinline__ float cvt_ubyte(uint32_t y) {
    float f;
    if constexpr (B == 0) asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(f) : "v"(y));
    else if constexpr (B == 1) asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(f) : "v"(y));
    else if constexpr (B == 2) asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(f) : "v"(y));
    else asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(f) : "v"(y));
    return f;
}

__device__ inline void emit_flat4(const uint32_t* FB, int n, float* dst) {
    const int lane = lane_id();
    const int nq = n >> 2;
    const uint32_t sh = (uint32_t)(lane & 7) << 2;
    const uint32_t* src = FB + (lane >> 3);
    GLOBAL char* base = (GLOBAL char*)dst;   // wave-uniform base + 32-bit lane offset
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    int q = lane;
    for (; q < nq; q += WAVE, src += 8) {
        const uint32_t b = __builtin_amdgcn_ubfe(*src, sh, 4u);
        const uint32_t y = (b * 0x204081u) & 0x01010101u;   // bit i -> byte i (no carries: b < 16)
        *(GLOBAL f32x4*)(base + ((uint32_t)q << 4)) = f32x4{cvt_ubyte<0>(y), cvt_ubyte<1>(y), cvt_ubyte<2>(y),
                                                            cvt_ubyte<3>(y)};
    }
    const int i = (nq << 2) + lane;   // n % 4 tail
    if (i < n) dst[i] = ((FB[i >> 5] >> (i & 31)) & 1u) ? 1.0f : 0.0f;
}

// The same, one dword per lane (an unaligned destination).
__device__ inline void emit_flat1(const uint32_t* FB, int n, float* dst) {
    for (int i = lane_id(); i < n; i += WAVE) dst[i] = ((FB[i >> 5] >> (i & 31)) & 1u) ? 1.0f : 0.0f;
}

// Lane-mask select with the mask in an SGPR pair: bit l set -> b, else a (one VALU op).
__device__ __forceinline__ uint32_t sel64(uint64_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}

// The lanes that keep the maximum in bitonic step (K, J) (ascending network).
template <int K, int J>
__host__ __device__ constexpr uint64_t bitonic_max_lanes() {
    uint64_t m = 0;
    for (int l = 0; l < 64; l++)
        if (((l & J) == 0) != ((l & K) == 0)) m |= 1ull << l;
    return m;
}

// x of lane (lane ^ J): DPP for 1, 2, 8; ds_swizzle (bitmask mode) for 4, 16;
// ds_bpermute for 32.
template <int J>
__device__ __forceinline__ uint32_t xor_lane(uint32_t x) {
    if constexpr (J == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xf, 0xf, false);   // quad_perm 1,0,3,2
    else if constexpr (J == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xf, 0xf, false);   // 2,3,0,1
    else if constexpr (J == 8) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xf, 0xf, false);   // row_ror:8
    else if constexpr (J == 4 || J == 16) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1f | (J << 10));
    else return (uint32_t)__builtin_amdgcn_ds_bpermute((lane_id() ^ J) << 2, (int)x);
}

template <int K, int J>
__device__ __forceinline__ uint32_t bitonic_step(uint32_t x) {
    const uint32_t y = xor_lane<J>(x);
    const uint32_t mn = x < y ? x : y, mx = x < y ? y : x;
    return sel64(bitonic_max_lanes<K, J>(), mn, mx);
}

// N independent wave sorts with their bitonic steps interleaved (each step applied to all N
// keys before the next): the N chains' DPP / swizzle / bpermute latencies overlap.
template <int N, int K, int J>
__device__ __forceinline__ void bitonic_stepn(uint32_t (&x)[N]) {
    uint32_t y[N];
#pragma unroll
    for (int i = 0; i < N; i++) y[i] = xor_lane<J>(x[i]);
#pragma unroll
    for (int i = 0; i < N; i++) {
        const uint32_t mn = x[i] < y[i] ? x[i] : y[i], mx = x[i] < y[i] ? y[i] : x[i];
        x[i] = sel64(bitonic_max_lanes<K, J>(), mn, mx);
    }
}

template <int N>
__device__ inline void sort64_u32xn(uint32_t (&x)[N]) {
    bitonic_stepn<N, 2, 1>(x);
    bitonic_stepn<N, 4, 2>(x);
    bitonic_stepn<N, 4, 1>(x);
    bitonic_stepn<N, 8, 4>(x);
    bitonic_stepn<N, 8, 2>(x);
    bitonic_stepn<N, 8, 1>(x);
    bitonic_stepn<N, 16, 8>(x);
    bitonic_stepn<N, 16, 4>(x);
    bitonic_stepn<N, 16, 2>(x);
    bitonic_stepn<N, 16, 1>(x);
    bitonic_stepn<N, 32, 16>(x);
    bitonic_stepn<N, 32, 8>(x);
    bitonic_stepn<N, 32, 4>(x);
    bitonic_stepn<N, 32, 2>(x);
    bitonic_stepn<N, 32, 1>(x);
    bitonic_stepn<N, 64, 32>(x);
    bitonic_stepn<N, 64, 16>(x);
    bitonic_stepn<N, 64, 8>(x);
    bitonic_stepn<N, 64, 4>(x);
    bitonic_stepn<N, 64, 2>(x);
    bitonic_stepn<N, 64, 1>(x);
}

// Ascending sort of one u32 per lane across the wave (bitonic network, 21 steps).
__device__ inline uint32_t sort64_u32(uint32_t x) {
    x = bitonic_step<2, 1>(x);
    x = bitonic_step<4, 2>(x);
    x = bitonic_step<4, 1>(x);
    x = bitonic_step<8, 4>(x);
    x = bitonic_step<8, 2>(x);
    x = bitonic_step<8, 1>(x);
    x = bitonic_step<16, 8>(x);
    x = bitonic_step<16, 4>(x);
    x = bitonic_step<16, 2>(x);
    x = bitonic_step<16, 1>(x);
    x = bitonic_step<32, 16>(x);
    x = bitonic_step<32, 8>(x);
    x = bitonic_step<32, 4>(x);
    x = bitonic_step<32, 2>(x);
    x = bitonic_step<32, 1>(x);
    x = bitonic_step<64, 32>(x);
    x = bitonic_step<64, 16>(x);
    x = bitonic_step<64, 8>(x);
    x = bitonic_step<64, 4>(x);
    x = bitonic_step<64, 2>(x);
    x = bitonic_step<64, 1>(x);
    return x;
}

// LDS bytes per wave: bitsets (5 NW words + a guard word), the actor planes' flat
// image (6A NW words), the critic planes' (4 NW words), carrier table and critic
// order (64 words each), order -> slot map (128 B), package order of each agent
// (8 x 64 B), each agent's (cell, carried target) index (16 words).
__host__ __device__ inline size_t obs_small_lds_base(int A, int HW) {
    const int NW = (HW + 31) / 32;
    return (4 * (size_t)((6 * A + 9) * NW + 1) + 2 * 256 + 128 + 512 + 64 + 15) & ~(size_t)15;
}
// The single-write image: the float4-aligned covers ("windows") of the actor-vector slab's data
// intervals -- per agent X(a) = its self / other-robot tuples with the previous agent's t/T, and
// Pk(a) = its filled package slots, then the last t/T -- plus the interval -> window tables.
// Upper bound of its float4s (each cover is at most len/4 + 2 float4s).
__host__ __device__ inline int obs_sw_f4(int A, int MOc, int MPc) {
    return A * ((7 + 5 * MOc) / 4 + 2 + (5 * MPc) / 4 + 2) + 2;
}
constexpr int OBS_SW_TAB = 16 * 2 * 8 + 16 * 3 * 8;   // bytes: [17] (q0, base) per interval, [17] windows
// Whether the single-write path applies to this configuration (the device also needs a 16-B
// aligned output, else it takes the early-fill path, which fits the same LDS slice).
__host__ __device__ inline bool obs_sw_config(int A, int P, int MO, int MP) {
    const int MOc = MO < A - 1 ? MO : A - 1, MPc = MP < P ? MP : P;
    return MO > MOc || MP > MPc;
}
__host__ __device__ inline size_t obs_small_lds(int A, int HW, int P, int MO, int MP) {
    const int MOc = MO < A - 1 ? MO : A - 1, MPc = MP < P ? MP : P;
    const size_t img = obs_sw_config(A, P, MO, MP) ? 16 * (size_t)obs_sw_f4(A, MOc, MPc) + OBS_SW_TAB : 0;
    return obs_small_lds_base(A, HW) + img;
}

// Eligibility (host and device agree): A <= 8 robots, P <= 64 packages, the
// package sort key (max(0,dl-t), rank, 7-bit order) in 32 bits, LDS slice <= 16 KiB.
__host__ __device__ inline bool obs_small_ok(int A, int P, int key7_dsh, int maxHW, int MO, int MP) {
    return A >= 1 && A <= 8 && P >= 1 && P <= WAVE && key7_dsh > 0 && obs_small_lds(A, maxHW, P, MO, MP) <= 16384;
}

// The builder's body for env e (output row w) from its state words as the lanes hold
// them: lane a < A the robot word, lane j < P package j's table entry, state word and
// (stale mode) tracker data, t the env clock.  k_obs_small loads them; the fused
// step + observation kernel (k_step<..., OBS = true>) passes the step's registers.
// `smem_wave` is this wave's LDS slice (obs_small_lds bytes).  rank_lds: the map's distance-rank
// table already copied into the workgroup's LDS (k_obs_small), or null: read from global memory.
template <bool STALE>
__device__ __forceinline__ void obs_small_emit(const DevParams& p, int w, int mi, uint32_t rv, uint64_t pkd,
                                               uint32_t f, uint64_t tdd, int t, float* __restrict__ amap,
                                               float* __restrict__ avec, float* __restrict__ cmap,
                                               float* __restrict__ cvec, unsigned char* smem_wave,
                                               const uint16_t* rank_lds = nullptr) {
    const int lane = lane_id();
    const int A = p.A, P = p.P;
    const MapDesc md = p.maps[mi];
    const int H = md.H, W = md.W, HW = H * W, NW = (HW + 31) / 32;
    const int T = p.obsT, MO = p.MO, MP = p.MP, MR = p.MR, MPs = p.MPs;
    const int MPc = MP < P ? MP : P, MPsc = MPs < P ? MPs : P;
    const int MOc = MO < A - 1 ? MO : A - 1;
    const double yH = p.obs_recip[2 * mi], yW = p.obs_recip[2 * mi + 1];   // RN(1/H), RN(1/W)
    const double yT = p.obs_recip[2 * p.n_maps], yM = p.obs_recip[2 * p.n_maps + 1];
    const uint16_t* rank = rank_lds ? rank_lds : p.rank + md.rank_off;
    const int rW = 2 * W - 1, rOff = (H - 1) * rW + (W - 1);   // rank[(dr+H-1)*(2W-1) + dc+W-1]

    uint32_t* bits = (uint32_t*)smem_wave;                       // [5][NW] + guard, critic planes first
    uint32_t* planes = bits + 5 * NW + 1;                         // flat image of the 6A actor planes
    uint32_t* cplanes = planes + 6 * A * NW;                      // flat image of the 4 critic planes
    int* scar = (int*)(cplanes + 4 * NW);                         // [64] carrier robot of a slot
    int* invc = scar + 64;                                        // [64] critic row -> slot
    uint8_t* o2j = (uint8_t*)(invc + 64);                         // [128] 7-bit order -> slot
    uint8_t* invp = o2j + 128;                                    // [8][64] (agent, rank) -> slot
    int* aidx = (int*)(invp + 512);                               // [8][2] agent's cell, carried target

    const bool rl = lane < A, pl = lane < P;
    if (lane == 0) bits[5 * NW] = 0;   // guard word read (and masked off) by bits_at
    for (int k = lane; k < NW; k += WAVE) {
        bits[BS_GRID * NW + k] = p.gridbits[md.bits_off + k];
        bits[BS_ROBOT * NW + k] = 0;
        bits[BS_MULTI * NW + k] = 0;
        bits[BS_WSTART * NW + k] = 0;
        bits[BS_ATARGET * NW + k] = 0;
    }
    scar[lane] = 0x7f;
    // Mostly-padding vectors (more slots than robots / packages, e.g. the 1007-dim
    // actor vector with 4 other robots in 100 slots): the whole slab is zeroed here
    // as one contiguous float4 stream, and the filled tuples are written over it
    // later, after an s_waitcnt vmcnt(0) (stores count in vmcnt on gfx9: the
    // zeros have reached L2 before any overwrite is issued).
    const bool sw = avec && obs_sw_config(A, P, MO, MP) && (((uintptr_t)avec & 15) == 0);
    const bool av_early = !sw && avec && (MO > MOc || MP > MPc);
    if (av_early) zero_fill(avec + (size_t)w * A * (6 + 5 * MO + 5 * MP + 1), A * (6 + 5 * MO + 5 * MP + 1));

    // ---- tracker view of each slot (TrkStale / TrkFresh) ----
    // ord7: the dict order as 7 bits -- survivors of earlier episodes by their
    // rank (< P <= 64), then this episode's entries by slot (MDL state words).
    bool pres, trans;
    uint64_t dat;
    uint32_t ord7;
    if (STALE) {
        pres = (f & PS_PRESENT) != 0;
        trans = (f & PS_TRANSIT) != 0;
        const bool sv = (f & PS_SURVIVOR) != 0;
        dat = sv ? tdd : pkd;
        ord7 = sv ? (f >> PS_RANK_SHIFT) & 63u : 64u + (uint32_t)lane;
    } else {
        const uint32_t s = f & PS_STATUS;
        pres = s == ST_WAITING || s == ST_IN_TRANSIT;
        trans = s == ST_IN_TRANSIT;
        dat = pkd;
        ord7 = (uint32_t)lane;
    }
    pres = pres && pl;
    trans = trans && pres;
    const int scl = pk_start(dat), tgl = pk_target(dat);
    const int sr = cell_r(scl), sc = cell_c(scl), tr = cell_r(tgl), tc = cell_c(tgl);
    const int stt = pk_st(dat);
    const bool wt = pres && !trans && stt <= t;     // waiting and spawned: actor ch3, actor package slots
    const bool actv = pres && (trans || stt <= t);  // critic package rows (MAPPO/helper.py:222-227)
    int dlc = pk_dl(dat) - t;
    dlc = (dlc < 0 || T <= 0) ? 0 : dlc;            // max(0, dl - t) (/T, or 0 when T <= 0)

    // ---- robots: cell, carried id, the carried slot's target (slot_of + in_transit) ----
    const int cell = rob_cell(rv), carry = rob_carry(rv);
    const int rr = cell_r(cell), rc = cell_c(cell);
    const bool cin = rl && carry >= 1 && carry <= P;
    const int cs = cin ? carry - 1 : 0;
    const int g_fl = bperm((int)pres | ((int)trans << 1), cs);
    const int g_tg = bperm(tgl, cs), g_dl = bperm(dlc, cs);
    const bool ctr = cin && (g_fl & 1) && (g_fl & 2);   // carrying an in-transit tracked package
    const int ctr_r = cell_r(g_tg), ctr_c = cell_c(g_tg);
    const int cidx = rr * W + rc, tidx = ctr ? ctr_r * W + ctr_c : -1;

    // ---- cell bitsets, carriers, critic order, order map ----
    wave_sync();
    if (rl) {
        aidx[2 * lane] = cidx;
        aidx[2 * lane + 1] = tidx;
        const uint32_t m = 1u << (cidx & 31);
        const uint32_t old = atomicOr(&bits[BS_ROBOT * NW + (cidx >> 5)], m);
        if (old & m) atomicOr(&bits[BS_MULTI * NW + (cidx >> 5)], m);   // a second robot on the cell
        if (carry >= 1 && carry <= WAVE) atomicMin(&scar[carry - 1], lane);   // first robot carrying the id
    }
    if (wt) {
        const int ci = sr * W + sc;
        atomicOr(&bits[BS_WSTART * NW + (ci >> 5)], 1u << (ci & 31));
    }
    if (wt || trans) {
        const int ci = tr * W + tc;
        atomicOr(&bits[BS_ATARGET * NW + (ci >> 5)], 1u << (ci & 31));
    }
    const uint64_t actm = ballot(actv);
    const int cpos = popc64(actm & lanemask_lt());
    const int nact = popc64(actm);
    if (actv) invc[cpos] = lane;   // critic package rows: active slots in id (= slot) order
    if (pres) o2j[ord7] = (uint8_t)lane;
    wave_sync();

    // ---- maps ----
    float* am = amap ? amap + (size_t)w * A * 6 * HW : nullptr;
    float* cm = cmap ? cmap + (size_t)w * 4 * HW : nullptr;
    if (am) {
        // plane p = (agent p/6, channel p%6): grid, self, other robots, waiting starts,
        // active targets, own carried target (MAPPO/helper.py:6-66)
        build_flat(planes, 6 * A, HW, [&](int pp, int c0) -> uint32_t {
            const int a = pp / 6, ch = pp - 6 * a;
            const int bs = ch == 0 ? BS_GRID : ch == 3 ? BS_WSTART : ch == 4 ? BS_ATARGET : BS_ROBOT;
            const uint32_t so = onehot32(aidx[2 * a], c0), to = onehot32(aidx[2 * a + 1], c0);
            uint32_t v = bits_at(bits, NW, bs, c0);
            v = ch == 2 ? (v & ~so) | bits_at(bits, NW, BS_MULTI, c0) : v;
            return ch == 1 ? so : ch == 5 ? to : v;
        });
    }
    if (cm)   // critic planes = bitsets 0..3 (grid, robots, waiting starts, active targets)
        build_flat(cplanes, 4, HW, [&](int pp, int c0) -> uint32_t { return bits_at(bits, NW, pp, c0); });
    wave_sync();
    if (am) {
        if (((uintptr_t)am & 15) == 0) emit_flat4(planes, 6 * A * HW, am);
        else emit_flat1(planes, 6 * A * HW, am);
    }
    if (cm) {
        if (((uintptr_t)cm & 15) == 0) emit_flat4(cplanes, 4 * HW, cm);
        else emit_flat1(cplanes, 4 * HW, cm);
    }

    // ---- actor vectors (MAPPO/helper.py:68-165) ----
    if (avec) {
        const int Dv = 6 + 5 * MO + 5 * MP + 1;
        float* av = avec + (size_t)w * A * Dv;
        // package order of each agent: (max(0,dl-t), distance rank, dict order) ascending
        const int np = popc64(ballot(wt));
        const int want = np < MPc ? np : MPc;
        const int dsh = p.key7_dsh;
        uint32_t key[8];
#pragma unroll
        for (int a = 0; a < 8; a++) {
            key[a] = 0xffffffffu;
            if (a < A) {
                const int ra_ = rdl(rr, a), ca_ = rdl(rc, a);
                const uint32_t rk = rank[rOff + (sr - ra_) * rW + (sc - ca_)];
                key[a] = wt ? ((uint32_t)dlc << dsh) | (rk << 7) | ord7 : 0xffffffffu;
            }
        }
        if (A == 5 && want > 6) {
            // the configs' five agents: their sorts as five interleaved bitonic networks
            uint32_t k5[5];
#pragma unroll
            for (int a = 0; a < 5; a++) k5[a] = key[a];
            sort64_u32xn<5>(k5);
#pragma unroll
            for (int a = 0; a < 5; a++)
                if (lane < want) invp[a * 64 + lane] = o2j[k5[a] & 127u];
        } else if (want <= 6) {
            // a few slots: repeated wave minima (keys are unique), all agents' at once by the
            // halving transpose (wave_min8_u32: ~20 VALU per slot for every agent instead of a
            // 6-stage DPP chain per agent)
            for (int s = 0; s < want; s++) {
                uint32_t k8[8];
#pragma unroll
                for (int a = 0; a < 8; a++) k8[a] = a < A ? key[a] : 0xffffffffu;
                const uint32_t v = wave_min8_u32(k8);
#pragma unroll
                for (int a = 0; a < 8; a++) {
                    if (a < A) {
                        const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)v, wave_min8_lane(a));
                        const bool hit = key[a] == m;
                        if (hit) invp[a * 64 + s] = (uint8_t)lane;
                        key[a] = hit ? 0xffffffffu : key[a];
                    }
                }
            }
        } else {
#pragma unroll
            for (int a = 0; a < 8; a++) {
                if (a < A) {
                    const uint32_t sk = sort64_u32(key[a]);
                    if (lane < want) invp[a * 64 + lane] = o2j[sk & 127u];
                }
            }
        }
        // Tuple lanes: q < A*A other robots (agent q/A, robot q%A); then A*ns package
        // slots (agent, slot); then A self tuples.  ns = MPc when every tuple fits one
        // pass (empty slots are zero tuples), else ns = want: only the filled slots, the
        // rest zero-filled with float4 stores below.  Other robots fit the first pass
        // (A <= 8), so their positions come from bpermutes within it.
        const int nq_o = A * A, ns = nq_o + A * MPc + A <= WAVE ? MPc : want;
        const int nq_p = A * ns, ntup = nq_o + nq_p + A;
        const float inv_a = 1.0f / (float)A, inv_w = ns > 0 ? 1.0f / (float)ns : 0.0f;
        // Single-write: the slab [g0, g0 + A*Dv) (float indices from avec) holds 2A+1 data intervals
        // in order -- X(a) = [a*Dv - 1 (a > 0), a*Dv + 6 + 5MOc): agent a-1's t/T, agent a's self and
        // filled other-robot tuples; Pk(a) = [a*Dv + 6 + 5MO, +5*want): its filled package slots; the
        // last agent's t/T -- everything else is padding.  Each interval's float4 cover becomes a
        // window of the LDS image (covers that share a float4 are merged), laid out exactly as the
        // output, so the tuples are written into it and the slab is then streamed once: windows as
        // float4 copies, the gaps between them as zero float4s.
        const int g0 = w * A * Dv, S = A * Dv;
        const int xe = 6 + 5 * MOc, ps0 = 6 + 5 * MO;
        float4* img4 = reinterpret_cast<float4*>(smem_wave + obs_small_lds_base(A, HW));
        int2* ktab = reinterpret_cast<int2*>(img4 + obs_sw_f4(A, MOc, MPc));   // interval k -> (cover q0, image base)
        int4* wtab = reinterpret_cast<int4*>(ktab + 16 * 2 + 2);                // window -> (q0, q1, base)
        int nwin = 0;
        if (sw) {
            int nf4 = 0, cq0 = 0, cq1 = 0, cbase = 0;
            for (int k = 0; k <= 2 * A; k++) {   // uniform
                const int a = k >> 1;
                const int s0 = k == 2 * A ? S - 1 : (k & 1) ? a * Dv + ps0 : a * Dv - (a > 0 ? 1 : 0);
                const int s1 = k == 2 * A ? S : (k & 1) ? s0 + 5 * want : a * Dv + xe;
                if (s1 <= s0) continue;
                const int qs = (g0 + s0) >> 2, qe = (g0 + s1 + 3) >> 2;
                if (nwin > 0 && qs < cq1) {   // shares a float4 with the open window: merge
                    cq1 = qe > cq1 ? qe : cq1;
                } else {
                    if (nwin > 0 && lane == 0) wtab[nwin - 1] = int4{cq0, cq1, cbase, 0};
                    nf4 += cq1 - cq0;
                    cq0 = qs;
                    cq1 = qe;
                    cbase = nf4;
                    nwin++;
                }
                if (lane == 0) ktab[k] = int2{cq0, cbase};
            }
            if (lane == 0) wtab[nwin - 1] = int4{cq0, cq1, cbase, 0};
            nf4 += cq1 - cq0;
            for (int q = lane; q < nf4; q += WAVE) img4[q] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
        wave_sync();
        // float f of the slab (interval k) -> its image float
        auto img_at = [&](int k, int f) -> float* {
            const int2 kt = ktab[k];
            return reinterpret_cast<float*>(img4) + 4 * kt.y + (g0 + f - 4 * kt.x);
        };
        if (sw && lane < A)   // t/T of every agent: the first float of X(a+1), or the last interval
            *img_at(lane + 1 < A ? 2 * (lane + 1) : 2 * A, lane * Dv + Dv - 1) = qdiv_r(t, yT);
        wave_sync();
#ifndef MDL_EXP_NOWAIT   // profiling builds only (wrong results): no wait between the fill and the tuples
        if (av_early) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the slab's zeros are in L2
#endif
        for (int q0 = 0; q0 < ntup; q0 += WAVE) {   // uniform trip count
            const int q = q0 + lane;
            const bool is_o = q < nq_o, is_p = !is_o && q < nq_o + nq_p, is_s = !is_o && !is_p && q < ntup;
            int qa, qb;   // agent, and other robot / package slot / (self) agent
            if (is_o) {
                qa = fdivi(q, A, inv_a);
                qb = q - qa * A;
            } else if (is_p) {
                qa = fdivi(q - nq_o, ns, inv_w);
                qb = q - nq_o - qa * ns;
            } else {
                qa = is_s ? q - nq_o - nq_p : 0;
                qb = qa;
            }
            const int ra = bperm(rr, qa), ca = bperm(rc, qa);
            const int ob = is_o ? qb : 0;
            const int ro = bperm(rr, ob), co = bperm(rc, ob);
            const bool ovalid = is_o && qb != qa;
            const int orank = rank[rOff + (ro - ra) * rW + (co - ca)];
            const int okey = ovalid ? (orank << 3) | qb : 0x7fffffff;   // (rank, robot index)
            int opos = 0;
            for (int k = 0; k < A; k++) opos += bperm(okey, (qa * A + k) & 63) < okey;
            const bool phas = is_p && qb < want;
            const int pj = phas ? invp[qa * 64 + qb] : 0;
            const int p_sc = bperm(scl, pj), p_tg = bperm(tgl, pj), p_dl = bperm(dlc, pj);
            const int rsrc = is_o ? qb : qa;   // the robot a self / other tuple describes
            const int o_cy = bperm(carry, rsrc), o_ctr = bperm((int)ctr, rsrc);
            const int o_tr = bperm(ctr_r, rsrc), o_tc = bperm(ctr_c, rsrc), o_dl = bperm(g_dl, rsrc);
            int x1, x2, x3, x4, x5;
            if (is_p) {
                x1 = phas ? cell_r(p_sc) - ra : 0;
                x2 = phas ? cell_c(p_sc) - ca : 0;
                x3 = phas ? cell_r(p_tg) - ra : 0;
                x4 = phas ? cell_c(p_tg) - ca : 0;
                x5 = phas ? p_dl : 0;
            } else {
                const int br = is_o ? ro : ra, bc = is_o ? co : ca;
                x1 = is_o ? ro - ra : ra;
                x2 = is_o ? co - ca : ca;
                const bool ht = o_cy != 0 && o_ctr != 0;
                x3 = ht ? o_tr - br : 0;
                x4 = ht ? o_tc - bc : 0;
                x5 = ht ? o_dl : 0;
            }
            const float d1 = qdiv_r(x1, yH), d2 = qdiv_r(x2, yW), d3 = qdiv_r(x3, yH), d4 = qdiv_r(x4, yW);
            const float d5 = qdiv_r(x5, yT);   // x5 = 0 when T <= 0
            const float fl = o_cy != 0 ? 1.0f : 0.0f;
#ifdef MDL_EXP_NOTUPLES   // profiling builds only (wrong results): the actor vectors' tuples are not stored
            if (false) {
#else
            // (single-write: empty package slots are zeros in the image already, and their interval
            // may have no window)
            if ((ovalid && opos < MO) || (is_p && (phas || !sw)) || is_s) {
#endif
                const int off = is_s ? 0 : is_o ? 6 + 5 * opos : 6 + 5 * MO + 5 * qb;
                float* o = sw ? img_at(is_p ? 2 * qa + 1 : 2 * qa, qa * Dv + off) : av + qa * Dv + off;
                o[0] = d1;
                o[1] = d2;
                o[2] = is_p ? d3 : fl;
                o[3] = is_p ? d4 : d3;
                o[4] = is_p ? d5 : d4;
                if (is_s) {
                    o[5] = d5;
                    if (!sw) o[Dv - 1] = qdiv_r(t, yT);   // yT = 0 when T <= 0
                }
            }
        }
        if (sw) {
            // Stream the slab once: every window's float4s from the image (a float4 that also holds
            // another env's floats -- only at the slab's ends -- per float), the gap up to the next
            // window as zeros.  The first window starts at the slab's first float4 and the last ends
            // at its last, so every gap float4 lies inside the slab.
            wave_sync();
            float4* a4 = reinterpret_cast<float4*>(avec);
            // The slab's two end float4s may hold a neighbouring env's floats: written per float
            // by two lanes; every other float4 by uniform-trip loops in which lanes past a run's end
            // repeat its last float4 (the same value: no exec-mask branches per iteration).
            const int qh = g0 >> 2, qt = (g0 + S - 1) >> 2;   // the slab's first / last float4
            const bool ph = (g0 & 3) != 0, pt = ((g0 + S) & 3) != 0;
            if ((lane == 0 && ph) || (lane == 1 && pt)) {
                const int q = lane == 0 ? qh : qt;
                const int wi = lane == 0 ? 0 : nwin - 1;   // its window: the first / the last
                const int4 wt = wtab[wi];
                const float4 v = img4[wt.z + (q - wt.x)];
                const int f0 = 4 * q - g0;
                float* d = avec + 4 * (size_t)q;
                if ((unsigned)f0 < (unsigned)S) d[0] = v.x;
                if ((unsigned)(f0 + 1) < (unsigned)S) d[1] = v.y;
                if ((unsigned)(f0 + 2) < (unsigned)S) d[2] = v.z;
                if ((unsigned)(f0 + 3) < (unsigned)S) d[3] = v.w;
            }
            for (int wi = 0; wi < nwin; wi++) {   // uniform
                const int4 wt = wtab[wi];
                const int x0 = wt.x + ((wi == 0 && ph) ? 1 : 0);
                const int y0 = wt.y - ((wi == nwin - 1 && pt) ? 1 : 0);
                for (int q0 = x0; q0 < y0; q0 += WAVE) {   // uniform
                    const int q = min(q0 + lane, y0 - 1);
                    a4[q] = img4[wt.z + (q - wt.x)];
                }
                const int gend = wi + 1 < nwin ? wtab[wi + 1].x : wt.y;
                for (int q0 = wt.y; q0 < gend; q0 += WAVE)   // uniform
                    a4[min(q0 + lane, gend - 1)] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            }
        }
        // padding: other-robot slots [MOc, MO) and package slots [ns, MP) of every agent
        if (!sw && !av_early && (MO > MOc || MP > ns)) {
            for (int a = 0; a < A; a++) {
                zero_fill(av + a * Dv + 6 + 5 * MOc, 5 * (MO - MOc));
                zero_fill(av + a * Dv + 6 + 5 * MO + 5 * ns, 5 * (MP - ns));
            }
        }
    }

    // ---- critic vector (MAPPO/helper.py:199-255) ----
    if (cvec) {
        const int Dg = 6 * MR + 7 * MPs + 1;
        float* cv = cvec + (size_t)w * Dg;
        const int nr = A < MR ? A : MR;
        const int npr = nact < MPsc ? nact : MPsc;
        for (int q0 = 0; q0 < nr + npr; q0 += WAVE) {   // uniform trip count: bperm needs every lane
            const int q = q0 + lane;
            const bool isr = q < nr, live = q < nr + npr;
            const int j = (isr || !live) ? 0 : invc[q - nr];
            const int p_sc = bperm(scl, j), p_tg = bperm(tgl, j), p_dl = bperm(dlc, j);
            const int p_tr = bperm((int)trans, j), p_car = scar[j];
            const int rq = q & 63;
            const int r_cy = bperm(carry, rq), r_ctr = bperm((int)ctr, rq), r_r = bperm(rr, rq), r_c = bperm(rc, rq);
            const int r_tr = bperm(ctr_r, rq), r_tc = bperm(ctr_c, rq), r_dl = bperm(g_dl, rq);
            const bool rht = r_cy != 0 && r_ctr != 0;
            const bool waiting = p_tr == 0;
            const int x1 = isr ? r_r : (waiting ? cell_r(p_sc) : 0);
            const int x2 = isr ? r_c : (waiting ? cell_c(p_sc) : 0);
            const int x3 = isr ? (rht ? r_tr : 0) : cell_r(p_tg);
            const int x4 = isr ? (rht ? r_tc : 0) : cell_c(p_tg);
            const int x5 = isr ? (rht ? r_dl : 0) : p_dl;
            const bool hascar = !isr && !waiting && p_car != 0x7f;
            const float d1 = qdiv_r(x1, yH), d2 = qdiv_r(x2, yW), d3 = qdiv_r(x3, yH), d4 = qdiv_r(x4, yW);
            const float d5 = qdiv_r(x5, yT);
            const float d6 = hascar ? qdiv_r(p_car, yM) : -1.0f;   // yM = 0 when MR <= 1
            const float fl = isr ? (r_cy != 0 ? 1.0f : 0.0f) : (waiting ? 0.0f : 1.0f);
            if (live) {
                float* o = cv + (isr ? 6 * q : 6 * MR + 7 * (q - nr));
                o[0] = d1;
                o[1] = d2;
                o[2] = isr ? fl : d3;
                o[3] = isr ? d3 : d4;
                o[4] = isr ? d4 : d5;
                o[5] = isr ? d5 : fl;
                if (!isr) o[6] = d6;
            }
        }
        zero_fill(cv + 6 * nr, 6 * (MR - nr));
        zero_fill(cv + 6 * MR + 7 * npr, 7 * (MPs - npr));
        if (lane == 0) cv[Dg - 1] = qdiv_r(t, yT);
    }
}

// rank_lds > 0: the launch's maps (one shape, so one rank table) have their table copied into the
// first rank_lds bytes of the workgroup's LDS before the waves start: the package-order keys and the
// other-robot order then gather ranks from LDS (~64 cycles) instead of L2 (hundreds)
template <bool STALE, bool RL>
__global__ __launch_bounds__(256) void k_obs_small(DevParams p, int env_begin, int n, float* __restrict__ amap,
                                                   float* __restrict__ avec, float* __restrict__ cmap,
                                                   float* __restrict__ cvec, int wpb, int lds_stride, int rank_lds) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = wave_id();
    const int lane = lane_id();
    uint16_t* rk = (uint16_t*)smem;
    if constexpr (RL) {
        const MapDesc md0 = p.maps[p.env_map ? p.env_map[env_begin] : 0];   // every env of the launch: one shape
        const int nrk = (2 * md0.H - 1) * (2 * md0.W - 1);
        const uint16_t* src = p.rank + md0.rank_off;
        for (int i = (int)threadIdx.x; i < nrk; i += 256) rk[i] = src[i];
        __syncthreads();   // every wave of the block is still here (none has returned yet)
    }
    const int w = xcd_block() * wpb + wave;
    if (wave >= wpb || w >= n) return;
    const int e = env_begin + w;
    const int A = p.A, P = p.P;
    const int mi = p.env_map ? p.env_map[e] : 0;
    // ---- loads: robots, packages (+ tracker data), clock ----
    const uint32_t rv = lane < A ? p.rob[(size_t)e * A + lane] : 0u;
    uint64_t pkd = 0, tdd = 0;
    uint32_t f = 0;
    if (lane < P) {
        const size_t g = (size_t)e * P + lane;
        pkd = p.pkg[g];
        f = p.pstate[g];
        if (STALE) tdd = p.trk[g];
    }
    const int t = p.es[e].t;
    obs_small_emit<STALE>(p, w, mi, rv, pkd, f, tdd, t, amap, avec, cmap, cvec,
                          smem + rank_lds + (size_t)wave * lds_stride, RL ? rk : nullptr);
}

}  // namespace mdl
