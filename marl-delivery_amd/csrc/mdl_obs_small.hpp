// mdl_obs_small.hpp -- the engine's observation builder for small envs:
// A <= 8 robots, P <= 64 packages, <= 8 package slots per agent and 32-bit
// package sort keys (the trainers' featurizer sizes: config 3 is map1, A = 5,
// P = 50, MO = 4, MP = 5, MR = MPs = 100).  Same outputs as k_obs
// (MAPPO/helper.py:6-255: convert_observation x A, generate_vector_features x A,
// convert_global_state), built for VALU economy -- k_obs measured VALU-issue
// bound (2.6k VALU instructions per env, 4 cycles each on a 16-lane SIMD):
//   * packages on lanes (lane j = slot j), robots on lanes (lane a = robot a);
//     cross-lane data moves by ds_bpermute, never through per-value LDS tables;
//   * every vector tuple (self / other robot / waiting package of an agent, a
//     critic robot or package row) is computed by ONE lane in ONE uniform pass
//     (the tuple kinds differ only in which operands feed the same five
//     divisions), then stored straight to HBM; padding is a separate zero fill;
//   * maps: every output plane as bit words in LDS, one float4 per word nibble.
#pragma once
#include "mdl_features.hpp"

namespace mdl {

__device__ __forceinline__ int bperm(int v, int src_lane) { return __builtin_amdgcn_ds_bpermute(src_lane << 2, v); }

// n zeros at dst: dword head to 16-B alignment, float4 body, dword tail.
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

// Planes [0, np) of pl (HW cells each) as floats at dst, one dword per cell
// (maps with HW % 4 != 0 or an unaligned destination).
__device__ inline void emit_planes_dword(const uint32_t* pl, int NW, int np, int HW, float* dst) {
    const int lane = lane_id();
    const float inv = 1.0f / (float)HW;
    for (int i = lane; i < np * HW; i += WAVE) {
        const int p = fdivi(i, HW, inv);
        const int cell = i - p * HW;
        dst[i] = ((pl[p * NW + (cell >> 5)] >> (cell & 31)) & 1u) ? 1.0f : 0.0f;
    }
}

struct ObsSmallDims {
    int A, NW;
};
// LDS bytes per wave: bitsets (5 NW words), planes ((6A+4) NW words), carrier
// table (64 words), critic order (64 words), package selection (64 words).
__host__ __device__ inline size_t obs_small_lds(int A, int HW) {
    const int NW = (HW + 31) / 32;
    return 4 * (size_t)((6 * A + 9) * NW) + 3 * 256;
}

// Eligibility (host and device agree): see the file comment.
__host__ __device__ inline bool obs_small_ok(int A, int P, int MO, int MP, int key32_dsh, int maxHW) {
    const int MPc = MP < P ? MP : P;
    const int MOc = MO < A - 1 ? MO : (A - 1 > 0 ? A - 1 : 0);
    return A >= 1 && A <= 8 && P <= WAVE && MPc <= 8 && key32_dsh > 0 && A * (A + MPc + 1) <= WAVE &&
           MOc >= 0 && obs_small_lds(A, maxHW) <= 16384;
}

template <bool STALE>
__global__ __launch_bounds__(256) void k_obs_small(DevParams p, int env_begin, int n, float* __restrict__ amap,
                                                   float* __restrict__ avec, float* __restrict__ cmap,
                                                   float* __restrict__ cvec, int wpb, int lds_stride) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = wave_id();
    const int lane = lane_id();
    const int w = blockIdx.x * wpb + wave;
    if (wave >= wpb || w >= n) return;
    const int e = env_begin + w;
    const int A = p.A, P = p.P;
    const MapDesc md = p.maps[p.env_map ? p.env_map[e] : 0];
    const int H = md.H, W = md.W, HW = H * W, NW = (HW + 31) / 32;
    const int T = p.obsT, MO = p.MO, MP = p.MP, MR = p.MR, MPs = p.MPs;
    const int MPc = MP < P ? MP : P, MPsc = MPs < P ? MPs : P;
    const int MOc = MO < A - 1 ? MO : A - 1;
    const int mi = p.env_map ? p.env_map[e] : 0;
    const double yH = p.obs_recip[2 * mi], yW = p.obs_recip[2 * mi + 1];   // RN(1/H), RN(1/W)
    const double yT = p.obs_recip[2 * p.n_maps], yM = p.obs_recip[2 * p.n_maps + 1];
    const uint16_t* rank = p.rank + md.rank_off;
    const int rW = 2 * W - 1, rOff = (H - 1) * rW + (W - 1);   // rank[(dr+H-1)*(2W-1) + dc+W-1]

    uint32_t* bits = (uint32_t*)(smem + (size_t)wave * lds_stride);   // [5][NW]
    uint32_t* planes = bits + 5 * NW;                                 // [(6A+4)][NW]
    int* scar = (int*)(planes + (6 * A + 4) * NW);                    // [64] carrier robot of a slot
    int* invc = scar + 64;                                            // [64] critic row -> slot
    int* invp = invc + 64;                                            // [64] (agent, slot) -> package

    // ---- loads: robots, packages (+ tracker data), clock ----
    const bool rl = lane < A, pl = lane < P;
    const uint32_t rv = rl ? p.rob[(size_t)e * A + lane] : 0u;
    uint64_t pkd = 0, tdd = 0;
    uint32_t f = 0;
    if (pl) {
        const size_t g = (size_t)e * P + lane;
        pkd = p.pkg[g];
        f = p.pstate[g];
        if (STALE) tdd = p.trk[g];
    }
    const int t = p.es[e].t;
    for (int k = lane; k < NW; k += WAVE) {
        bits[BS_GRID * NW + k] = p.gridbits[md.bits_off + k];
        bits[BS_ROBOT * NW + k] = 0;
        bits[BS_MULTI * NW + k] = 0;
        bits[BS_WSTART * NW + k] = 0;
        bits[BS_ATARGET * NW + k] = 0;
    }
    scar[lane] = 0x7f;

    // ---- tracker view of each slot (TrkStale / TrkFresh) ----
    bool pres, trans;
    uint64_t dat;
    uint32_t ord;
    if (STALE) {
        pres = (f & PS_PRESENT) != 0;
        trans = (f & PS_TRANSIT) != 0;
        const bool sv = (f & PS_SURVIVOR) != 0;
        dat = sv ? tdd : pkd;
        ord = sv ? f >> PS_RANK_SHIFT : ORD_EPISODE + (uint32_t)lane;
    } else {
        const uint32_t s = f & PS_STATUS;
        pres = s == ST_WAITING || s == ST_IN_TRANSIT;
        trans = s == ST_IN_TRANSIT;
        dat = pkd;
        ord = (uint32_t)lane;
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

    // ---- cell bitsets, carriers ----
    wave_sync();
    if (rl) {
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
    // critic package rows: active slots in id (= slot) order
    const uint64_t actm = ballot(actv);
    const int cpos = popc64(actm & lanemask_lt());
    const int nact = popc64(actm);
    if (actv) invc[cpos] = lane;
    wave_sync();

    // ---- maps ----
    float* am = amap ? amap + (size_t)w * A * 6 * HW : nullptr;
    float* cm = cmap ? cmap + (size_t)w * 4 * HW : nullptr;
    if (am || cm) {
        const int npl = (6 * A + 4) * NW;
        const float inv_nw = 1.0f / (float)NW;
        // uniform trip count: the robot gathers below need every lane active
        for (int k0 = 0; k0 < npl; k0 += WAVE) {
            const int k = k0 + lane;
            const int pp = fdivi(k, NW, inv_nw);
            const int wd = k - pp * NW;
            const int base = wd << 5;
            const uint32_t g = bits[BS_GRID * NW + wd], rb = bits[BS_ROBOT * NW + wd];
            const uint32_t ws = bits[BS_WSTART * NW + wd], at = bits[BS_ATARGET * NW + wd];
            const uint32_t mu = bits[BS_MULTI * NW + wd];
            const int a = pp / 6, ch = pp - 6 * a;   // a >= A: critic plane ch - 6(a - A)
            const int asrc = a < A ? a : 0;
            const unsigned od = (unsigned)(bperm(cidx, asrc) - base), td = (unsigned)(bperm(tidx, asrc) - base);
            const uint32_t ow = od < 32u ? 1u << od : 0u;
            const uint32_t tw = td < 32u ? 1u << td : 0u;   // no carried target: -1
            uint32_t v;
            if (pp < 6 * A) {
                v = ch == 0 ? g : ch == 1 ? ow : ch == 2 ? ((rb & ~ow) | mu) : ch == 3 ? ws : ch == 4 ? at : tw;
            } else {
                const int cc = pp - 6 * A;
                v = cc == 0 ? g : cc == 1 ? rb : cc == 2 ? ws : at;
            }
            if (k < npl) planes[k] = v;
        }
        wave_sync();
        const bool f4 = (HW & 3) == 0;
        if (am) {
            if (f4 && ((uintptr_t)am & 15) == 0) emit_planes(planes, NW, 6 * A, HW, am);
            else emit_planes_dword(planes, NW, 6 * A, HW, am);
        }
        if (cm) {
            if (f4 && ((uintptr_t)cm & 15) == 0) emit_planes(planes + 6 * A * NW, NW, 4, HW, cm);
            else emit_planes_dword(planes + 6 * A * NW, NW, 4, HW, cm);
        }
    }

    // ---- actor vectors (MAPPO/helper.py:68-165) ----
    if (avec) {
        const int Dv = 6 + 5 * MO + 5 * MP + 1;
        float* av = avec + (size_t)w * A * Dv;
        // tuple lanes: q < A*A other robots (agent q/A, robot q%A); then A*MPc package
        // slots (agent, slot); then A self tuples
        const int nq_o = A * A, nq_p = A * MPc;
        const int q = lane;
        const bool is_o = q < nq_o, is_p = !is_o && q < nq_o + nq_p, is_s = !is_o && !is_p && q < nq_o + nq_p + A;
        int qa, qb;   // agent, and other robot / package slot / (self) agent
        if (is_o) {
            qa = q / A;
            qb = q - qa * A;
        } else if (is_p) {
            qa = (q - nq_o) / MPc;
            qb = q - nq_o - qa * MPc;
        } else {
            qa = is_s ? q - nq_o - nq_p : 0;
            qb = qa;
        }
        const int ra = bperm(rr, qa), ca = bperm(rc, qa);
        const int ro = bperm(rr, qb), co = bperm(rc, qb);
        const bool ovalid = is_o && qb != qa;
        // other-robot key (rank, index) -- its rank gather issued with the package keys'
        const int orank = rank[rOff + (ro - ra) * rW + (co - ca)];
        // waiting-package selection: per agent the MPc smallest (max(0,dl-t), rank, order)
        // keys by repeated wave minima; (agent a, slot s) -> package lane in invp[a*8+s]
        const int np = popc64(ballot(wt));
        const int want = np < MPc ? np : MPc;
        const int dsh = p.key32_dsh;
        uint32_t key[8];
#pragma unroll
        for (int a = 0; a < 8; a++) {
            key[a] = 0xffffffffu;
            if (a < A) {
                const int ra_ = rdl(rr, a), ca_ = rdl(rc, a);
                const uint32_t rk = rank[rOff + (sr - ra_) * rW + (sc - ca_)];
                key[a] = wt ? ((uint32_t)dlc << dsh) | (rk << 11) | ord : 0xffffffffu;
            }
        }
        for (int s = 0; s < want; s++) {
#pragma unroll
            for (int a = 0; a < 8; a++) {
                if (a < A) {
                    const uint32_t m = wave_min_u32(key[a]);
                    const bool hit = key[a] == m;
                    if (hit) invp[a * 8 + s] = lane;
                    key[a] = hit ? 0xffffffffu : key[a];
                }
            }
        }
        const int okey = ovalid ? (orank << 3) | qb : 0x7fffffff;
        int opos = 0;
        for (int k = 0; k < A; k++) opos += bperm(okey, qa * A + k) < okey;
        wave_sync();
        const int j = is_p ? invp[qa * 8 + qb] : 0;
        const bool phas = is_p && qb < want;
        // the operands: robot qb (self / other) or package j (package slot)
        const int pj = phas ? j : 0;
        const int p_sc = bperm(scl, pj), p_tg = bperm(tgl, pj), p_dl = bperm(dlc, pj);
        const int rsrc = is_o ? qb : qa;   // robot whose carried target is reported
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
            const int br = is_o ? ro : ra, bc = is_o ? co : ca;   // the robot described
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
        const bool wr = (is_o && ovalid && opos < MO) || is_p || is_s;
        if (wr) {
            const int off = qa * Dv + (is_s ? 0 : is_o ? 6 + 5 * opos : 6 + 5 * MO + 5 * qb);
            float* o = av + off;
            o[0] = d1;
            o[1] = d2;
            o[2] = is_p ? d3 : fl;
            o[3] = is_p ? d4 : d3;
            o[4] = is_p ? d5 : d4;
            if (is_s) {
                o[5] = d5;
                o[Dv - 1] = qdiv_r(t, yT);   // yT = 0 when T <= 0
            }
        }
        // padding: other-robot slots [MOc, MO) and package slots [MPc, MP) of every agent
        if (MO > MOc || MP > MPc) {
            for (int a = 0; a < A; a++) {
                zero_fill(av + a * Dv + 6 + 5 * MOc, 5 * (MO - MOc));
                zero_fill(av + a * Dv + 6 + 5 * MO + 5 * MPc, 5 * (MP - MPc));
            }
        }
    }

    // ---- critic vector (MAPPO/helper.py:199-255) ----
    if (cvec) {
        const int Dg = 6 * MR + 7 * MPs + 1;
        float* cv = cvec + (size_t)w * Dg;
        const int nr = A < MR ? A : MR;
        const int npr = nact < MPsc ? nact : MPsc;
        // uniform trip count (ds_bpermute reads inactive lanes as 0): stores masked
        for (int q0 = 0; q0 < nr + npr; q0 += WAVE) {
            const int q = q0 + lane;
            const bool isr = q < nr, live = q < nr + npr;
            const int j = (isr || !live) ? 0 : invc[q - nr];
            // package j's row operands (gathered for every lane; robot lanes use their own)
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

}  // namespace mdl
