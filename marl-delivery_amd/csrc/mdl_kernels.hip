// mdl_kernels.hip -- gfx950 kernels of the marl-delivery batched step engine.
//
//   k_seed       RandomState(seed) + the constructor's reset   env.py:40-41
//   k_reset      Environment.reset()                           env.py:81-125
//   k_step<S>    Environment.step + compute_shaped_rewards + tracker update
//                + reset-on-done                               env.py:173-316,
//                MAPPO/helper.py:257-369, MAPPO/trainer.py:95-130,211-257
//   k_obs<S>     convert_observation / generate_vector_features /
//                convert_global_state for every agent          MAPPO/helper.py:6-255
//   k_views_*    the same builders / shaping fed from packed dict views
//
// One wavefront per env; `wpb` envs per 256-thread workgroup, each with its
// own LDS slice of `lds_stride` bytes (dynamic shared memory).  Waves never
// block on each other, so a workgroup's envs may take different paths
// (e.g. one of them resetting).
#include "mdl_kernels.hpp"
#include "mdl_features.hpp"

namespace mdl {

// --------------------------------------------------------------- LDS carve
struct StepLds {
    uint64_t* pk;       // [P] package table
    uint64_t* scratch;  // [P] reset scratch
    uint64_t* tpk;      // [P] tracker data (stale)
    uint32_t* mt;       // [624]
    uint32_t* tseq;     // [P]
    uint16_t* taken;    // [64]
    uint8_t* pst;       // [P] status
    uint8_t* pst0;      // [P] status before the step (fresh tracker_prev)
    uint8_t* tflag;     // [P]
};

__host__ __device__ inline size_t step_lds_bytes(int P) {
    return align16(8 * (size_t)P) * 3 + align16(4 * MT_N) + align16(4 * (size_t)P) + align16(2 * 64) +
           align16((size_t)P) * 3;
}

__device__ inline StepLds step_carve(unsigned char* b, int P) {
    StepLds L;
    size_t o = 0;
    L.pk = (uint64_t*)(b + o); o += align16(8 * (size_t)P);
    L.scratch = (uint64_t*)(b + o); o += align16(8 * (size_t)P);
    L.tpk = (uint64_t*)(b + o); o += align16(8 * (size_t)P);
    L.mt = (uint32_t*)(b + o); o += align16(4 * MT_N);
    L.tseq = (uint32_t*)(b + o); o += align16(4 * (size_t)P);
    L.taken = (uint16_t*)(b + o); o += align16(2 * 64);
    L.pst = b + o; o += align16((size_t)P);
    L.pst0 = b + o; o += align16((size_t)P);
    L.tflag = b + o;
    return L;
}

// Tracker update with the current state (MAPPO/trainer.py:95-130), explicit
// per-id slots: insert ids spawned at t (state['packages']) that are absent,
// in id order; then carried -> in_transit, in_transit & not carried -> delete.
__device__ inline void stale_tracker_update(StepLds& L, int P, int A, int carry, int t, uint32_t& ctr) {
    const int lane = lane_id();
    for (int j0 = 0; j0 < P; j0 += WAVE) {
        const int j = j0 + lane;
        const bool ins = j < P && pk_st(L.pk[j]) == t && !(L.tflag[j] & 1);
        const uint64_t b = ballot(ins);
        if (ins) {
            L.tflag[j] = 1;
            L.tseq[j] = ctr + (uint32_t)popc64(b & lanemask_lt());
            L.tpk[j] = L.pk[j];
        }
        ctr += (uint32_t)popc64(b);
    }
    wave_sync();
    for (int j0 = 0; j0 < P; j0 += WAVE) {
        const int j = j0 + lane;
        bool carried = false;
        for (int i = 0; i < A; i++) carried |= rdl(carry, i) == j + 1;
        if (j < P) {
            const uint8_t f = L.tflag[j];
            if (f & 1) {
                if (carried) L.tflag[j] = 3;
                else if (f & 2) L.tflag[j] = 0;
            }
        }
    }
    wave_sync();
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

// Write robots / packages / statuses / clock after a reset (or seed).
__device__ inline void store_layout(const DevParams& p, int e, const StepLds& L, int cell) {
    const int lane = lane_id();
    if (lane < p.A) {
        p.rob[(size_t)e * p.A + lane] = (uint16_t)cell;
        p.carry[(size_t)e * p.A + lane] = 0;
    }
    for (int j = lane; j < p.P; j += WAVE) {
        p.pkg[(size_t)e * p.P + j] = L.pk[j];
        p.status[(size_t)e * p.P + j] = L.pst[j];
    }
    if (lane == 0) {
        p.t[e] = 0;
        p.total[e] = 0.0;
    }
}

__device__ inline void load_tracker(const DevParams& p, int e, StepLds& L) {
    for (int j = lane_id(); j < p.P; j += WAVE) {
        const size_t g = (size_t)e * p.P + j;
        L.tflag[j] = p.trk_flag[g];
        L.tseq[j] = p.trk_seq[g];
        L.tpk[j] = p.trk_pkg[g];
    }
    wave_sync();
}

__device__ inline void store_tracker(const DevParams& p, int e, const StepLds& L, uint32_t ctr) {
    for (int j = lane_id(); j < p.P; j += WAVE) {
        const size_t g = (size_t)e * p.P + j;
        p.trk_flag[g] = L.tflag[j];
        p.trk_seq[g] = L.tseq[j];
        p.trk_pkg[g] = L.tpk[j];
    }
    if (lane_id() == 0) p.trk_ctr[e] = ctr;
}

// ------------------------------------------------------------------ seed
__global__ __launch_bounds__(256) void k_seed(DevParams p, const uint32_t* __restrict__ seeds, int wpb,
                                              int lds_stride) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = threadIdx.x >> 6;
    const int e = blockIdx.x * wpb + wave;
    if (wave >= wpb || e >= p.E) return;
    StepLds L = step_carve(smem + (size_t)wave * lds_stride, p.P);
    const MapDesc md = p.maps[p.env_map ? p.env_map[e] : 0];
    if (lane_id() == 0) {  // init_genrand: a serial recurrence
        uint32_t s = seeds[e];
        for (int i = 0; i < MT_N; i++) {
            L.mt[i] = s;
            s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
        }
    }
    wave_sync();
    MTState ms{L.mt, MT_N};
    const int cell = reset_env(ms, p, md, L.pk, L.pst, L.scratch, L.taken);
    store_layout(p, e, L, cell);
    store_mt(p, e, L.mt, ms.pos);
    if (p.stale) {  // the trainer's dict starts empty (MAPPO/trainer.py:92)
        for (int j = lane_id(); j < p.P; j += WAVE) {
            const size_t g = (size_t)e * p.P + j;
            p.trk_flag[g] = 0;
            p.trk_seq[g] = 0;
            p.trk_pkg[g] = 0;
        }
        if (lane_id() == 0) p.trk_ctr[e] = 0;
    }
    if (lane_id() == 0) {
        p.ep_total[e] = 0.0;
        p.ep_len[e] = 0;
    }
}

// ------------------------------------------------------------------ reset
__global__ __launch_bounds__(256) void k_reset(DevParams p, const int* __restrict__ env_ids, int n, int wpb,
                                               int lds_stride) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = threadIdx.x >> 6;
    const int w = blockIdx.x * wpb + wave;
    if (wave >= wpb || w >= n) return;
    const int e = env_ids ? env_ids[w] : w;
    StepLds L = step_carve(smem + (size_t)wave * lds_stride, p.P);
    const MapDesc md = p.maps[p.env_map ? p.env_map[e] : 0];
    load_mt(p, e, L.mt);
    MTState ms{L.mt, p.mt_pos[e]};
    const int cell = reset_env(ms, p, md, L.pk, L.pst, L.scratch, L.taken);
    store_layout(p, e, L, cell);
    store_mt(p, e, L.mt, ms.pos);
    if (p.stale) {
        load_tracker(p, e, L);
        uint32_t ctr = p.trk_ctr[e];
        stale_tracker_update(L, p.P, p.A, 0, 0, ctr);
        store_tracker(p, e, L, ctr);
    }
}

__global__ __launch_bounds__(256) void k_tracker_clear(DevParams p, const int* __restrict__ env_ids, int n) {
    const int wave = threadIdx.x >> 6;
    const int w = blockIdx.x * 4 + wave;
    if (w >= n) return;
    const int e = env_ids ? env_ids[w] : w;
    for (int j = lane_id(); j < p.P; j += WAVE) {
        const size_t g = (size_t)e * p.P + j;
        p.trk_flag[g] = 0;
    }
    if (lane_id() == 0) p.trk_ctr[e] = 0;
}

// ------------------------------------------------------------------- step
template <bool STALE>
__global__ __launch_bounds__(256) void k_step(DevParams p, const uint8_t* __restrict__ actions, int fmt,
                                              const int* __restrict__ env_ids, int n, int auto_reset,
                                              double* __restrict__ r_out, float* __restrict__ sh_out,
                                              uint8_t* __restrict__ done_out, int wpb, int lds_stride) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = threadIdx.x >> 6;
    const int lane = lane_id();
    const int w = blockIdx.x * wpb + wave;
    if (wave >= wpb || w >= n) return;
    const int e = env_ids ? env_ids[w] : w;
    const int A = p.A, P = p.P;
    StepLds L = step_carve(smem + (size_t)wave * lds_stride, P);
    const MapDesc md = p.maps[p.env_map ? p.env_map[e] : 0];
    const int H = md.H, W = md.W;
    const uint8_t* grid = p.grids + md.grid_off;

    // ---- load (robots on lanes, packages into LDS) ----
    const bool act = lane < A;
    const int t0 = p.t[e];
    int cell = act ? (int)p.rob[(size_t)e * A + lane] : 0;
    int carry = act ? (int)p.carry[(size_t)e * A + lane] : 0;
    int mv = MV_S, op = 0;
    if (act) decode_action(actions[(size_t)w * A + lane], fmt, mv, op);
    for (int j = lane; j < P; j += WAVE) {
        const size_t g = (size_t)e * P + j;
        L.pk[j] = p.pkg[g];
        const uint8_t s = p.status[g];
        L.pst[j] = s;
        L.pst0[j] = s;
        if (STALE) {
            L.tflag[j] = p.trk_flag[g];
            L.tseq[j] = p.trk_seq[g];
            L.tpk[j] = p.trk_pkg[g];
        }
    }
    wave_sync();

    // ---- movement (env.py:188-257) ----
    // moved = least fixed point of
    //   moved[i] = mover[i] & winner(prop[i]) == i & (occ(prop[i]) none | moved[occ])
    // winner = lowest-index mover into the cell; equivalent to the reference's
    // restart-from-zero loop (checked against the oracle's literal
    // restatement of that loop).
    const int prev_cell = cell, prev_carry = carry;
    int prop = cell;
    {
        int nr = cell_r(cell), nc = cell_c(cell);
        if (mv == MV_L) nc -= 1;
        else if (mv == MV_R) nc += 1;
        else if (mv == MV_U) nr -= 1;
        else if (mv == MV_D) nr += 1;
        if (nr >= 0 && nr < H && nc >= 0 && nc < W && grid[nr * W + nc] != 1) prop = nr | (nc << 8);
    }
    const bool mover = act && prop != cell;
    const uint64_t movers = ballot(mover);
    bool win = true;
    int occ = -1;
    for (int j = 0; j < A; j++) {
        const int pj = rdl(cell, j), qj = rdl(prop, j);
        if (j < lane && ((movers >> j) & 1) && qj == prop) win = false;
        if (pj == prop) occ = j;
    }
    uint64_t moved = 0;
    for (int it = 0; it <= A; it++) {
        const bool m = mover && win && (occ < 0 || ((moved >> occ) & 1ull));
        const uint64_t nm = ballot(m);
        if (nm == moved) break;
        moved = nm;
    }
    if ((moved >> lane) & 1ull) cell = prop;
    const int n_cost = popc64(moved);

    // ---- package actions (env.py:259-292) ----
    uint64_t pickers = ballot(act && op == 1 && carry == 0);
    while (pickers) {
        const int i = ffs64(pickers);
        pickers &= pickers - 1;
        const int ci = rdl(cell, i);
        int found = -1;
        for (int j0 = 0; j0 < P; j0 += WAVE) {
            const int j = j0 + lane;
            const bool cand = j < P && L.pst[j] == ST_WAITING && pk_start(L.pk[j]) == ci;
            const uint64_t b = ballot(cand);
            if (b) {
                found = j0 + ffs64(b);
                break;
            }
        }
        if (found >= 0) {
            if (lane == i) carry = found + 1;
            if (lane == 0) L.pst[found] = ST_IN_TRANSIT;
        }
    }
    wave_sync();
    bool at_tgt = false, ontime = false;
    if (act && op == 2 && carry != 0) {
        const uint64_t d = L.pk[carry - 1];
        if (pk_target(d) == cell) {
            at_tgt = true;
            ontime = t0 <= pk_dl(d);
            L.pst[carry - 1] = ST_DELIVERED;
            carry = 0;
        }
    }
    const uint64_t dmask = ballot(at_tgt), omask = ballot(ontime);
    wave_sync();
    // reward: fp64 fold in the reference's order (move costs, then deliveries)
    double rr = 0.0;
    for (int k = 0; k < n_cost; k++) rr += p.move_cost;
    for (uint64_t m = dmask; m; m &= m - 1) {
        const int i = ffs64(m);
        rr += ((omask >> i) & 1ull) ? p.delivery_reward : p.delay_reward;
    }
    const int t1 = t0 + 1;
    const double total = p.total[e] + rr;

    // ---- terminate (env.py:308-316) + spawn (get_state env.py:133-137) ----
    int ndel = 0;
    for (int j0 = 0; j0 < P; j0 += WAVE) {
        const int j = j0 + lane;
        bool dv = false;
        if (j < P) {
            dv = L.pst[j] == ST_DELIVERED;
            if (pk_st(L.pk[j]) == t1) L.pst[j] = ST_WAITING;
        }
        ndel += popc64(ballot(dv));
    }
    const bool done = (t1 == p.T) || (ndel == P);
    wave_sync();

    // ---- shaped reward with the pre-step tracker (MAPPO/trainer.py:211-218) ----
    float s_a;
    if (STALE) {
        TrkStale trk{L.tflag, L.tseq, L.tpk, P};
        s_a = shaped_agent(trk, p.shaping, act, prev_cell, prev_carry, cell, carry, mv, op, t0, t1);
    } else {
        TrkFresh trk{L.pk, L.pst0, P};
        s_a = shaped_agent(trk, p.shaping, act, prev_cell, prev_carry, cell, carry, mv, op, t0, t1);
    }
    const float shaped = (float)rr + np_sum_lanes(s_a, A);

    // ---- tracker update with the new state; a done env that is reset here
    // skips it and updates with the reset state instead (MAPPO/trainer.py:230-259) ----
    uint32_t ctr = 0;
    if (STALE) {
        ctr = p.trk_ctr[e];
        if (!(done && auto_reset)) stale_tracker_update(L, P, A, carry, t1, ctr);
    }

    // ---- reset on done (MAPPO/trainer.py:230-235) ----
    int t_out = t1;
    double total_out = total;
    bool did_reset = false;
    if (done && auto_reset) {
        load_mt(p, e, L.mt);
        MTState ms{L.mt, p.mt_pos[e]};
        const int nc = reset_env(ms, p, md, L.pk, L.pst, L.scratch, L.taken);
        store_mt(p, e, L.mt, ms.pos);
        if (act) {
            cell = nc;
            carry = 0;
        }
        t_out = 0;
        total_out = 0.0;
        did_reset = true;
        if (STALE) stale_tracker_update(L, P, A, 0, 0, ctr);  // tracker NOT cleared (trainer.py:233)
    }

    // ---- write back ----
    if (act) {
        p.rob[(size_t)e * A + lane] = (uint16_t)cell;
        p.carry[(size_t)e * A + lane] = (uint16_t)carry;
    }
    for (int j = lane; j < P; j += WAVE) {
        const size_t g = (size_t)e * P + j;
        p.status[g] = L.pst[j];
        if (did_reset) p.pkg[g] = L.pk[j];
        if (STALE) {
            p.trk_flag[g] = L.tflag[j];
            p.trk_seq[g] = L.tseq[j];
            p.trk_pkg[g] = L.tpk[j];
        }
    }
    if (lane == 0) {
        p.t[e] = t_out;
        p.total[e] = total_out;
        if (STALE) p.trk_ctr[e] = ctr;
        if (done) {
            p.ep_total[e] = total;
            p.ep_len[e] = t1;
        }
        if (r_out) r_out[w] = rr;
        if (sh_out) sh_out[w] = shaped;
        if (done_out) done_out[w] = done ? 1 : 0;
    }
}

// ------------------------------------------------------------- observations
struct ObsLdsPre {
    uint64_t* pk;
    uint64_t* tpk;
    uint32_t* tseq;
    uint8_t* pst;
    uint8_t* tflag;
};

__host__ __device__ inline size_t obs_pre_bytes(int P) {
    return align16(8 * (size_t)P) * 2 + align16(4 * (size_t)P) + align16((size_t)P) * 2;
}

template <bool STALE>
__global__ __launch_bounds__(256) void k_obs(DevParams p, int env_begin, int n, float* __restrict__ amap,
                                             float* __restrict__ avec, float* __restrict__ cmap,
                                             float* __restrict__ cvec, int wpb, int lds_stride) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = threadIdx.x >> 6;
    const int lane = lane_id();
    const int w = blockIdx.x * wpb + wave;
    if (wave >= wpb || w >= n) return;
    const int e = env_begin + w;
    const int A = p.A, P = p.P;
    unsigned char* base = smem + (size_t)wave * lds_stride;
    ObsLdsPre S;
    {
        size_t o = 0;
        S.pk = (uint64_t*)(base + o); o += align16(8 * (size_t)P);
        S.tpk = (uint64_t*)(base + o); o += align16(8 * (size_t)P);
        S.tseq = (uint32_t*)(base + o); o += align16(4 * (size_t)P);
        S.pst = base + o; o += align16((size_t)P);
        S.tflag = base + o; o += align16((size_t)P);
    }
    const MapDesc md = p.maps[p.env_map ? p.env_map[e] : 0];
    FeatCtx c;
    c.A = A; c.NS = P; c.H = md.H; c.W = md.W; c.HW = md.H * md.W; c.t = p.t[e]; c.T = p.obsT;
    c.MO = p.MO; c.MP = p.MP; c.MR = p.MR; c.MPs = p.MPs;
    c.MPc = p.MP < P ? p.MP : P;
    c.MPsc = p.MPs < P ? p.MPs : P;
    c.grid = p.grids + md.grid_off;
    c.rank = p.rank + md.rank_off;
    c.inv_hw = md.inv_hw;
    FeatDims fd{A, P, c.HW, c.MPc, c.MPsc};
    FeatLds L = feat_carve(base + obs_pre_bytes(P), fd);

    const bool act = lane < A;
    const int cell = act ? (int)p.rob[(size_t)e * A + lane] : 0;
    const int carry = act ? (int)p.carry[(size_t)e * A + lane] : 0;
    for (int j = lane; j < P; j += WAVE) {
        const size_t g = (size_t)e * P + j;
        if (STALE) {
            S.tflag[j] = p.trk_flag[g];
            S.tseq[j] = p.trk_seq[g];
            S.tpk[j] = p.trk_pkg[g];
        } else {
            S.pk[j] = p.pkg[g];
            S.pst[j] = p.status[g];
        }
    }
    wave_sync();
    auto run = [&](const auto& trk) {
        feat_prepare(trk, c, L, cell, carry);
        const size_t le = (size_t)w;
        if (amap) emit_actor_maps(c, L, 0, A, true, amap + le * (size_t)A * 6 * c.HW);
        if (cmap) emit_critic_map(c, L, cmap + le * 4 * (size_t)c.HW);
        if (avec) {
            for (int a = 0; a < A; a++) feat_sort_agent(trk, c, L, a, cell);
            const int Dv = 6 + 5 * c.MO + 5 * c.MP + 1;
            emit_actor_vecs(trk, c, L, 0, A, true, avec + le * (size_t)A * Dv);
        }
        if (cvec) {
            const int Dg = 6 * c.MR + 7 * c.MPs + 1;
            emit_critic_vec(trk, c, L, cvec + le * (size_t)Dg);
        }
    };
    if (STALE) {
        TrkStale trk{S.tflag, S.tseq, S.tpk, P};
        run(trk);
    } else {
        TrkFresh trk{S.pk, S.pst, P};
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

__global__ __launch_bounds__(256) void k_views_features(DevParams p, const int32_t* __restrict__ views,
                                                        const int64_t* __restrict__ offs, int n,
                                                        const int32_t* __restrict__ agent_idx, int T, int MO, int MP,
                                                        int MR, int MPs, int MPc, int MPsc, int NSmax,
                                                        float* __restrict__ obs, float* __restrict__ vec,
                                                        float* __restrict__ gmap, float* __restrict__ gvec, int wpb,
                                                        int lds_stride, int HW) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = threadIdx.x >> 6;
    const int w = blockIdx.x * wpb + wave;
    if (wave >= wpb || w >= n) return;
    unsigned char* base = smem + (size_t)wave * lds_stride;
    ViewLdsPre V;
    {
        const int nsm = NSmax > 0 ? NSmax : 1;
        size_t o = 0;
        V.ids = (int32_t*)(base + o); o += align16(4 * (size_t)nsm);
        V.pk = (uint64_t*)(base + o); o += align16(8 * (size_t)nsm);
        V.flag = base + o;
    }
    int t, A, map, cell, carry;
    const TrkView trk = load_view(views + offs[w], V, t, A, map, cell, carry);
    const MapDesc md = p.maps[map];
    FeatCtx c;
    c.A = A; c.NS = trk.n; c.H = md.H; c.W = md.W; c.HW = md.H * md.W; c.t = t; c.T = T;
    c.MO = MO; c.MP = MP; c.MR = MR; c.MPs = MPs; c.MPc = MPc; c.MPsc = MPsc;
    c.grid = p.grids + md.grid_off;
    c.rank = p.rank + md.rank_off;
    c.inv_hw = md.inv_hw;
    FeatDims fd{64, NSmax, HW, MPc, MPsc};
    FeatLds L = feat_carve(base + view_pre_bytes(NSmax), fd);
    feat_prepare(trk, c, L, cell, carry);
    const int a = agent_idx ? agent_idx[w] : 0;
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

__global__ __launch_bounds__(256) void k_views_shaped(DevParams p, const int32_t* __restrict__ prev,
                                                      const int64_t* __restrict__ prev_offs,
                                                      const int32_t* __restrict__ cur,
                                                      const int64_t* __restrict__ cur_offs,
                                                      const uint8_t* __restrict__ acts,
                                                      const int64_t* __restrict__ act_offs,
                                                      const double* __restrict__ g, int n, ShapingConsts C,
                                                      float* __restrict__ out, int wpb, int lds_stride, int NSmax) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int wave = threadIdx.x >> 6;
    const int lane = lane_id();
    const int w = blockIdx.x * wpb + wave;
    if (wave >= wpb || w >= n) return;
    unsigned char* base = smem + (size_t)wave * lds_stride;
    ViewLdsPre V;
    {
        const int nsm = NSmax > 0 ? NSmax : 1;
        size_t o = 0;
        V.ids = (int32_t*)(base + o); o += align16(4 * (size_t)nsm);
        V.pk = (uint64_t*)(base + o); o += align16(8 * (size_t)nsm);
        V.flag = base + o;
    }
    int t_prev, A, map, pcell, pcarry;
    const TrkView trk = load_view(prev + prev_offs[w], V, t_prev, A, map, pcell, pcarry);
    const int32_t* cr = cur + cur_offs[w];
    const int t_cur = cr[0];
    const bool act = lane < A;
    int ccell = 0, ccarry = 0, mv = MV_S, op = 0;
    if (act) {
        ccell = cr[2 + 3 * lane] | (cr[3 + 3 * lane] << 8);
        ccarry = cr[4 + 3 * lane];
        decode_action(acts[act_offs[w] + lane], 1, mv, op);
    }
    const float s_a = shaped_agent(trk, C.c, act, pcell, pcarry, ccell, ccarry, mv, op, t_prev, t_cur);
    const float res = (float)g[w] + np_sum_lanes(s_a, A);
    if (lane == 0) out[w] = res;
}

// ------------------------------------------------------------ state export
// int32 views of the SoA state for the dict-compat layer and the tests.
__global__ __launch_bounds__(256) void k_export(DevParams p, int32_t* __restrict__ robots, int32_t* __restrict__ pkgs,
                                                int32_t* __restrict__ tt, double* __restrict__ total,
                                                int32_t* __restrict__ trk, int32_t* __restrict__ trk_data) {
    const int wave = threadIdx.x >> 6;
    const int lane = lane_id();
    const int e = blockIdx.x * 4 + wave;
    if (e >= p.E) return;
    const int A = p.A, P = p.P;
    if (robots && lane < A) {
        const int c = p.rob[(size_t)e * A + lane];
        int32_t* o = robots + ((size_t)e * A + lane) * 3;
        o[0] = cell_r(c);
        o[1] = cell_c(c);
        o[2] = p.carry[(size_t)e * A + lane];
    }
    for (int j = lane; j < P; j += WAVE) {
        const size_t g = (size_t)e * P + j;
        const uint64_t d = p.pkg[g];
        const int st = p.status[g];
        if (pkgs) {
            int32_t* o = pkgs + g * 8;
            o[0] = cell_r(pk_start(d)); o[1] = cell_c(pk_start(d));
            o[2] = cell_r(pk_target(d)); o[3] = cell_c(pk_target(d));
            o[4] = pk_st(d); o[5] = pk_dl(d); o[6] = j + 1; o[7] = st;
        }
        int present, intr, order;
        uint64_t td;
        if (p.stale) {
            const int f = p.trk_flag[g];
            present = f & 1; intr = (f >> 1) & 1; order = (int)p.trk_seq[g]; td = p.trk_pkg[g];
        } else {
            present = st == ST_WAITING || st == ST_IN_TRANSIT; intr = st == ST_IN_TRANSIT; order = j; td = d;
        }
        if (trk) {
            int32_t* o = trk + g * 4;
            o[0] = present; o[1] = intr; o[2] = order; o[3] = 0;
        }
        if (trk_data) {
            int32_t* o = trk_data + g * 6;
            o[0] = cell_r(pk_start(td)); o[1] = cell_c(pk_start(td));
            o[2] = cell_r(pk_target(td)); o[3] = cell_c(pk_target(td));
            o[4] = pk_st(td); o[5] = pk_dl(td);
        }
    }
    if (lane == 0) {
        if (tt) tt[e] = p.t[e];
        if (total) total[e] = p.total[e];
    }
}

// ---------------------------------------------------------------- launchers
static int blocks_for(int n, int wpb) { return (n + wpb - 1) / wpb; }

hipError_t launch_seed(const DevParams& p, const uint32_t* seeds, int wpb, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL(k_seed, dim3(blocks_for(p.E, wpb)), dim3(256), lds * wpb, s, p, seeds, wpb, (int)lds);
    return hipGetLastError();
}

hipError_t launch_reset(const DevParams& p, const int* ids, int n, int wpb, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL(k_reset, dim3(blocks_for(n, wpb)), dim3(256), lds * wpb, s, p, ids, n, wpb, (int)lds);
    return hipGetLastError();
}

hipError_t launch_tracker_clear(const DevParams& p, const int* ids, int n, hipStream_t s) {
    hipLaunchKernelGGL(k_tracker_clear, dim3(blocks_for(n, 4)), dim3(256), 0, s, p, ids, n);
    return hipGetLastError();
}

hipError_t launch_step(const DevParams& p, const uint8_t* actions, int fmt, const int* ids, int n, int auto_reset,
                       double* r, float* sh, uint8_t* done, int wpb, size_t lds, hipStream_t s) {
    if (p.stale)
        hipLaunchKernelGGL(k_step<true>, dim3(blocks_for(n, wpb)), dim3(256), lds * wpb, s, p, actions, fmt, ids, n,
                           auto_reset, r, sh, done, wpb, (int)lds);
    else
        hipLaunchKernelGGL(k_step<false>, dim3(blocks_for(n, wpb)), dim3(256), lds * wpb, s, p, actions, fmt, ids,
                           n, auto_reset, r, sh, done, wpb, (int)lds);
    return hipGetLastError();
}

hipError_t launch_obs(const DevParams& p, int env_begin, int n, float* amap, float* avec, float* cmap, float* cvec,
                      int wpb, size_t lds, hipStream_t s) {
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
                                 size_t lds, hipStream_t s) {
    hipLaunchKernelGGL(k_views_features, dim3(blocks_for(n, wpb)), dim3(256), lds * wpb, s, p, views, offs, n,
                       agent_idx, T, MO, MP, MR, MPs, MPc, MPsc, NSmax, obs, vec, gmap, gvec, wpb, (int)lds, HW);
    return hipGetLastError();
}

hipError_t launch_views_shaped(const DevParams& p, const int32_t* prev, const int64_t* prev_offs, const int32_t* cur,
                               const int64_t* cur_offs, const uint8_t* acts, const int64_t* act_offs, const double* g,
                               int n, const ShapingConsts& C, float* out, int wpb, size_t lds, int NSmax,
                               hipStream_t s) {
    hipLaunchKernelGGL(k_views_shaped, dim3(blocks_for(n, wpb)), dim3(256), lds * wpb, s, p, prev, prev_offs, cur,
                       cur_offs, acts, act_offs, g, n, C, out, wpb, (int)lds, NSmax);
    return hipGetLastError();
}

hipError_t launch_export(const DevParams& p, int32_t* robots, int32_t* pkgs, int32_t* t, double* total,
                         int32_t* tracker, int32_t* tracker_data, hipStream_t s) {
    hipLaunchKernelGGL(k_export, dim3(blocks_for(p.E, 4)), dim3(256), 0, s, p, robots, pkgs, t, total, tracker,
                       tracker_data);
    return hipGetLastError();
}

size_t step_lds(int P) { return step_lds_bytes(P); }
size_t obs_lds(int A, int P, int HW, int MP, int MPs) {
    FeatDims d{A, P, HW, MP < P ? MP : P, MPs < P ? MPs : P};
    return obs_pre_bytes(P) + feat_lds_bytes(d);
}
size_t views_lds(int NSmax, int HW, int MPc, int MPsc) {
    FeatDims d{64, NSmax, HW, MPc, MPsc};
    return view_pre_bytes(NSmax) + feat_lds_bytes(d);
}
size_t views_shaped_lds(int NSmax) { return view_pre_bytes(NSmax); }

}  // namespace mdl
