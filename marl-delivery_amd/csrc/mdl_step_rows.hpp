// mdl_step_rows.hpp -- the step kernel with FOUR ENVS PER WAVEFRONT, one per 16-lane DPP row
// (included by mdl_kernels.hip after k_step; same reference semantics, env.py:173-316,
// MAPPO/helper.py:257-369, MAPPO/trainer.py:95-130,211-259).
//
// Why: at the configs' A = 5 robots and P = 50 packages, k_step's one wave per env leaves most
// lanes idle in its serial sections and pays every scalar instruction (kernel prologue, branch and
// exec-mask handling, readlane chains, loop control) once per env.  The step is issue bound at
// every measured batch (profiles/r05: ~3 cycles per wave instruction per SIMD, 4096 to 131,072
// envs).  Here env r of the wave lives on lanes 16r..16r+15: robot a on row lane a (A <= AU <= 8),
// package j on row lane j & 15 of chunk j >> 4 (NC = 4 chunks, P <= 64; an eight-chunk form for
// P <= 128 measured slower than k_step at P = 100 and was removed, profiles/r05/rows_ab.txt).  Everything an env does is
// row-local: broadcasts are DPP row_newbcast (one VALU op, no SGPR), minima are four in-row DPP
// stages, a ballot's row part is one 64-bit vector shift -- and each of those instructions serves
// four envs.  The scalar instructions are shared by the four envs as well.
//
// Scope: full-batch steps (no env_ids), one step per launch, A <= 8, P <= 64; the one-wave-per-env
// k_step stays for everything else (subset stepping, the fused bench mode, the mailbox and
// step + observation launches, wider configs).  Results are bit-identical to k_step's
// (tests/test_gpu_step_rows.py steps both layouts side by side).
#pragma once

constexpr int ROW = 16;        // lanes per env
// package chunks per lane: NC = 4 (P <= 64), the only form built (a template parameter of the kernel)

// lane J of this lane's row, on every lane of the row (DPP row_newbcast, gfx90a+)
template <int J>
__device__ __forceinline__ int row_bcast(int v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x150 + J, 0xf, 0xf, false);
}
template <int J>
__device__ __forceinline__ float row_bcastf(float v) {
    return __int_as_float(row_bcast<J>(__float_as_int(v)));
}
// this lane's row of a wave mask (bits 16r..16r+15 -> 0..15); rbase = 16r
__device__ __forceinline__ uint32_t row_bits(uint64_t m, int rbase) { return (uint32_t)(m >> rbase) & 0xffffu; }
// the union over the four rows of a wave mask
__device__ __forceinline__ uint32_t rows_union(uint64_t m) { return (uint32_t)((m | (m >> 16) | (m >> 32) | (m >> 48)) & 0xffffull); }
// minimum over the row, on every lane of the row: xor 1, xor 2, then rotations by 4 and 8
// (row_ror:n: lane l reads row lane (l - n) & 15)
__device__ __forceinline__ uint32_t row_min_u32(uint32_t m) {
    const int id = (int)0xffffffff;
    uint32_t t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)m, 0xB1, 0xf, 0xf, false); m = t < m ? t : m;   // quad_perm 1,0,3,2
    t = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)m, 0x4E, 0xf, 0xf, false); m = t < m ? t : m;   // quad_perm 2,3,0,1
    t = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)m, 0x124, 0xf, 0xf, false); m = t < m ? t : m;  // row_ror:4
    t = (uint32_t)__builtin_amdgcn_update_dpp(id, (int)m, 0x128, 0xf, 0xf, false); m = t < m ? t : m;  // row_ror:8
    return m;
}
__device__ __forceinline__ uint32_t row_or_u32(uint32_t m) {
    m |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0xB1, 0xf, 0xf, false);
    m |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x4E, 0xf, 0xf, false);
    m |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x124, 0xf, 0xf, false);
    m |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x128, 0xf, 0xf, false);
    return m;
}

// numpy float32 add.reduce of the row's lanes 0..A-1 (A <= AU), on every lane of the row: the
// sequential n < 8 branch as a row_shr:1 chain (np_sum_lanes_dpp's argument: lanes A..AU-1 hold
// +0.0f, no lane holds -0.0f), numpy's 8-partial form when A == 8.
template <int AU>
__device__ __forceinline__ float row_np_sum(float v, int A) {
    static_assert(AU >= 1 && AU <= 8, "row_np_sum: AU <= 8");
    constexpr int L = AU < 8 ? AU : 7;
    if (AU == 8 && A == 8) {
        const float a = v + dppf<0xB1>(v);    // lanes 0, 2, 4, 6: x0+x1, x2+x3, x4+x5, x6+x7
        const float b = a + dppf<0x4E>(a);    // lanes 0, 4: (x0+x1)+(x2+x3), (x4+x5)+(x6+x7)
        const float c = b + dppf<0x124>(b);   // lane 4 (row_ror:4 reads lane l - 4): the two halves
        return 0.0f + row_bcastf<4>(c);
    }
    float t = v;
#pragma unroll
    for (int i = 1; i < L; i++) t = v + dppf<0x111>(t);   // row_shr:1 (lane 0 of the row reads +0)
    return row_bcastf<L - 1>(t);
}

// The carried package's fields a robot needs, gathered through LDS (one 16-byte record per
// package slot): its state word, env-table target | deadline << 16, tracker target | deadline << 16.
__device__ __forceinline__ uint32_t tgt_dl(uint64_t v) {
    return __builtin_amdgcn_perm((uint32_t)(v >> 32), (uint32_t)v, 0x07060302u);
}

// LDS bytes per wave: the gather records (4 chunks x 64 lanes x 16 B), then the 256 flag bytes;
// the reset scratch reuses the slice after both are consumed.
__host__ __device__ constexpr size_t rows_scratch_bytes(int NC) { return (size_t)NC * 64 * 16 + 64 * (size_t)NC; }
// where a resetting wave keeps its state words during the reset: the slice's last 512 bytes, past the
// reset scratch of P <= 64 packages (reset_lds_bytes(64) = 3,712 <= 3,840)
constexpr size_t ROWS_PS_STASH = rows_scratch_bytes(4) - 4 * 64 * 2;
// one flag byte per package slot, a lane's NC slots in one load
template <int NC> struct FlagWord;
template <> struct FlagWord<4> { typedef uint32_t T; };

// (93 VGPRs, 5 waves per SIMD.  Capping it at 6 waves (79 VGPRs) was 1 % faster on config 4 and 3-6 %
// slower at 4,096-16,384 envs, at 7 waves 20 % slower: profiles/r05/rows_ab.txt.)
// NFULL: package chunks known to be full (slot c * 16 + 15 < P for c < NFULL; 3 when P >= 48): their
// slots need no "no package" handling.
template <bool STALE, int AU, int NC, int NFULL>
__global__ __launch_bounds__(256) void k_step_rows(const uint32_t* __restrict__ rob_pre,
                                                   const uint64_t* __restrict__ pkg_pre,
                                                   const uint16_t* __restrict__ pst_pre,
                                                   const u32x4* __restrict__ es_pre,
                                                   const uint64_t* __restrict__ trk_pre,
                                                   const uint8_t* __restrict__ act_pre, uint32_t ap, uint32_t nw,
                                                   StepArgs args) {
    static_assert(AU >= 1 && AU <= 8, "k_step_rows: A <= 8");
    static_assert(NC == 4, "k_step_rows: P <= 64 (the only form built and tested)");
    constexpr uint32_t NONE = 255u;   // no package slot (slots < 16 * NC <= 128)
    extern __shared__ __align__(16) unsigned char smem[];
    const DevParams& p = args.p;
    const int A = (int)(ap & 0x7fu), P = (int)((ap >> 7) & 0x7ffu);
    const int n_ = (int)(nw & 0xffffffu), wpb_ = (int)((nw >> 24) & 31u);
    GLOBAL const uint32_t* robp = (GLOBAL const uint32_t*)rob_pre;
    GLOBAL const uint64_t* pkgp = (GLOBAL const uint64_t*)pkg_pre;
    GLOBAL const uint16_t* pstp = (GLOBAL const uint16_t*)pst_pre;
    GLOBAL const u32x4* esp = (GLOBAL const u32x4*)es_pre;
    GLOBAL const uint64_t* trkp = (GLOBAL const uint64_t*)trk_pre;
    GLOBAL const uint8_t* actp = (GLOBAL const uint8_t*)act_pre;

    const int wave = wave_id();
    const int lane = lane_id();
    const int nbp = (int)(ap >> AP_NB_SHIFT);
    const int w = (nbp ? xcd_slot((int)blockIdx.x, nbp) : (int)blockIdx.x) * wpb_ + wave;
    const int e0 = 4 * w;   // this wave's envs: e0 .. e0 + 3
    if (wave >= wpb_ || e0 >= n_) return;
    const int r = lane >> 4, rl = lane & 15, rbase = lane & 48;
    const bool live = e0 + r < n_;   // the last wave's rows past n hold no env ...
    const int re = live ? r : 0;     // ... and read env e0 (they store nothing)
    const bool act = live && rl < A;

    // ---- loads: one round trip, everything independent.  No exec-masked load blocks: every lane
    // loads (lanes without data read an in-bounds word of env e0 and discard it), so the loads
    // issue back to back with no branch and no wait between them. ----
    const uint32_t roff = (uint32_t)(r * A + rl);
    // (offsets masked to their range -- r * A + rl < 64, re * P + rl < 256 -- so the loads take the
    // scalar-base + 32-bit-offset form instead of a 64-bit address per lane; slot j = c * 16 + rl of
    // env e0 + re is element lb + 16 c, the chunks' byte offsets folded into the loads' immediates,
    // and lanes past P read the next env's slots or the 256-slot tail padding of the package
    // buffers, MdlEngine)
    const uint32_t roff_c = (act ? roff : 0u) & 0x3fu;
    const uint32_t rv_ld = (robp + (size_t)e0 * A)[roff_c];
    const uint32_t ar_ld = (actp + (size_t)e0 * A)[roff_c];
    uint64_t pk[NC], td[NC];
    uint32_t ps[NC], ps_in[NC];
    bool dirty[NC];
    GLOBAL const uint64_t* pkge = pkgp + (size_t)e0 * P;
    GLOBAL const uint16_t* pste = pstp + (size_t)e0 * P;
    GLOBAL const uint64_t* trke = trkp + (size_t)e0 * P;
    bool pv[NC];   // package slot c * 16 + rl of this row's env exists (the stores also test live)
    const uint32_t lb = (uint32_t)(re * P + rl) & 0xffu;
#pragma unroll
    for (int c = 0; c < NC; c++) {
        pv[c] = c < NFULL || c * ROW + rl < P;
        pk[c] = pkge[lb + c * ROW];
        ps[c] = pste[lb + c * ROW];
        td[c] = STALE ? trke[lb + c * ROW] : 0ull;
        dirty[c] = false;
    }
    // the env record's clock and total (its reward-term word is only written): two loads, so no
    // register of an unused component is recycled under a load still in flight (a forced wait)
    const uint32_t erow = (uint32_t)re & 3u;
    const uint32_t t_ld = ((GLOBAL const uint32_t*)(esp + e0))[4u * erow];
    const uint64_t tot_ld = ((GLOBAL const uint64_t*)(esp + e0))[2u * erow + 1u];
    // cost_fold[k] on row lane k (k <= A <= 8): the move-cost fold of the row's n_cost movers, fetched
    // by a row-local permute once n_cost is known
    KargPtr kap = (KargPtr)((__attribute__((address_space(4))) const char*)__builtin_amdgcn_kernarg_segment_ptr() +
                            offsetof(StepKarg, args));
    const double cst = kap->p.cost_fold[rl];
    __builtin_amdgcn_sched_barrier(0);   // every load above is issued before any use
    const uint32_t rv = act ? rv_ld : 0u;
    int araw = act ? (int)(ar_ld & 0xffu) : 0;
    const uint32_t t_rec = t_ld;
    const uint64_t tot_rec = tot_ld;
    // Slots without a package (j >= P, or a row past n) hold sentinels that fail every test by
    // themselves, so only the loads and the stores test the slot's existence: status delivered (the
    // all-delivered test passes over them; not waiting, not present), start time 0xffff (no spawn
    // or insert while t1 < 0xffff; past that only the stores' existence test keeps them out of
    // memory), start cell 0xffff (no cell of a map of at most 255 rows).
#pragma unroll
    for (int c = 0; c < NC; c++) {
        if (c >= NFULL) {
            pk[c] = pv[c] ? pk[c] : ~0ull;
            ps[c] = pv[c] ? ps[c] : (uint32_t)ST_DELIVERED;
            td[c] = pv[c] ? td[c] : ~0ull;
        }
        ps_in[c] = ps[c];
    }
    const int fmt = args.fmt, auto_reset = args.auto_reset, lds_stride = args.lds_stride;
    const int T = p.T;
    unsigned char* slice = smem + (size_t)wave * lds_stride;
    int mvoff = p.maps[0].mvc_off;
    int mi = 0;
    if (nw & NW_MAP) {   // mixed maps: each row's map, its move-validity table by a select chain
        mi = (int)((GLOBAL const uint8_t*)p.env_map)[e0 + re];
#pragma unroll
        for (int k = 1; k < MAX_MAPS; k++) mvoff = (mi == k) ? p.maps[k].mvc_off : mvoff;
    }
    int cell = rob_cell(rv), carry = rob_carry(rv);
    uint32_t vmask = rob_valid(rv);
    const int t0 = (int)t_rec;
    const double tot_cur = __hiloint2double((int)(uint32_t)(tot_rec >> 32), (int)(uint32_t)tot_rec);

    int mv, op;
    decode_action(araw, fmt, mv, op);
    mv = act ? mv : MV_S;
    op = act ? op : 0;
    uint32_t ps0[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) {
        ps0[c] = ps[c];
        if (!STALE || !(ps0[c] & PS_SURVIVOR)) td[c] = pk[c];
    }
    // tracker_prev's dict-order key of slot j: a survivor's rank, else ORD_EPISODE + j (stale mode),
    // recomputed where it is needed rather than held in registers across the step
    auto order_key = [&](uint32_t f, int j) -> uint32_t {
        return STALE ? ((f & PS_SURVIVOR) ? (f >> PS_RANK_SHIFT) : ORD_EPISODE + (uint32_t)j) : (uint32_t)j;
    };

    // ---- the shaped reward's pre-step part (MAPPO/helper.py:257-369): every agent's nearest waiting
    // package of tracker_prev, from its pre-step cell -- nothing here depends on this step's
    // movement or package actions, so these in-row minima are issued first and run alongside
    // those dependent chains.  Computed for all AU agents of all four rows (the terms below mask
    // the agents that do not need it); key = distance << 16 + (order << 7 | slot) in one
    // v_sad_hi_u8, the order (7 bits) a survivor's rank (< P <= 64) or 64 + slot as order_key ranks
    // them (the reference's tie-break); a real distance is <= 508 (cells are row << 8 | column, both
    // < 255), a non-candidate's (cell ~0) >= 510. ----
    int stc[NC], swv[NC];
    uint32_t klo[NC];   // order << 7 | row-local slot, or 0xffff for no candidate
    uint64_t anyw = 0;
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const uint32_t f = ps0[c];
        const bool waiting = STALE ? ((f & PS_PRESENT) && !(f & PS_TRANSIT)) : ((f & PS_STATUS) == ST_WAITING);
        const bool wv = waiting && pk_st(td[c]) <= t0;
        stc[c] = pk_start(td[c]);
        swv[c] = wv ? stc[c] : -1;
        const uint32_t j = (uint32_t)(c * ROW + rl);
        const uint32_t ord = STALE ? ((f & PS_SURVIVOR) ? (f >> PS_RANK_SHIFT) : 64u + j) : j;
        klo[c] = wv ? (ord << 7) | j : 0xffffu;
        anyw |= ballot(wv);
    }
    uint32_t Midle = 0;
    int best_cell = -1;
    if (anyw) {
        uint32_t kmin = 0xffffffffu;
#define MDL_NEAR(J)                                                                                  \
    if constexpr (J < AU) {                                                                          \
        const int pa = row_bcast<J>(cell);                                                           \
        uint32_t k = 0xffffffffu;                                                                    \
        _Pragma("unroll") for (int c = 0; c < NC; c++) {                                             \
            const uint32_t kc = __builtin_amdgcn_sad_hi_u8((uint32_t)pa, (uint32_t)swv[c], klo[c]);   \
            k = kc < k ? kc : k;                                                                     \
        }                                                                                            \
        k = row_min_u32(k);                                                                          \
        kmin = rl == J ? k : kmin;                                                                   \
    }
        MDL_NEAR(0) MDL_NEAR(1) MDL_NEAR(2) MDL_NEAR(3) MDL_NEAR(4) MDL_NEAR(5) MDL_NEAR(6) MDL_NEAR(7)
#undef MDL_NEAR
        const int js = (int)(kmin & 127u);
        const int sl = (rbase + (js & 15)) << 2;
        int bc = __builtin_amdgcn_ds_bpermute(sl, stc[0]);
#pragma unroll
        for (int c = 1; c < NC; c++) {
            const int v = __builtin_amdgcn_ds_bpermute(sl, stc[c]);
            bc = (js >> 4) == c ? v : bc;
        }
        const bool found = act && kmin < (509u << 16);
        Midle = lmask(found && (kmin >> 16) <= 3u);
        best_cell = found ? bc : -1;
    }

    // ---- the pre-step carried package of each robot, through LDS (read while the movement runs);
    // the flag bytes of the package actions (below) are cleared under the same wave barrier ----
    const int pj = carry - 1;
    u32x4* grec = (u32x4*)slice;
    unsigned char* flb = slice + NC * 64 * 16;   // byte (r, rl * NC + c) <-> package slot c * 16 + rl of row r
    typedef typename FlagWord<NC>::T FW;
#pragma unroll
    for (int c = 0; c < NC; c++) grec[c * 64 + lane] = u32x4{ps0[c], tgt_dl(pk[c]), tgt_dl(td[c]), 0u};
    ((FW*)flb)[lane] = 0;
    wave_sync();
    const u32x4 g = grec[((pj >> 4) & (NC - 1)) * 64 + rbase + (pj & 15)];
    const uint32_t g_pf = g.x, g_pk = g.y, g_td = g.z;

    // ---- movement (env.py:188-257): as k_step's AU > 0 form, row-local ----
    const int pcell = cell, pcarry = carry;
    constexpr uint64_t DTAB = (uint64_t)(0x3ffu & (uint32_t)-256) << 10 | (uint64_t)256 << 20 |
                              (uint64_t)(0x3ffu & (uint32_t)-1) << 30 | (uint64_t)1 << 40;
    const int dtab = __builtin_amdgcn_sbfe((int)(uint32_t)(DTAB >> (10 * mv)), 0, 10);
    const int vok = __builtin_amdgcn_sbfe((int)vmask, mv, 1);
    const int prop = cell + (int)(lmask(act) & (uint32_t)(dtab & vok));
    const bool mover = act && prop != cell;
    const uint64_t movers = ballot(mover);
    const uint32_t pvm = (uint32_t)(p.movevalid_cell + mvoff)[(uint32_t)prop];
    uint64_t moved = 0;
    if (movers) {
        const int propx = act ? prop : -2, cellx = act ? cell : -3;
        int pjs[AU], cjs[AU];
#define MDL_ROWB(J)                          \
    if constexpr (J < AU) {                  \
        pjs[J] = row_bcast<J>(propx);        \
        cjs[J] = row_bcast<J>(cellx);        \
    }
        MDL_ROWB(0) MDL_ROWB(1) MDL_ROWB(2) MDL_ROWB(3) MDL_ROWB(4) MDL_ROWB(5) MDL_ROWB(6) MDL_ROWB(7)
#undef MDL_ROWB
        uint32_t hit = 0;
        int occ = -1;
#pragma unroll
        for (int j = 0; j < AU; j++) {
            hit |= pjs[j] == prop ? (1u << j) : 0u;
            occ = cjs[j] == prop ? j : occ;
        }
        const bool blocked = (hit & ((1u << rl) - 1u) & row_bits(movers, rbase)) != 0u;
        const uint32_t Mbase = lmask(mover && !blocked), Mfree = lmask(occ < 0);
        moved = ballot((Mbase & Mfree) != 0u);
        if (ballot((Mbase & ~Mfree) != 0u)) {   // some walk into an occupied cell: resolve the chains
            const int oln = rbase + (occ & 15);
            for (int it = 0; it < A; it++) {
                const uint64_t nm = ballot((Mbase & (Mfree | vbit(moved, oln))) != 0u);
                if (nm == moved) break;
                moved = nm;
            }
        }
        if ((moved >> lane) & 1ull) cell = prop;
    }
    const int n_cost = (int)__popc(row_bits(moved, rbase));

    // ---- package actions (env.py:259-292) ----
    // Pick-ups: each picking robot takes the lowest-index waiting package at its cell.  Robots sit on
    // distinct cells, so their choices are independent of the reference's robot order; per robot
    // index J, one in-row minimum over the row's package slots answers robot J of all four envs.
    const bool picker = act && op == 1 && carry == 0;
    const uint64_t pickers = ballot(picker);
    int cnew = carry;
    if (pickers) {
        const uint32_t pu = rows_union(pickers);
        int sw[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) sw[c] = (ps[c] & PS_STATUS) == ST_WAITING ? pk_start(pk[c]) : -2;
#define MDL_PICK(J)                                                                                  \
    if constexpr (J < AU) {                                                                          \
        if (pu & (1u << J)) {                                                                        \
            const int ci = row_bcast<J>(cell);                                                       \
            uint32_t k = NONE;                                                                           \
            _Pragma("unroll") for (int c = NC - 1; c >= 0; c--) k = sw[c] == ci ? (uint32_t)(c * ROW + rl) : k; \
            k = row_min_u32(k);                                                                      \
            cnew = (rl == J && picker && k != NONE) ? (int)k + 1 : cnew;                             \
        }                                                                                            \
    }
        MDL_PICK(0) MDL_PICK(1) MDL_PICK(2) MDL_PICK(3) MDL_PICK(4) MDL_PICK(5) MDL_PICK(6) MDL_PICK(7)
#undef MDL_PICK
    }
    const bool picked = cnew != carry;
    carry = cnew;
    // drops: a robot with op 2 carrying a package (its pre-step one: it did not pick) and standing on
    // that package's target delivers it
    const int g_tgt = (int)(g_pk & 0xffffu), g_dl = (int)(g_pk >> 16);
    const bool drop = act && op == 2 && carry != 0 && g_tgt == cell;
    const uint64_t dmask = ballot(drop), omask = ballot(drop && t0 <= g_dl);
    // One flag byte per package slot, written by the robot concerned (each robot names at most one
    // slot, different robots different slots): picked (and now carried), delivered, carried.  The
    // package lanes read their NC slots' bytes in one word: the status changes and, for the
    // tracker update, the carried ids.
    // byte = the slot's new status (bits 0-1) | F_CHG (status changed) | F_CARRY (carried after the step)
    constexpr uint32_t F_CHG = 8u, F_CARRY = 4u;
    {
        const int fs = drop ? pj : carry - 1;
        const uint32_t fv = picked ? (F_CHG | F_CARRY | (uint32_t)ST_IN_TRANSIT)
                            : drop ? (F_CHG | (uint32_t)ST_DELIVERED) : F_CARRY;
        if (act && carry != 0) flb[(rbase + (fs & 15)) * NC + (fs >> 4)] = (unsigned char)fv;
    }
    carry = drop ? 0 : carry;
    wave_sync();
    const FW fw = ((const FW*)flb)[lane];
#pragma unroll
    for (int c = 0; c < NC; c++) {   // bit arithmetic, no branch: unchanged slots' bytes have status bits 0
        const uint32_t f = (uint32_t)(fw >> (8 * c));
        const uint32_t clr = (0u - ((f >> 3) & 1u)) & PS_STATUS;
        ps[c] = (ps[c] & ~clr) | (f & PS_STATUS);
    }
    // reward: fp64 fold in the reference's order (move costs, then deliveries in robot order)
    double rr;
    {
        const int src = (rbase + n_cost) << 2;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)__double2loint(cst));
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)__double2hiint(cst));
        rr = __hiloint2double((int)hi, (int)lo);
    }
    const uint32_t drow = row_bits(dmask, rbase), orow = row_bits(omask, rbase);
    if (dmask) {
        double DR = p.delivery_reward, DL = p.delay_reward;
        pin(DR);
        pin(DL);
        for (uint32_t u = rows_union(dmask); u; u &= u - 1) {
            const int i = __ffs((int)u) - 1;
            const double add = ((orow >> i) & 1u) ? DR : DL;
            rr = ((drow >> i) & 1u) ? rr + add : rr;
        }
    }
    const uint32_t rfl = (n_cost ? RT_MOVE : 0u) | (orow ? RT_ONTIME : 0u) | ((drow & ~orow) ? RT_LATE : 0u);
    const int t1 = t0 + 1;
    const double total = tot_cur + rr;

    // ---- terminate (env.py:308-316: every package delivered, or t == T) + spawn (get_state
    // env.py:133-137) ----
    uint32_t undel = 0;   // nonzero: some slot of this lane is not delivered (sentinel slots are)
    uint64_t spawned = 0;
#pragma unroll
    for (int c = 0; c < NC; c++) {
        undel |= (ps[c] & PS_STATUS) ^ (uint32_t)ST_DELIVERED;
        const bool sp = pk_st(pk[c]) == t1;
        spawned |= ballot(sp);
        ps[c] = sp ? ((ps[c] & ~PS_STATUS) | ST_WAITING) : ps[c];
    }
    // (no short-circuit: a ballot under a divergent branch costs exec juggling)
    const uint32_t alldel = lmask(row_bits(ballot(undel != 0u), rbase) == 0u);
    const bool done = (lmask(live) & (lmask(t1 == T) | alldel)) != 0u;

    // ---- shaped reward with the pre-step tracker (MAPPO/helper.py:257-369) ----
    float s_lane;
    {
        const uint32_t pf = g_pf;
        const uint32_t Mact = lmask(act), Mpc0 = lmask(pcarry == 0), Mc0 = lmask(carry == 0);
        const uint32_t Mpres =
            Mact & ~Mpc0 & lmask(pcarry <= P) &
            (STALE ? lmask((pf & PS_PRESENT) != 0)
                   : lmask((pf & PS_STATUS) == ST_WAITING) | lmask((pf & PS_STATUS) == ST_IN_TRANSIT));
        const uint32_t Mmov = lmask(pcell != cell), MS = lmask(mv == MV_S);
        const uint32_t Mop1 = lmask(op == 1), Mop2 = lmask(op == 2);
        const bool need_can = (Mact & Mop1 & Mpc0 & Mc0) != 0u;
        uint32_t Mcan = 0;
        if (anyw) {
            // can-pick-up: a waiting package starts at the agent's (new) cell
            if (ballot(need_can)) {
                uint32_t hm = 0;
#define MDL_CAN(J)                                                                                   \
    if constexpr (J < AU) {                                                                          \
        const int ca = row_bcast<J>(cell);                                                           \
        bool h = false;                                                                              \
        _Pragma("unroll") for (int c = 0; c < NC; c++) h = h | (swv[c] == ca);                   \
        hm |= h ? (1u << J) : 0u;                                                                    \
    }
                MDL_CAN(0) MDL_CAN(1) MDL_CAN(2) MDL_CAN(3) MDL_CAN(4) MDL_CAN(5) MDL_CAN(6) MDL_CAN(7)
#undef MDL_CAN
                hm = row_or_u32(hm);
                Mcan = ((hm >> rl) & 1u) ? ~0u : 0u;
            }
        }
        float cs[9];
#pragma unroll
        for (int k = 0; k < 9; k++) {
            cs[k] = p.shaping[k];
            pin(cs[k]);
        }
        const int ptg = (int)(g_td & 0xffffu), pdl = (int)(g_td >> 16);
        const uint32_t Mtg = lmask(cell == ptg);
        const uint32_t Mpick = Mpc0 & ~Mc0;
        const uint32_t Mdeliv = ~Mpc0 & Mc0 & Mpres & Mtg;
        const float t1v = fmask(Mpick, cs[SH_PICK]) + fmask(Mdeliv, fpick(lmask(t1 <= pdl), cs[SH_ONTIME], cs[SH_LATE]));
        const uint32_t Mwpick = Mop1 & (~Mpc0 | (Mc0 & ~Mcan));
        const uint32_t Mwdrop = Mop2 & (Mpc0 | (~Mc0 & Mpres & ~Mtg));
        const float t2v = fmask(Mwpick, cs[SH_WPICK]) + fmask(Mwdrop, cs[SH_WDROP]);
        const float t3v = fmask(~MS & ~Mmov, cs[SH_STUCK]);
        const int tgt = ipick(~Mpc0 & Mpres, ptg, best_cell);
        const int db = manhattan_sad(pcell, tgt), da = manhattan_sad(cell, tgt);
        const uint32_t Mt = lmask(tgt >= 0) & Mmov;
        const float t4v = fmask(Mt & lmask(da < db), cs[SH_CLOSER]) + fmask(Mt & lmask(da > db), cs[SH_AWAY]);
        const float t5v = fmask(~Mmov & MS & Mpc0 & Midle, cs[SH_IDLE]);
        float s = t1v;
        s = s + t2v;
        s = s + t3v;
        s = s + t4v;
        s = s + t5v;
        s_lane = fmask(Mact, s);
    }
    const float shaped = (float)rr + row_np_sum<AU>(s_lane, A);

    // ---- tracker update with the new state (MAPPO/trainer.py:95-130); rows that reset below
    // update with the reset state instead ----
    const bool do_rst = done && auto_reset;
    const uint64_t rst = ballot(do_rst);
    if (STALE && (ballot(picked) | dmask | spawned)) {
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const bool ins = !do_rst && (pk_st(pk[c]) == t1) && !(ps[c] & PS_PRESENT);
            ps[c] = ins ? ((ps[c] & PS_STATUS) | PS_PRESENT) : ps[c];
            td[c] = ins ? pk[c] : td[c];
            dirty[c] = dirty[c] || ins;
            // present entries: carried -> in transit; in transit and not carried -> deleted (status only)
            const uint32_t m_p = lmask((ps[c] & PS_PRESENT) != 0u && !do_rst);
            const uint32_t m_c = lmask(((uint32_t)(fw >> (8 * c)) & F_CARRY) != 0u);
            const uint32_t m_t = lmask((ps[c] & PS_TRANSIT) != 0u);
            ps[c] = (ps[c] | (PS_TRANSIT & m_c & m_p)) & (PS_STATUS | ~(m_p & ~m_c & m_t));
        }
    }

    // ---- outputs and write-back of the step (pointers fetched in one late scalar batch, as k_step).
    // A row that resets stores only its outputs and env record here: the reset below writes its rows
    // after these stores, so the package registers are dead while it runs (with the reset in the
    // middle, its path set the kernel's register count: 80 VGPRs and 26 SGPR spills, against 72 and
    // none for the step alone) ----
    const int t_out = do_rst ? 0 : t1;
    const double total_out = do_rst ? 0.0 : total;
    vmask = (((moved >> lane) & 1ull) && !do_rst) ? pvm : vmask;
    asm volatile("" : "+v"(vmask));
    GLOBAL double* rop = (GLOBAL double*)kap->r_out;
    GLOBAL float* shp = (GLOBAL float*)kap->sh_out;
    GLOBAL uint8_t* dnp = (GLOBAL uint8_t*)kap->done_out;
    GLOBAL uint32_t* robw = (GLOBAL uint32_t*)kap->p.rob;
    GLOBAL uint16_t* pstw = (GLOBAL uint16_t*)kap->p.pstate;
    GLOBAL uint64_t* trkw = (GLOBAL uint64_t*)kap->p.trk;
    GLOBAL u32x4* esw = (GLOBAL u32x4*)kap->p.es;
    // every store: a scalar row base (env e0's) + a 32-bit lane offset, one flat predicate each
    const uint32_t er = (uint32_t)r & 3u;
    if (live && rl == 0) {
        if (rop) (rop + e0)[er] = rr;
        if (shp) (shp + e0)[er] = shaped;
        if (dnp) (dnp + e0)[er] = done ? 1 : 0;
        (esw + e0)[er] = u32x4{(uint32_t)t_out, rfl, (uint32_t)__double2loint(total_out),
                               (uint32_t)__double2hiint(total_out)};
    }
    if (live && rl == 0 && done) {
        ((GLOBAL double*)p.ep_total + e0)[er] = total;
        ((GLOBAL int32_t*)p.ep_len + e0)[er] = t1;
    }
    if (act && !do_rst) (robw + (size_t)e0 * A)[roff] = rob_pack(cell, carry, vmask);
    const size_t eb = (size_t)e0 * P;
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const uint32_t o = lb + c * ROW;
        // Every store tests the slot's existence (pv: j < P in a live row).  A sentinel slot's start
        // time 0xffff equals t1 once a done env steps on without reset to t = 65535, which "spawns"
        // it (and inserts it into the stale tracker); its masked offset then names the next env's
        // slot, or lies past the allocation for the last env.  (k_step guards its stores with j < P.)
        // dirty marks inserts of this step, which a resetting row does not make.
        if (live && pv[c] && !do_rst && ps[c] != ps_in[c]) (pstw + eb)[o] = (uint16_t)ps[c];
        if (STALE && live && pv[c] && dirty[c]) (trkw + eb)[o] = td[c];
    }

    // ---- reset on done (MAPPO/trainer.py:230-235): one row at a time, by the whole wave; it writes
    // the row's robots, package table and state words (and the tracker's t = 0 inserts) ----
    if (rst) {
        GLOBAL uint64_t* pkgw = (GLOBAL uint64_t*)kap->p.pkg;
        wave_sync();   // the flag bytes and gather records are consumed (the reset scratch overlays them)
        for (uint64_t m = rst & 0x0001000100010001ull; m; m &= m - 1) {
            const int rb = ffs64(m);   // 16 * the resetting row
            const int er2 = e0 + (rb >> 4);
            const bool mine = rbase == rb;
            if (STALE) {
                // every present entry of the row becomes a survivor ranked by its current key
                uint32_t rk[NC], tq[NC];
#pragma unroll
                for (int c = 0; c < NC; c++) {
                    rk[c] = 0;
                    tq[c] = order_key(ps[c], c * ROW + rl);   // the key bits survive the step's updates
                }
#pragma unroll
                for (int c2 = 0; c2 < NC; c2++) {
                    uint64_t pm = ballot(c2 * ROW + rl < P && (ps[c2] & PS_PRESENT)) & (0xffffull << rb);
                    while (pm) {
                        const uint32_t ki = (uint32_t)rdl((int)tq[c2], ffs64(pm));
                        pm &= pm - 1;
#pragma unroll
                        for (int c = 0; c < NC; c++) rk[c] += ki < tq[c] ? 1u : 0u;
                    }
                }
#pragma unroll
                for (int c = 0; c < NC; c++) {
                    if (mine) {
                        if (c * ROW + rl < P && (ps[c] & PS_PRESENT)) {
                            ps[c] = (ps[c] & PS_FLAGS) | PS_SURVIVOR | (rk[c] << PS_RANK_SHIFT);
                        } else {
                            ps[c] &= PS_STATUS;
                        }
                    }
                }
            }
            // the state words wait in LDS past the reset scratch while the reset runs (registers,
            // not LDS, bound this kernel's occupancy)
            uint16_t* pss = (uint16_t*)(slice + ROWS_PS_STASH);
#pragma unroll
            for (int c = 0; c < NC; c++) pss[c * 64 + lane] = (uint16_t)ps[c];
            ResetLds L = reset_carve(slice, P);
            // the row's map by a scalar load (no per-lane map registers live across the reset)
            const int mr = (nw & NW_MAP) ? (int)((GLOBAL const uint8_t*)p.env_map)[er2] : 0;
            const MapDesc md = p.maps[mr];
            const int nc = do_reset(p, er2, md, L, false);   // robot a's cell on lane a
            const int ncr = __builtin_amdgcn_ds_bpermute(rl << 2, nc);
            if (mine && act)
                (robw + (size_t)e0 * A)[roff] = rob_pack(ncr, 0, p.movevalid_cell[(uint32_t)(md.mvc_off + ncr)]);
#pragma unroll
            for (int c = 0; c < NC; c++) ps[c] = pss[c * 64 + lane];
#pragma unroll
            for (int c = 0; c < NC; c++) {
                const int j = c * ROW + rl;
                if (mine && j < P) {
                    const uint64_t npk = L.pk[j];
                    uint32_t nps = (uint32_t)L.pst[j] | (STALE ? (ps[c] & ~PS_STATUS) : 0u);
                    const uint32_t o = (uint32_t)(r * P + j) & 0x1ffu;
                    if (STALE) {   // the update with the reset state: inserts at t = 0, nothing carried
                        const bool ins = (pk_st(npk) == 0) & !(nps & PS_PRESENT);
                        nps = ins ? ((nps & PS_STATUS) | PS_PRESENT) : nps;
                        if (ins) (trkw + eb)[o] = npk;
                        const uint32_t upd = (nps & PS_TRANSIT) ? (nps & PS_STATUS) : nps;
                        nps = (nps & PS_PRESENT) ? upd : nps;
                    }
                    (pkgw + eb)[o] = npk;
                    (pstw + eb)[o] = (uint16_t)nps;
                }
            }
            wave_sync();   // L is read by every lane before the next row's reset rewrites it
        }
    }
}
