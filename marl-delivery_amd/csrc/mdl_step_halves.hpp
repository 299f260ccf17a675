// mdl_step_halves.hpp -- the step kernel with TWO ENVS PER WAVEFRONT, one per 32-lane half, for
// the eight-to-sixteen-robot configurations (8 <= A <= 16, P <= 128: BASELINE config 5's 16 robots
// and 100 packages).  Included by mdl_kernels.hip after mdl_step_rows.hpp; same reference semantics
// (env.py:173-316, MAPPO/helper.py:257-369, MAPPO/trainer.py:95-130,211-259).
//
// Why: k_step<.., 16> runs one env per wave and is issue bound at config 5's 131,072 envs (~395
// VALU + ~264 SALU per wave at 128 waves per SIMD; profiles/r05 prices each wave instruction at ~3
// cycles per SIMD there).  Its scalar work (prologue, loop control, exec handling, ballots and
// their SALU follow-up) and every cross-lane operation serve one env.  Here env h of the wave lives
// on lanes 32h..32h+31:
//   * robot a on lanes 32h + a AND 32h + 16 + a (both 16-lane rows of the half hold every robot and
//     compute the same robot values, so a robot's data is a row-local DPP broadcast away from every
//     lane of its half, and no value has to cross the rows);
//   * package j on half-lane j & 31 of chunk j >> 5 (NC = 4 chunks, P <= 128);
//   * a minimum over the half is four in-row DPP stages plus one v_permlane16_swap (rows 0 <-> 1,
//     2 <-> 3) and a min.
// Every scalar instruction and every ballot serves both envs.  The shaped reward's nearest waiting
// package keeps k_step's compacted candidate scan, per half: each half packs its waiting candidates
// into its own LDS list and the two rows of a half scan alternate candidates for the same agent.
//
// Scope: full-batch steps (no env_ids), one step per launch; k_step stays for everything else.
// Results are bit-identical to k_step's (tests/test_gpu_step_halves.py steps both layouts side by
// side and compares every output and the whole saved state).
#pragma once

constexpr int HALF = 32;                 // lanes per env
constexpr int HALF_NC = 4;               // package chunks per lane: P <= 128
constexpr int HALF_CAND = 136;           // candidate slots per half (<= 128 candidates, padded to a multiple of 4)

// minimum over the 32 lanes of this lane's half, on every lane of the half
__device__ __forceinline__ uint32_t half_min_u32(uint32_t m) {
    m = row_min_u32(m);
    const auto r = __builtin_amdgcn_permlane16_swap(m, m, false, false);   // [r0, r0, r2, r2], [r1, r1, r3, r3]
    return r[0] < r[1] ? r[0] : r[1];
}

// LDS bytes per wave: the carried-package gather records (4 chunks x 64 lanes x (8 + 2) B), the flag
// bytes (64 lanes x 4), the two halves' candidate lists; the reset scratch reuses the slice.
constexpr size_t HALF_GREC = (size_t)HALF_NC * 64 * 8, HALF_GPS = (size_t)HALF_NC * 64 * 2;
__host__ __device__ constexpr size_t halves_scratch_bytes() {
    return HALF_GREC + HALF_GPS + 64 * (size_t)HALF_NC + 2 * (size_t)HALF_CAND * 8;
}

// NFULL: package chunks known to be full (slot c * 32 + 31 < P for c < NFULL; 3 when P >= 96): their
// slots need no "no package" handling.
template <bool STALE, int NFULL>
__global__ __launch_bounds__(256) void k_step_halves(const uint32_t* __restrict__ rob_pre,
                                                     const uint64_t* __restrict__ pkg_pre,
                                                     const uint16_t* __restrict__ pst_pre,
                                                     const u32x4* __restrict__ es_pre,
                                                     const uint64_t* __restrict__ trk_pre,
                                                     const uint8_t* __restrict__ act_pre, uint32_t ap, uint32_t nw,
                                                     StepArgs args) {
    constexpr int NC = HALF_NC;
    constexpr uint32_t NONE = 255u;   // no package slot (slots < 128)
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
    const int e0 = 2 * w;   // this wave's envs: e0, e0 + 1
    if (wave >= wpb_ || e0 >= n_) return;
    const int h = lane >> 5, hl = lane & 31, hbase = lane & 32, rbase = lane & 48;
    const int ri = lane & 15;                // the robot this lane holds (on both rows of the half)
    const bool live = e0 + h < n_;           // the last wave's second half past n holds no env ...
    const int hh = live ? h : 0;             // ... and reads env e0 (it stores nothing)
    const bool act = live && ri < A;
    const bool row0 = (lane & 16) == 0;      // the robot copy that stores

    // ---- loads: one round trip, every lane loads (in-bounds offsets, discarded where unused).  Slot
    // j = c * 32 + hl of env e0 + hh is element lb + 32 c (lb < 160: the chunks' byte offsets fold
    // into the loads' immediates); lanes past P read the next env's slots or the 256-slot tail
    // padding of the package buffers (MdlEngine) ----
    const uint32_t roff = (uint32_t)(h * A + ri);
    const uint32_t roff_c = (act ? roff : 0u) & 0x1fu;   // h * A + ri < 32
    const uint32_t rv_ld = (robp + (size_t)e0 * A)[roff_c];
    const uint32_t ar_ld = (actp + (size_t)e0 * A)[roff_c];
    uint64_t pk[NC], td[NC];
    uint32_t ps[NC], ps_in[NC];
    bool dirty[NC], pv[NC];
    GLOBAL const uint64_t* pkge = pkgp + (size_t)e0 * P;
    GLOBAL const uint16_t* pste = pstp + (size_t)e0 * P;
    GLOBAL const uint64_t* trke = trkp + (size_t)e0 * P;
    const uint32_t lb = (uint32_t)(hh * P + hl) & 0xffu;   // hh * P + hl < 160
#pragma unroll
    for (int c = 0; c < NC; c++) {
        pv[c] = c < NFULL || c * HALF + hl < P;
        pk[c] = pkge[lb + c * HALF];
        ps[c] = pste[lb + c * HALF];
        td[c] = STALE ? trke[lb + c * HALF] : 0ull;
        dirty[c] = false;
    }
    const uint32_t erow = (uint32_t)hh & 1u;
    const uint32_t t_ld = ((GLOBAL const uint32_t*)(esp + e0))[4u * erow];
    const uint64_t tot_ld = ((GLOBAL const uint64_t*)(esp + e0))[2u * erow + 1u];
    KargPtr kap = (KargPtr)((__attribute__((address_space(4))) const char*)__builtin_amdgcn_kernarg_segment_ptr() +
                            offsetof(StepKarg, args));
    const double cst = kap->p.cost_fold[hl];   // cost_fold[k] on half-lane k (n_cost <= 16)
    __builtin_amdgcn_sched_barrier(0);   // every load above is issued before any use
    const uint32_t rv = act ? rv_ld : 0u;
    int araw = act ? (int)(ar_ld & 0xffu) : 0;
    const uint32_t t_rec = t_ld;
    const uint64_t tot_rec = tot_ld;
    // slots without a package: the sentinels of k_step_rows (status delivered, start time and
    // start cell 0xffff); every store below tests pv (and live)
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
    if (nw & NW_MAP) {   // mixed maps: each half's map
        mi = (int)((GLOBAL const uint8_t*)p.env_map)[e0 + hh];
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

    // ---- the shaped reward's candidates (tracker_prev's waiting entries with st <= t): pre-step
    // state only, packed now into each half's LDS list {start cell, order << 7 | slot}, where the
    // order (8 bits) is a survivor's rank (< P <= 128) or 128 + slot, in the order of order_key ----
    int stc[NC];
    uint64_t anyw = 0, wvm[NC];
    bool wv[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const uint32_t f = ps0[c];
        const bool waiting = STALE ? ((f & PS_PRESENT) && !(f & PS_TRANSIT)) : ((f & PS_STATUS) == ST_WAITING);
        wv[c] = !(MDL_ABLATE & 64) && waiting && pk_st(td[c]) <= t0;
        stc[c] = pk_start(td[c]);
        wvm[c] = ballot(wv[c]);
        anyw |= wvm[c];
    }
    uint64_t* cand = (uint64_t*)(slice + HALF_GREC + HALF_GPS + 64 * NC) + h * HALF_CAND;   // this lane's half
    int nwg = 0;
    if (anyw) {
        // list position: the candidates below this lane in the whole wave (v_mbcnt), less half 0's
        // in half 1, plus the half's earlier chunks
        int n0 = 0, n1 = 0;
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const int lo = popc64(wvm[c] & 0x00000000ffffffffull);
            const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(wvm[c] >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)wvm[c], 0u));
            const int idx = below + (h ? n1 - lo : n0);
            const uint32_t j = (uint32_t)(c * HALF + hl);
            const uint32_t ord = STALE ? ((ps0[c] & PS_SURVIVOR) ? (ps0[c] >> PS_RANK_SHIFT) : 128u + j) : j;
            const uint32_t klo = (ord << 7) | j;
            if (wv[c]) cand[idx] = (uint64_t)(uint32_t)stc[c] | ((uint64_t)klo << 32);
            n0 += lo;
            n1 += popc64(wvm[c] & 0xffffffff00000000ull);
        }
        const int nh = h ? n1 : n0;
        // both halves scan the same (wave-uniform) count: each pads its list with sentinels (cell ~0:
        // no map cell, at distance >= 510 from every cell; key bits 0xffff) to a multiple of 4 of the
        // longer one
        nwg = (max(n0, n1) + 3) & ~3;
        for (int k = nh + hl; k < nwg; k += HALF) cand[k] = 0x0000ffffffffffffull;
    }

    // ---- the pre-step carried package of each robot, through LDS; the flag bytes cleared ----
    const int pj = carry - 1;
    uint64_t* grec = (uint64_t*)slice;                    // env-table | tracker target | deadline << 16
    uint16_t* gps = (uint16_t*)(slice + HALF_GREC);       // the pre-step state word
    unsigned char* flb = slice + HALF_GREC + HALF_GPS;    // byte (lane, c) <-> package slot c * 32 + (lane & 31) of the half
#pragma unroll
    for (int c = 0; c < NC; c++) {
        grec[c * 64 + lane] = (uint64_t)tgt_dl(pk[c]) | ((uint64_t)tgt_dl(td[c]) << 32);
        gps[c * 64 + lane] = (uint16_t)ps0[c];
    }
    ((uint32_t*)flb)[lane] = 0;
    wave_sync();
    const int gi = ((pj >> 5) & (NC - 1)) * 64 + hbase + (pj & 31);
    const uint64_t gv = grec[gi];
    const uint32_t g_pf = gps[gi], g_pk = (uint32_t)gv, g_td = (uint32_t)(gv >> 32);

    // ---- movement (env.py:188-257), row-local: every row holds its half's 16 robots ----
    const int pcell = cell, pcarry = carry;
    constexpr uint64_t DTAB = (uint64_t)(0x3ffu & (uint32_t)-256) << 10 | (uint64_t)256 << 20 |
                              (uint64_t)(0x3ffu & (uint32_t)-1) << 30 | (uint64_t)1 << 40;
    const int dtab = __builtin_amdgcn_sbfe((int)(uint32_t)(DTAB >> (10 * mv)), 0, 10);
    const int vok = __builtin_amdgcn_sbfe((int)vmask, mv, 1);
    const int prop = cell + (int)(lmask(act) & (uint32_t)(dtab & vok));
    const bool mover = !(MDL_ABLATE & 4) && act && prop != cell;
    const uint64_t movers = ballot(mover);
    const uint32_t pvm = (uint32_t)(p.movevalid_cell + mvoff)[(uint32_t)prop];
    uint64_t moved = 0;
    if (movers) {
        // one word per robot: its proposal if it moves (0xffff otherwise: a non-mover blocks nobody) |
        // its cell << 16 (0xfffe where there is no robot)
        const uint32_t wd = (mover ? (uint32_t)prop : 0xffffu) | ((act ? (uint32_t)cell : 0xfffeu) << 16);
        // Each row tests its robot against half of the partners -- row 0 robots 0-7, row 1 robots
        // 8-15, fetched from row 0's copies -- and one swap joins the rows' answers.
        const int g8 = (lane & 16) >> 1;
        uint32_t hk = 0;
        int ok = -1;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t wj = (uint32_t)__builtin_amdgcn_ds_bpermute((hbase + g8 + k) << 2, (int)wd);
            hk |= (wj & 0xffffu) == (uint32_t)prop ? (1u << k) : 0u;
            ok = (wj >> 16) == (uint32_t)prop ? k : ok;   // robots stand on distinct cells: one match at most
        }
        uint32_t hit = hk << g8;
        int occ = ok < 0 ? -1 : ok + g8;
        {
            const auto rh = __builtin_amdgcn_permlane16_swap(hit, hit, false, false);
            hit = rh[0] | rh[1];
            const auto ro = __builtin_amdgcn_permlane16_swap((uint32_t)occ, (uint32_t)occ, false, false);
            occ = max((int)ro[0], (int)ro[1]);
        }
        // a lower-index mover into the same cell (hit holds movers only)
        const bool blocked = (hit & ((1u << ri) - 1u)) != 0u;
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
    // Pick-ups: each picking robot takes the lowest-index waiting package at its cell (robots sit on
    // distinct cells, so the reference's robot order changes nothing).  Per robot index J, one
    // minimum over the half's package slots answers robot J of both envs.
    const bool picker = !(MDL_ABLATE & 8) && act && op == 1 && carry == 0;
    const uint64_t pickers = ballot(picker);
    int cnew = carry;
    if (pickers) {
        int sw[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) sw[c] = (ps[c] & PS_STATUS) == ST_WAITING ? pk_start(pk[c]) : -2;
        if (nw & NW_SMALLMAP) {
            // Every map within 64 x 64: each half's pickers mark their cells in a 4096-bit map in LDS
            // (over the gather records, consumed before the movement); a waiting package tests one
            // bit, and the few packages under a picker are assigned in index order by the scalar
            // unit -- the first one at a picker's cell is its lowest-index package.  Cell
            // row << 8 | column is bit column & 31 of word 2 row + column / 32.
            uint32_t* pb = (uint32_t*)slice + h * 128;
            auto word_of = [](int cl) { return (((uint32_t)cl >> 7) | (((uint32_t)cl >> 5) & 1u)) & 127u; };
            wave_sync();
            reinterpret_cast<u32x4*>((uint32_t*)slice)[lane] = u32x4{0u, 0u, 0u, 0u};   // both halves' maps: 1 KB
            wave_sync();
            if (picker && row0) atomicOr(&pb[word_of(cell)], 1u << (cell & 31));
            wave_sync();
            uint64_t left = pickers & 0x0000ffff0000ffffull;   // row 0's robot copies
#pragma unroll
            for (int c = 0; c < NC; c++) {
                // sw < 0: some in-range word, masked (no short-circuit: no branch per chunk)
                const uint32_t bit = __builtin_amdgcn_ubfe(pb[word_of(sw[c])], (uint32_t)sw[c] & 31u, 1u);
                const uint64_t mt = ballot((sw[c] >= 0) & (bit != 0u));
                for (uint64_t m = mt; m && left; m &= m - 1) {
                    const int j = ffs64(m);
                    const uint64_t who = ballot(cell == rdl(sw[c], j)) & left & (0xffffull << (j & 32));
                    if (who) {
                        const int i = ffs64(who);
                        left &= ~(1ull << i);
                        cnew = (lane & ~16) == i ? c * HALF + (j & 31) + 1 : cnew;
                    }
                }
            }
        } else
        for (uint32_t u = rows_union(pickers); u; u &= u - 1) {
            const int J = __ffs((int)u) - 1;
            const int ci = __builtin_amdgcn_ds_bpermute((rbase + J) << 2, cell);   // robot J's cell, row-local
            uint32_t k = NONE;
#pragma unroll
            for (int c = NC - 1; c >= 0; c--) k = sw[c] == ci ? (uint32_t)(c * HALF + hl) : k;
            k = half_min_u32(k);
            cnew = (ri == J && picker && k != NONE) ? (int)k + 1 : cnew;
        }
    }
    const bool picked = cnew != carry;
    carry = cnew;
    const int g_tgt = (int)(g_pk & 0xffffu), g_dl = (int)(g_pk >> 16);
    const bool drop = act && op == 2 && carry != 0 && g_tgt == cell;
    const uint64_t dmask = ballot(drop), omask = ballot(drop && t0 <= g_dl);
    // one flag byte per package slot, written by the robot concerned (row 0's copy): the slot's new
    // status (bits 0-1) | F_CHG | F_CARRY, as k_step_rows
    constexpr uint32_t F_CHG = 8u, F_CARRY = 4u;
    {
        const int fs = drop ? pj : carry - 1;
        const uint32_t fv = picked ? (F_CHG | F_CARRY | (uint32_t)ST_IN_TRANSIT)
                            : drop ? (F_CHG | (uint32_t)ST_DELIVERED) : F_CARRY;
        if (act && row0 && carry != 0) flb[(hbase + (fs & 31)) * NC + (fs >> 5)] = (unsigned char)fv;
    }
    carry = drop ? 0 : carry;
    wave_sync();
    const uint32_t fw = ((const uint32_t*)flb)[lane];
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const uint32_t f = fw >> (8 * c);
        const uint32_t clr = (0u - ((f >> 3) & 1u)) & PS_STATUS;
        ps[c] = (ps[c] & ~clr) | (f & PS_STATUS);
    }
    // reward: fp64 fold in the reference's order (move costs, then deliveries in robot order)
    double rr;
    {
        const int src = (hbase + n_cost) << 2;
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

    // ---- terminate (env.py:308-316) + spawn (get_state env.py:133-137) ----
    uint32_t undel = 0;
    uint64_t spawned = 0;
#pragma unroll
    for (int c = 0; c < NC; c++) {
        undel |= (ps[c] & PS_STATUS) ^ (uint32_t)ST_DELIVERED;
        const bool sp = pk_st(pk[c]) == t1;
        spawned |= ballot(sp);
        ps[c] = sp ? ((ps[c] & ~PS_STATUS) | ST_WAITING) : ps[c];
    }
    const uint64_t und = ballot(undel != 0u);
    const uint32_t alldel = lmask(((und >> hbase) & 0xffffffffull) == 0ull);
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
        uint32_t Midle = 0, Mcan = 0;
        int best_cell = -1;
        if (anyw && !(MDL_ABLATE & 32)) {
            // The two rows of a half scan alternate candidates for the same agent (two per step, two
            // LDS reads in flight): nearest key from the pre-step cell, and "a waiting package starts
            // at my new cell" (can-pick-up) into a lane mask; one swap joins the rows.  The key is one
            // v_sad_hi_u8: distance << 16 + (order << 7 | slot); a real distance is <= 508 (cells
            // are row << 8 | column, both < 255), a sentinel's >= 510.
            const uint64_t* cp = cand + ((lane >> 4) & 1);
            uint32_t kmin = 0xffffffffu;
            uint64_t hmc = 0;
            for (int i0 = 0; i0 < nwg; i0 += 4) {   // wave-uniform trip count
                const uint64_t ce = cp[i0], cf = cp[i0 + 2];
                const uint32_t ke = __builtin_amdgcn_sad_hi_u8((uint32_t)pcell, (uint32_t)ce, (uint32_t)(ce >> 32));
                const uint32_t kf = __builtin_amdgcn_sad_hi_u8((uint32_t)pcell, (uint32_t)cf, (uint32_t)(cf >> 32));
                kmin = min(kmin, min(ke, kf));
                hmc |= ballot((int)(uint32_t)ce == cell) | ballot((int)(uint32_t)cf == cell);
            }
            {
                const auto r = __builtin_amdgcn_permlane16_swap(kmin, kmin, false, false);
                kmin = r[0] < r[1] ? r[0] : r[1];
            }
            const uint32_t h16 = (uint32_t)(((hmc >> hbase) | (hmc >> (hbase + 16))) & 0xffffull);
            Mcan = ((h16 >> ri) & 1u) ? ~0u : 0u;
            const int js = (int)(kmin & 127u);
            const int sl = (hbase + (js & 31)) << 2;
            int bc = __builtin_amdgcn_ds_bpermute(sl, stc[0]);
#pragma unroll
            for (int c = 1; c < NC; c++) {
                const int v = __builtin_amdgcn_ds_bpermute(sl, stc[c]);
                bc = (js >> 5) == c ? v : bc;
            }
            const bool found = act && kmin < (509u << 16);
            Midle = lmask(found && (kmin >> 16) <= 3u);
            best_cell = found ? bc : -1;
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
    // numpy's pairwise float32 sum of the A (8..16) agents, in-row: lanes A..15 hold +0.0f, so every
    // A in 8..16 takes numpy's n >= 8 form r_j = x_j + x_{j+8}, ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))
    float ssum;
    {
        const float r8 = s_lane + dppf<0x128>(s_lane);   // row_ror:8: lane j < 8 gets x_j + x_{j+8}
        const float s2 = r8 + dppf<0xB1>(r8);
        const float c4 = s2 + dppf<0x4E>(s2);
        const float d = c4 + dppf<0x124>(c4);           // lane 0: c[0] + c[12] (c[12] == c[4])
        ssum = 0.0f + row_bcastf<0>(d);
    }
    const float shaped = (float)rr + ssum;

    // ---- tracker update with the new state (MAPPO/trainer.py:95-130); halves that reset below
    // update with the reset state instead ----
    const bool do_rst = done && auto_reset;
    const uint64_t rst = ballot(do_rst);
    if (STALE && !(MDL_ABLATE & 2) && (ballot(picked) | dmask | spawned)) {
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const bool ins = !do_rst && (pk_st(pk[c]) == t1) && !(ps[c] & PS_PRESENT);
            ps[c] = ins ? ((ps[c] & PS_STATUS) | PS_PRESENT) : ps[c];
            td[c] = ins ? pk[c] : td[c];
            dirty[c] = dirty[c] || ins;
            const uint32_t m_p = lmask((ps[c] & PS_PRESENT) != 0u && !do_rst);
            const uint32_t m_c = lmask(((fw >> (8 * c)) & F_CARRY) != 0u);
            const uint32_t m_t = lmask((ps[c] & PS_TRANSIT) != 0u);
            ps[c] = (ps[c] | (PS_TRANSIT & m_c & m_p)) & (PS_STATUS | ~(m_p & ~m_c & m_t));
        }
    }

    // ---- outputs and write-back of the step (pointers fetched in one late scalar batch).  A half
    // that resets stores only its outputs and env record here: the reset below writes its rows,
    // after these stores, so the package registers are dead while it runs (the reset path would
    // otherwise set the kernel's register count: 85 VGPRs and 28 SGPR spills, against 72 and none) ----
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
    const uint32_t er = (uint32_t)h & 1u;
    if (live && hl == 0) {
        if (rop) (rop + e0)[er] = rr;
        if (shp) (shp + e0)[er] = shaped;
        if (dnp) (dnp + e0)[er] = done ? 1 : 0;
        (esw + e0)[er] = u32x4{(uint32_t)t_out, rfl, (uint32_t)__double2loint(total_out),
                               (uint32_t)__double2hiint(total_out)};
    }
    if (live && hl == 0 && done) {
        ((GLOBAL double*)p.ep_total + e0)[er] = total;
        ((GLOBAL int32_t*)p.ep_len + e0)[er] = t1;
    }
    if (act && row0 && !do_rst) (robw + (size_t)e0 * A)[roff] = rob_pack(cell, carry, vmask);
    const size_t eb = (size_t)e0 * P;
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const uint32_t o = lb + c * HALF;
        // (dirty marks inserts of this step, which a resetting half does not make)
        if (live && pv[c] && !do_rst && ps[c] != ps_in[c]) (pstw + eb)[o] = (uint16_t)ps[c];
        if (STALE && live && pv[c] && dirty[c]) (trkw + eb)[o] = td[c];
    }

    // ---- reset on done (MAPPO/trainer.py:230-235): one half at a time, by the whole wave; it writes
    // the half's robots, package table and state words (and the tracker's t = 0 inserts) ----
    if (rst) {
        GLOBAL uint64_t* pkgw = (GLOBAL uint64_t*)kap->p.pkg;
        wave_sync();   // the flag bytes, gather records and candidates are consumed (the reset scratch overlays them)
        for (uint64_t m = rst & 0x0000000100000001ull; m; m &= m - 1) {
            const int hb = ffs64(m);   // 32 * the resetting half
            const int er2 = e0 + (hb >> 5);
            ResetLds L = reset_carve(slice, P);
            const int mr = rdl(mi, hb);
            const MapDesc md = p.maps[mr];
            const int nc = do_reset(p, er2, md, L, false);   // robot a's cell on lane a
            const int ncr = __builtin_amdgcn_ds_bpermute(ri << 2, nc);
            const bool mine = hbase == hb;
            if (mine && act && row0)
                (robw + (size_t)e0 * A)[roff] = rob_pack(ncr, 0, p.movevalid_cell[(uint32_t)(mvoff + ncr)]);
            if (STALE) {
                // every present entry of the half becomes a survivor ranked by its current key
                uint32_t rk[NC], tq[NC];
#pragma unroll
                for (int c = 0; c < NC; c++) {
                    rk[c] = 0;
                    tq[c] = order_key(ps[c], c * HALF + hl);   // the key bits survive the step's updates
                }
#pragma unroll
                for (int c2 = 0; c2 < NC; c2++) {
                    uint64_t pm = ballot(c2 * HALF + hl < P && (ps[c2] & PS_PRESENT)) & (0xffffffffull << hb);
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
                        if (c * HALF + hl < P && (ps[c] & PS_PRESENT)) {
                            ps[c] = (ps[c] & PS_FLAGS) | PS_SURVIVOR | (rk[c] << PS_RANK_SHIFT);
                        } else {
                            ps[c] &= PS_STATUS;
                        }
                    }
                }
            }
#pragma unroll
            for (int c = 0; c < NC; c++) {
                const int j = c * HALF + hl;
                if (mine && j < P) {
                    const uint64_t npk = L.pk[j];
                    uint32_t nps = (uint32_t)L.pst[j] | (STALE ? (ps[c] & ~PS_STATUS) : 0u);
                    if (STALE) {   // the update with the reset state: inserts at t = 0, nothing carried
                        const bool ins = (pk_st(npk) == 0) & !(nps & PS_PRESENT);
                        nps = ins ? ((nps & PS_STATUS) | PS_PRESENT) : nps;
                        if (ins) (trkw + eb)[(uint32_t)(h * P + j) & 0xffu] = npk;
                        const uint32_t upd = (nps & PS_TRANSIT) ? (nps & PS_STATUS) : nps;
                        nps = (nps & PS_PRESENT) ? upd : nps;
                    }
                    const uint32_t o = (uint32_t)(h * P + j) & 0xffu;
                    (pkgw + eb)[o] = npk;
                    (pstw + eb)[o] = (uint16_t)nps;
                }
            }
            wave_sync();   // L is read by every lane before the next half's reset rewrites it
        }
    }
}
