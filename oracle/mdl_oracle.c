/*
 * mdl_oracle.c -- CPU ORACLE for the marl-delivery step/observation hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is a plain-C restatement of the
 * reference's Python algorithm, written to be read side by side with it.  It
 * is the checker for the HIP engine (tests/, __graft_entry__.smoke()) and the
 * "port" CPU baseline timed by bench.py.  Product code never links, loads or
 * calls it.
 *
 * It deliberately follows the reference LITERALLY (sequential restart loop for
 * movement, ordered-dict tracker, libm pow() sort keys, float32 NEP-50 shaped
 * reward with numpy's pairwise sum) and NOT the parallel formulations used by
 * the HIP kernels, so that agreement between the two is evidence.
 *
 * Parity pinning: tests/test_oracle_golden.py checks every function here
 * against fixtures produced by running the reference itself
 * (tests/golden/gen_golden.py).
 *
 * Reference citations are path:line under /root/reference.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MT_N 624
#define MT_M 397

/* ----------------------------------------------------------------------- */
/* numpy legacy RandomState: MT19937 + masked-rejection randint             */
/* (numpy/random/src/mt19937 + distributions.c; used by env.py:40,157,168) */
/* ----------------------------------------------------------------------- */
typedef struct {
    uint32_t key[MT_N];
    int pos;
} OMT;

static void mt_seed(OMT* mt, uint32_t seed) {
    /* RandomState(int seed) -> mt19937_seed(): init_genrand */
    for (int i = 0; i < MT_N; i++) {
        mt->key[i] = seed;
        seed = (uint32_t)(1812433253UL * (seed ^ (seed >> 30)) + (uint32_t)(i + 1));
    }
    mt->pos = MT_N;
}

static void mt_gen(OMT* mt) {
    uint32_t y;
    int i;
    for (i = 0; i < MT_N - MT_M; i++) {
        y = (mt->key[i] & 0x80000000UL) | (mt->key[i + 1] & 0x7fffffffUL);
        mt->key[i] = mt->key[i + MT_M] ^ (y >> 1) ^ ((uint32_t)(-(int32_t)(y & 1)) & 0x9908b0dfUL);
    }
    for (; i < MT_N - 1; i++) {
        y = (mt->key[i] & 0x80000000UL) | (mt->key[i + 1] & 0x7fffffffUL);
        mt->key[i] = mt->key[i + (MT_M - MT_N)] ^ (y >> 1) ^ ((uint32_t)(-(int32_t)(y & 1)) & 0x9908b0dfUL);
    }
    y = (mt->key[MT_N - 1] & 0x80000000UL) | (mt->key[0] & 0x7fffffffUL);
    mt->key[MT_N - 1] = mt->key[MT_M - 1] ^ (y >> 1) ^ ((uint32_t)(-(int32_t)(y & 1)) & 0x9908b0dfUL);
    mt->pos = 0;
}

static uint32_t mt_next32(OMT* mt) {
    if (mt->pos == MT_N) mt_gen(mt);
    uint32_t y = mt->key[mt->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680UL;
    y ^= (y << 15) & 0xefc60000UL;
    y ^= (y >> 18);
    return y;
}

/* RandomState.randint(lo, hi) for int64 output, hi exclusive, hi-lo <= 2^32.
 * rng == 0 returns lo WITHOUT consuming a draw. Returns lo-1 on lo >= hi
 * (numpy raises ValueError there). */
static long or_randint(OMT* mt, long lo, long hi) {
    if (lo >= hi) return lo - 1;
    uint64_t rng = (uint64_t)(hi - 1 - lo);
    if (rng == 0) return lo;
    uint32_t mask = (uint32_t)rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (mt_next32(mt) & mask)) > (uint32_t)rng) {
    }
    return lo + (long)v;
}

/* ----------------------------------------------------------------------- */
/* Environment (env.py:4-316)                                               */
/* ----------------------------------------------------------------------- */
enum { ST_NONE = 0, ST_WAITING = 1, ST_IN_TRANSIT = 2, ST_DELIVERED = 3 };
enum { MV_S = 0, MV_L = 1, MV_R = 2, MV_U = 3, MV_D = 4, MV_UNKNOWN = 5 };

typedef struct {
    int r, c, carrying;
} ORobot;

typedef struct {
    int sr, sc, tr, tc, start_time, deadline, id, status;
} OPkg;

typedef struct {
    int H, W, A, P, T;
    uint8_t* grid;
    double move_cost, delivery_reward, delay_reward;
    OMT mt;
    int t;
    double total_reward;
    ORobot* robots;
    OPkg* pkgs;
    /* scratch */
    int* free_cells;
    uint8_t* tmp;
    int* old_pos;
    int* occupied;
} OEnv;

/* get_state() side effect: spawn (env.py:127-147) */
static void env_spawn(OEnv* e) {
    for (int i = 0; i < e->P; i++)
        if (e->pkgs[i].start_time == e->t) e->pkgs[i].status = ST_WAITING;
}

/* env.py:81-125 */
void or_env_reset(OEnv* e) {
    e->t = 0;
    e->total_reward = 0.0;
    int H = e->H, W = e->W;
    memcpy(e->tmp, e->grid, (size_t)H * W);
    for (int i = 0; i < e->A; i++) {
        /* get_random_free_cell(tmp_grid) env.py:161-170 */
        int nf = 0;
        for (int r = 0; r < H; r++)
            for (int c = 0; c < W; c++)
                if (e->tmp[r * W + c] == 0) e->free_cells[nf++] = r * W + c;
        long k = or_randint(&e->mt, 0, nf);
        int cell = e->free_cells[k];
        e->tmp[cell] = 1;
        e->robots[i].r = cell / W;
        e->robots[i].c = cell % W;
        e->robots[i].carrying = 0;
    }
    int N = e->H;
    /* get_random_free_cell_p() env.py:150-158 (original grid) */
    int nfp = 0;
    for (int r = 0; r < H; r++)
        for (int c = 0; c < W; c++)
            if (e->grid[r * W + c] == 0) e->free_cells[nfp++] = r * W + c;
    int lim = e->A < 20 ? e->A : 20;
    OPkg* lst = (OPkg*)malloc(sizeof(OPkg) * (size_t)(e->P > 0 ? e->P : 1));
    for (int i = 0; i < e->P; i++) {
        int start = e->free_cells[or_randint(&e->mt, 0, nfp)];
        int target;
        for (;;) {
            target = e->free_cells[or_randint(&e->mt, 0, nfp)];
            if (start != target) break;
        }
        long to_deadline = 10 + or_randint(&e->mt, (long)(N / 2), 3L * N); /* int(N/2) */
        int start_time = (i <= lim) ? 0 : (int)or_randint(&e->mt, 1, e->T);
        lst[i].sr = start / W; lst[i].sc = start % W;
        lst[i].tr = target / W; lst[i].tc = target % W;
        lst[i].start_time = start_time;
        lst[i].deadline = start_time + (int)to_deadline;
    }
    /* list.sort(key=start_time): stable (insertion sort) env.py:119 */
    for (int i = 1; i < e->P; i++) {
        OPkg x = lst[i];
        int j = i - 1;
        while (j >= 0 && lst[j].start_time > x.start_time) { lst[j + 1] = lst[j]; j--; }
        lst[j + 1] = x;
    }
    for (int i = 0; i < e->P; i++) {
        e->pkgs[i] = lst[i];
        e->pkgs[i].id = i + 1;
        e->pkgs[i].status = ST_NONE;
    }
    free(lst);
    env_spawn(e);
}

OEnv* or_env_new(const uint8_t* grid, int H, int W, int A, int P, int T,
                 double move_cost, double delivery_reward, double delay_reward, uint32_t seed) {
    OEnv* e = (OEnv*)calloc(1, sizeof(OEnv));
    e->H = H; e->W = W; e->A = A; e->P = P; e->T = T;
    e->grid = (uint8_t*)malloc((size_t)H * W);
    memcpy(e->grid, grid, (size_t)H * W);
    e->move_cost = move_cost; e->delivery_reward = delivery_reward; e->delay_reward = delay_reward;
    e->robots = (ORobot*)calloc((size_t)(A > 0 ? A : 1), sizeof(ORobot));
    e->pkgs = (OPkg*)calloc((size_t)(P > 0 ? P : 1), sizeof(OPkg));
    e->free_cells = (int*)malloc(sizeof(int) * (size_t)H * W);
    e->tmp = (uint8_t*)malloc((size_t)H * W);
    e->old_pos = (int*)malloc(sizeof(int) * (size_t)H * W);
    e->occupied = (int*)malloc(sizeof(int) * (size_t)H * W);
    mt_seed(&e->mt, seed);      /* env.py:40 */
    or_env_reset(e);            /* env.py:41: the constructor draws one layout */
    return e;
}

void or_env_free(OEnv* e) {
    if (!e) return;
    free(e->grid); free(e->robots); free(e->pkgs); free(e->free_cells); free(e->tmp);
    free(e->old_pos); free(e->occupied); free(e);
}

/* valid_position env.py:336-345 */
static int env_valid(const OEnv* e, int r, int c) {
    if (r < 0 || r >= e->H || c < 0 || c >= e->W) return 0;
    if (e->grid[r * e->W + c] == 1) return 0;
    return 1;
}

/* env.py:173-306.  move: MV_* codes, op: 0 none, 1 pick, 2 drop, 3 any other
 * string.  Returns done; *r gets the step reward, *r_is_int = reward stayed
 * the Python int 0. */
int or_env_step(OEnv* e, const uint8_t* move, const uint8_t* op, double* r_out, int* r_is_int) {
    int A = e->A, W = e->W, HW = e->H * e->W;
    double r = 0.0;
    int r_int = 1;
    int* prop = (int*)malloc(sizeof(int) * (size_t)(A > 0 ? A : 1));
    int* fin = (int*)malloc(sizeof(int) * (size_t)(A > 0 ? A : 1));
    int* computed = (int*)calloc((size_t)(A > 0 ? A : 1), sizeof(int));
    for (int i = 0; i < HW; i++) { e->old_pos[i] = -1; e->occupied[i] = -1; }
    for (int i = 0; i < A; i++) {
        int pr = e->robots[i].r, pc = e->robots[i].c;
        int nr = pr, nc = pc;                      /* compute_new_position env.py:318-334 */
        switch (move[i]) {
            case MV_L: nc = pc - 1; break;
            case MV_R: nc = pc + 1; break;
            case MV_U: nr = pr - 1; break;
            case MV_D: nr = pr + 1; break;
            default: break;
        }
        if (!env_valid(e, nr, nc)) { nr = pr; nc = pc; }
        prop[i] = nr * W + nc;
        e->old_pos[pr * W + pc] = i;
    }
    /* restart-from-zero resolution loop env.py:207-246 */
    for (;;) {
        int updated = 0;
        for (int i = 0; i < A; i++) {
            if (computed[i] != 0) continue;
            int pos = e->robots[i].r * W + e->robots[i].c;
            int np_ = prop[i];
            int can_move = 0;
            if (e->old_pos[np_] < 0) {
                can_move = 1;
            } else {
                int j = e->old_pos[np_];
                if (j != i && computed[j] == 0) continue;
                can_move = 1;
            }
            if (can_move) {
                if (e->occupied[np_] < 0) {
                    e->occupied[np_] = i;
                    fin[i] = np_;
                } else {
                    e->occupied[pos] = i;
                    fin[i] = pos;
                }
                computed[i] = 1;
                updated = 1;
            }
            if (updated) break;
        }
        if (!updated) break;
    }
    for (int i = 0; i < A; i++)
        if (computed[i] == 0) fin[i] = e->robots[i].r * W + e->robots[i].c;
    /* move cost env.py:253-257 */
    for (int i = 0; i < A; i++) {
        int pos = e->robots[i].r * W + e->robots[i].c;
        int lrud = move[i] == MV_L || move[i] == MV_R || move[i] == MV_U || move[i] == MV_D;
        if (lrud && fin[i] != pos) { r += e->move_cost; r_int = 0; }
        e->robots[i].r = fin[i] / W;
        e->robots[i].c = fin[i] % W;
    }
    /* package actions env.py:260-292 */
    for (int i = 0; i < A; i++) {
        ORobot* rb = &e->robots[i];
        if (op[i] == 1) {
            if (rb->carrying == 0) {
                for (int j = 0; j < e->P; j++) {
                    OPkg* p = &e->pkgs[j];
                    if (p->status == ST_WAITING && p->sr == rb->r && p->sc == rb->c && p->start_time <= e->t) {
                        rb->carrying = p->id;
                        p->status = ST_IN_TRANSIT;
                        break;
                    }
                }
            }
        } else if (op[i] == 2) {
            if (rb->carrying != 0) {
                OPkg* p = &e->pkgs[rb->carrying - 1];
                if (rb->r == p->tr && rb->c == p->tc) {
                    p->status = ST_DELIVERED;
                    if (e->t <= p->deadline) r += e->delivery_reward;
                    else r += e->delay_reward;
                    r_int = 0;
                    rb->carrying = 0;
                }
            }
        }
    }
    e->t += 1;                                   /* env.py:295 */
    e->total_reward += r;                        /* env.py:297 */
    int done = 0;                                /* check_terminate env.py:308-316 */
    if (e->t == e->T) {
        done = 1;
    } else {
        done = 1;
        for (int j = 0; j < e->P; j++)
            if (e->pkgs[j].status != ST_DELIVERED) { done = 0; break; }
    }
    env_spawn(e);                                /* get_state() env.py:306 */
    free(prop); free(fin); free(computed);
    *r_out = r;
    *r_is_int = r_int;
    return done;
}

/* robots: A*3 (r, c, carrying) 0-indexed; pkgs: P*8 (sr,sc,tr,tc,st,dl,id,status) */
void or_env_get(const OEnv* e, int32_t* t, double* total, int32_t* robots, int32_t* pkgs) {
    *t = e->t;
    *total = e->total_reward;
    for (int i = 0; i < e->A; i++) {
        robots[3 * i] = e->robots[i].r; robots[3 * i + 1] = e->robots[i].c; robots[3 * i + 2] = e->robots[i].carrying;
    }
    for (int j = 0; j < e->P; j++) {
        const OPkg* p = &e->pkgs[j];
        int32_t* o = pkgs + 8 * j;
        o[0] = p->sr; o[1] = p->sc; o[2] = p->tr; o[3] = p->tc; o[4] = p->start_time; o[5] = p->deadline;
        o[6] = p->id; o[7] = p->status;
    }
}

/* ----------------------------------------------------------------------- */
/* Persistent-package tracker: an insertion-ordered dict                    */
/* MAPPO/trainer.py:95-130 (== QMIX/trainer.py:69-103)                      */
/* row layout (8 ints): id, status(1 waiting / 2 in_transit), sr, sc, tr, tc, start_time, deadline */
/* ----------------------------------------------------------------------- */
typedef struct {
    int n, cap;
    int32_t* rows;
} OTrk;

OTrk* or_trk_new(int cap) {
    OTrk* k = (OTrk*)calloc(1, sizeof(OTrk));
    k->cap = cap > 0 ? cap : 1;
    k->rows = (int32_t*)malloc(sizeof(int32_t) * 8 * (size_t)k->cap);
    return k;
}
void or_trk_free(OTrk* k) { if (k) { free(k->rows); free(k); } }
void or_trk_clear(OTrk* k) { k->n = 0; }
int or_trk_get(const OTrk* k, int32_t* rows) { memcpy(rows, k->rows, sizeof(int32_t) * 8 * (size_t)k->n); return k->n; }
void or_trk_set(OTrk* k, const int32_t* rows, int n) {
    if (n > k->cap) { k->cap = n; k->rows = (int32_t*)realloc(k->rows, sizeof(int32_t) * 8 * (size_t)n); }
    memcpy(k->rows, rows, sizeof(int32_t) * 8 * (size_t)n);
    k->n = n;
}

static int trk_find(const int32_t* rows, int n, int id) {
    for (int k = 0; k < n; k++) if (rows[8 * k] == id) return k;
    return -1;
}

/* state['packages'] = packages with start_time == t (env.py:133-137), in index order */
void or_trk_update_from_env(OTrk* k, const OEnv* e) {
    for (int j = 0; j < e->P; j++) {
        const OPkg* p = &e->pkgs[j];
        if (p->start_time != e->t) continue;
        if (trk_find(k->rows, k->n, p->id) >= 0) continue;
        if (k->n == k->cap) { k->cap *= 2; k->rows = (int32_t*)realloc(k->rows, sizeof(int32_t) * 8 * (size_t)k->cap); }
        int32_t* o = k->rows + 8 * k->n++;
        o[0] = p->id; o[1] = ST_WAITING; o[2] = p->sr; o[3] = p->sc; o[4] = p->tr; o[5] = p->tc;
        o[6] = p->start_time; o[7] = p->deadline;
    }
    int w = 0;
    for (int q = 0; q < k->n; q++) {
        int32_t* o = k->rows + 8 * q;
        int carried = 0;
        for (int i = 0; i < e->A; i++) if (e->robots[i].carrying != 0 && e->robots[i].carrying == o[0]) carried = 1;
        int keep = 1;
        if (carried) o[1] = ST_IN_TRANSIT;
        else if (o[1] == ST_IN_TRANSIT) keep = 0;
        if (keep) {
            if (w != q) memmove(k->rows + 8 * w, o, sizeof(int32_t) * 8);
            w++;
        }
    }
    k->n = w;
}

/* ----------------------------------------------------------------------- */
/* Feature builders: MAPPO/helper.py (QMIX/helper.py identical)             */
/* robots1: A*3 as in the state dict: (r+1, c+1, carrying)                  */
/* ----------------------------------------------------------------------- */
static double (*volatile pow_fn)(double, double) = pow;   /* stop gcc folding pow(x,2) -> x*x */

/* CPython float_pow: negative base with integral exponent -> pow(-x, y) (sign even) */
static double py_sq(double x) {
    if (x == 0.0) return 0.0;
    if (x < 0) x = -x;
    return pow_fn(x, 2.0);
}

/* MAPPO/helper.py:6-66 */
void or_convert_observation(const uint8_t* grid, int H, int W, int t, int A, const int32_t* robots1,
                            const int32_t* trk, int ntrk, int idx, float* obs) {
    memset(obs, 0, sizeof(float) * 6 * (size_t)H * W);
    for (int i = 0; i < H * W; i++) obs[i] = (float)grid[i];
    if (!(0 <= idx && idx < A)) return;
    int my_r = robots1[3 * idx] - 1, my_c = robots1[3 * idx + 1] - 1, my_pkg = robots1[3 * idx + 2];
    if (0 <= my_r && my_r < H && 0 <= my_c && my_c < W) obs[1 * H * W + my_r * W + my_c] = 1.0f;
    for (int i = 0; i < A; i++) {
        if (i == idx) continue;
        int r = robots1[3 * i] - 1, c = robots1[3 * i + 1] - 1;
        if (0 <= r && r < H && 0 <= c && c < W) obs[2 * H * W + r * W + c] = 1.0f;
    }
    for (int q = 0; q < ntrk; q++) {
        const int32_t* p = trk + 8 * q;
        if (p[1] == ST_WAITING && p[6] <= t) {
            if (0 <= p[2] && p[2] < H && 0 <= p[3] && p[3] < W) obs[3 * H * W + p[2] * W + p[3]] = 1.0f;
        }
        if ((p[1] == ST_WAITING && p[6] <= t) || p[1] == ST_IN_TRANSIT) {
            if (0 <= p[4] && p[4] < H && 0 <= p[5] && p[5] < W) obs[4 * H * W + p[4] * W + p[5]] = 1.0f;
        }
    }
    if (my_pkg != 0) {
        int q = trk_find(trk, ntrk, my_pkg);
        if (q >= 0) {
            const int32_t* p = trk + 8 * q;
            if (p[1] == ST_IN_TRANSIT && 0 <= p[4] && p[4] < H && 0 <= p[5] && p[5] < W)
                obs[5 * H * W + p[4] * W + p[5]] = 1.0f;
        }
    }
}

typedef struct {
    double v[5];
    double k0, k1;
    int order;
} SortItem;

static int item_less(const SortItem* a, const SortItem* b) {
    if (a->k0 != b->k0) return a->k0 < b->k0;
    return a->k1 < b->k1;
}

static void stable_sort(SortItem* it, int n) {
    for (int i = 1; i < n; i++) {
        SortItem x = it[i];
        int j = i - 1;
        while (j >= 0 && item_less(&x, &it[j])) { it[j + 1] = it[j]; j--; }
        it[j + 1] = x;
    }
}

/* MAPPO/helper.py:68-165 */
void or_generate_vector_features(int H, int W, int t, int A, const int32_t* robots1, const int32_t* trk, int ntrk,
                                 int idx, int T, int MO, int MP, float* out) {
    int total = 6 + MO * 5 + MP * 5 + 1;
    memset(out, 0, sizeof(float) * (size_t)total);
    if (!(0 <= idx && idx < A)) return;
    int my_r = robots1[3 * idx] - 1, my_c = robots1[3 * idx + 1] - 1, my_pkg = robots1[3 * idx + 2];
    double f[6] = {(double)my_r / H, (double)my_c / W, my_pkg != 0 ? 1.0 : 0.0, 0.0, 0.0, 0.0};
    if (my_pkg != 0) {
        int q = trk_find(trk, ntrk, my_pkg);
        if (q >= 0 && trk[8 * q + 1] == ST_IN_TRANSIT) {
            const int32_t* p = trk + 8 * q;
            int d = p[7] - t; if (d < 0) d = 0;
            f[3] = (double)(p[4] - my_r) / H;
            f[4] = (double)(p[5] - my_c) / W;
            f[5] = T > 0 ? (double)d / T : 0.0;
        }
    }
    int o = 0;
    for (int i = 0; i < 6; i++) out[o++] = (float)f[i];
    SortItem* it = (SortItem*)malloc(sizeof(SortItem) * (size_t)((A > ntrk ? A : ntrk) + 1));
    int n = 0;
    for (int i = 0; i < A; i++) {
        if (i == idx) continue;
        int r = robots1[3 * i] - 1, c = robots1[3 * i + 1] - 1, pid = robots1[3 * i + 2];
        SortItem s;
        memset(&s, 0, sizeof(s));
        s.v[0] = (double)(r - my_r) / H;
        s.v[1] = (double)(c - my_c) / W;
        s.v[2] = pid != 0 ? 1.0 : 0.0;
        if (pid != 0) {
            int q = trk_find(trk, ntrk, pid);
            if (q >= 0 && trk[8 * q + 1] == ST_IN_TRANSIT) {
                s.v[3] = (double)(trk[8 * q + 4] - r) / H;
                s.v[4] = (double)(trk[8 * q + 5] - c) / W;
            }
        }
        s.k0 = py_sq(s.v[0]) + py_sq(s.v[1]);
        s.k1 = 0.0;
        s.order = n;
        it[n++] = s;
    }
    stable_sort(it, n);
    for (int i = 0; i < MO; i++)
        for (int k = 0; k < 5; k++) out[o++] = i < n ? (float)it[i].v[k] : 0.0f;
    n = 0;
    for (int q = 0; q < ntrk; q++) {
        const int32_t* p = trk + 8 * q;
        if (!(p[1] == ST_WAITING && p[6] <= t)) continue;
        SortItem s;
        int d = p[7] - t; if (d < 0) d = 0;
        s.v[0] = (double)(p[2] - my_r) / H;
        s.v[1] = (double)(p[3] - my_c) / W;
        s.v[2] = (double)(p[4] - my_r) / H;
        s.v[3] = (double)(p[5] - my_c) / W;
        s.v[4] = T > 0 ? (double)d / T : 0.0;
        s.k0 = s.v[4];
        s.k1 = py_sq(s.v[0]) + py_sq(s.v[1]);
        s.order = n;
        it[n++] = s;
    }
    stable_sort(it, n);
    for (int i = 0; i < MP; i++)
        for (int k = 0; k < 5; k++) out[o++] = i < n ? (float)it[i].v[k] : 0.0f;
    out[o++] = T > 0 ? (float)((double)t / T) : 0.0f;
    free(it);
}

/* MAPPO/helper.py:167-255 */
void or_convert_global_state(const uint8_t* grid, int H, int W, int t, int A, const int32_t* robots1,
                             const int32_t* trk, int ntrk, int T, int MR, int MPs, float* gmap, float* vec) {
    int HW = H * W;
    memset(gmap, 0, sizeof(float) * 4 * (size_t)HW);
    for (int i = 0; i < HW; i++) gmap[i] = (float)grid[i];
    for (int i = 0; i < A; i++) {
        int r = robots1[3 * i] - 1, c = robots1[3 * i + 1] - 1;
        if (0 <= r && r < H && 0 <= c && c < W) gmap[HW + r * W + c] = 1.0f;
    }
    for (int q = 0; q < ntrk; q++) {
        const int32_t* p = trk + 8 * q;
        if (p[1] == ST_WAITING && p[6] <= t)
            if (0 <= p[2] && p[2] < H && 0 <= p[3] && p[3] < W) gmap[2 * HW + p[2] * W + p[3]] = 1.0f;
        if ((p[1] == ST_WAITING && p[6] <= t) || p[1] == ST_IN_TRANSIT)
            if (0 <= p[4] && p[4] < H && 0 <= p[5] && p[5] < W) gmap[3 * HW + p[4] * W + p[5]] = 1.0f;
    }
    int o = 0;
    for (int i = 0; i < MR; i++) {
        double v[6] = {0, 0, 0, 0, 0, 0};
        if (i < A) {
            int r0 = robots1[3 * i] - 1, c0 = robots1[3 * i + 1] - 1, carried = robots1[3 * i + 2];
            v[0] = (double)r0 / H; v[1] = (double)c0 / W; v[2] = carried != 0 ? 1.0 : 0.0;
            if (carried != 0) {
                int q = trk_find(trk, ntrk, carried);
                if (q >= 0 && trk[8 * q + 1] == ST_IN_TRANSIT) {
                    int d = trk[8 * q + 7] - t; if (d < 0) d = 0;
                    v[3] = (double)trk[8 * q + 4] / H; v[4] = (double)trk[8 * q + 5] / W;
                    v[5] = T > 0 ? (double)d / T : 0.0;
                }
            }
        }
        for (int k = 0; k < 6; k++) vec[o++] = (float)v[k];
    }
    /* active packages sorted by id (sorted() is stable; ids are dict keys -> unique) */
    int* act = (int*)malloc(sizeof(int) * (size_t)(ntrk + 1));
    int na = 0;
    for (int q = 0; q < ntrk; q++) {
        const int32_t* p = trk + 8 * q;
        if ((p[1] == ST_WAITING && p[6] <= t) || p[1] == ST_IN_TRANSIT) act[na++] = q;
    }
    for (int i = 1; i < na; i++) {
        int x = act[i], j = i - 1;
        while (j >= 0 && trk[8 * act[j]] > trk[8 * x]) { act[j + 1] = act[j]; j--; }
        act[j + 1] = x;
    }
    for (int i = 0; i < MPs; i++) {
        double v[7] = {0, 0, 0, 0, 0, 0, 0};
        if (i < na) {
            const int32_t* p = trk + 8 * act[i];
            int waiting = p[1] == ST_WAITING;
            if (waiting) { v[0] = (double)p[2] / H; v[1] = (double)p[3] / W; }
            v[2] = (double)p[4] / H; v[3] = (double)p[5] / W;
            int d = p[7] - t; if (d < 0) d = 0;
            v[4] = T > 0 ? (double)d / T : 0.0;
            v[5] = waiting ? 0.0 : 1.0;
            double carrier = -1.0;
            if (p[1] == ST_IN_TRANSIT) {
                for (int ridx = 0; ridx < A; ridx++) {
                    if (robots1[3 * ridx + 2] == p[0]) {
                        carrier = MR > 1 ? (double)ridx / (MR - 1) : 0.0;
                        break;
                    }
                }
            }
            v[6] = carrier;
        }
        for (int k = 0; k < 7; k++) vec[o++] = (float)v[k];
    }
    vec[o++] = T > 0 ? (float)((double)t / T) : 0.0f;
    free(act);
}

/* numpy float32 add.reduce of a contiguous 1-D array: 0 + pairwise_sum
 * (numpy/_core/src/umath/loops_utils.h.src, PW_BLOCKSIZE 128) */
static float np_pairwise_f32(const float* a, int n) {
    if (n < 8) {
        float res = 0.0f;
        for (int i = 0; i < n; i++) res = res + a[i];
        return res;
    } else if (n <= 128) {
        float r[8];
        for (int j = 0; j < 8; j++) r[j] = a[j];
        int i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] = r[j] + a[i + j];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res = res + a[i];
        return res;
    } else {
        int n2 = n / 2;
        n2 -= n2 % 8;
        return np_pairwise_f32(a, n2) + np_pairwise_f32(a + n2, n - n2);
    }
}

float or_np_sum_f32(const float* a, int n) { return 0.0f + np_pairwise_f32(a, n); }

static int manhattan(int r0, int c0, int r1, int c1) { return abs(r0 - r1) + abs(c0 - c1); }

/* MAPPO/helper.py:257-369 (constants :271-279; QMIX/helper.py:270-278).
 * consts (Python numbers): pickup, on_time, late, closer, wasted_pick,
 * wasted_drop, stuck, idle, away.  move: MV_* codes (5 = any other string,
 * which is != 'S'); op: int(pkg_op_str) (0,1,2; 3 = other integer). */
float or_compute_shaped_rewards(double global_reward, int prev_t, const int32_t* prev1, int cur_t, const int32_t* cur1,
                                const uint8_t* move, const uint8_t* op, const int32_t* trk, int ntrk, int A,
                                const double* C) {
    float* s = (float*)calloc((size_t)(A > 0 ? A : 1), sizeof(float));
    const float PICK = (float)C[0], ONTIME = (float)C[1], LATE = (float)C[2], CLOSER = (float)C[3];
    const float WPICK = (float)C[4], WDROP = (float)C[5], STUCK = (float)C[6], IDLE = (float)C[7], AWAY = (float)C[8];
    int current_time = cur_t;
    for (int a = 0; a < A; a++) {
        int prev_r = prev1[3 * a] - 1, prev_c = prev1[3 * a + 1] - 1, prev_pkg = prev1[3 * a + 2];
        int curr_r = cur1[3 * a] - 1, curr_c = cur1[3 * a + 1] - 1, curr_pkg = cur1[3 * a + 2];
        int pkg_op = op[a];
        if (prev_pkg == 0 && curr_pkg != 0) {
            s[a] = s[a] + PICK;
        } else if (prev_pkg != 0 && curr_pkg == 0) {
            int q = trk_find(trk, ntrk, prev_pkg);
            if (q >= 0) {
                const int32_t* p = trk + 8 * q;
                if (curr_r == p[4] && curr_c == p[5]) {
                    if (current_time <= p[7]) s[a] = s[a] + ONTIME;
                    else s[a] = s[a] + LATE;
                }
            }
        }
        if (pkg_op == 1) {
            if (prev_pkg != 0) {
                s[a] = s[a] + WPICK;
            } else if (curr_pkg == 0) {
                int can = 0;
                for (int q = 0; q < ntrk; q++) {
                    const int32_t* p = trk + 8 * q;
                    if (p[1] == ST_WAITING && p[6] <= prev_t && p[2] == curr_r && p[3] == curr_c) { can = 1; break; }
                }
                if (!can) s[a] = s[a] + WPICK;
            }
        } else if (pkg_op == 2) {
            if (prev_pkg == 0) {
                s[a] = s[a] + WDROP;
            } else if (curr_pkg != 0) {
                int q = trk_find(trk, ntrk, prev_pkg);
                if (q >= 0) {
                    const int32_t* p = trk + 8 * q;
                    if (!(curr_r == p[4] && curr_c == p[5])) s[a] = s[a] + WDROP;
                }
            }
        }
        int moved = (prev_r != curr_r) || (prev_c != curr_c);
        int intended = move[a] != MV_S;
        if (intended && !moved) s[a] = s[a] + STUCK;
        int has_target = 0, tr = 0, tc = 0;
        int qp = prev_pkg != 0 ? trk_find(trk, ntrk, prev_pkg) : -1;
        if (prev_pkg != 0 && qp >= 0) {
            has_target = 1; tr = trk[8 * qp + 4]; tc = trk[8 * qp + 5];
        } else {
            int best = -1, bestd = 0;
            for (int q = 0; q < ntrk; q++) {
                const int32_t* p = trk + 8 * q;
                if (!(p[1] == ST_WAITING && p[6] <= prev_t)) continue;
                int d = manhattan(prev_r, prev_c, p[2], p[3]);
                if (best < 0 || d < bestd) { best = q; bestd = d; }      /* min(): first minimum */
            }
            if (best >= 0) { has_target = 1; tr = trk[8 * best + 2]; tc = trk[8 * best + 3]; }
        }
        if (has_target && moved) {
            int db = manhattan(prev_r, prev_c, tr, tc), da = manhattan(curr_r, curr_c, tr, tc);
            if (da < db) s[a] = s[a] + CLOSER;
            else if (da > db) s[a] = s[a] + AWAY;
        }
        if (!moved && move[a] == MV_S && prev_pkg == 0) {
            int idle = 0;
            for (int q = 0; q < ntrk; q++) {
                const int32_t* p = trk + 8 * q;
                if (p[1] == ST_WAITING && p[6] <= prev_t && manhattan(prev_r, prev_c, p[2], p[3]) <= 3) { idle = 1; break; }
            }
            if (idle) s[a] = s[a] + IDLE;
        }
    }
    float sum = or_np_sum_f32(s, A);
    float res = (float)global_reward + sum;
    free(s);
    return res;
}

/* ----------------------------------------------------------------------- */
/* Batched MAPPO rollout env path (MAPPO/trainer.py:194-286 without the    */
/* learner): decode -> step -> shaped reward (pre-update tracker) ->        */
/* reset-on-done -> tracker update.  Used for the CPU baseline and tests.   */
/* ----------------------------------------------------------------------- */
typedef struct {
    int E, A, P, T, tracker_clear_on_reset;
    OEnv** envs;
    OTrk** trk;
    int32_t* scratch_prev;
    int32_t* scratch_cur;
} OBatch;

static const uint8_t TRAINER_MOVE[5] = {MV_D, MV_L, MV_R, MV_S, MV_U};   /* LabelEncoder classes_ order */

static void env_robots1(const OEnv* e, int32_t* out) {
    for (int i = 0; i < e->A; i++) {
        out[3 * i] = e->robots[i].r + 1; out[3 * i + 1] = e->robots[i].c + 1; out[3 * i + 2] = e->robots[i].carrying;
    }
}

OBatch* or_batch_new(int E, const uint8_t* grid, int H, int W, int A, int P, int T, double mc, double dr, double dl,
                     uint32_t seed_base, int tracker_clear_on_reset) {
    OBatch* b = (OBatch*)calloc(1, sizeof(OBatch));
    b->E = E; b->A = A; b->P = P; b->T = T; b->tracker_clear_on_reset = tracker_clear_on_reset;
    b->envs = (OEnv**)calloc((size_t)E, sizeof(OEnv*));
    b->trk = (OTrk**)calloc((size_t)E, sizeof(OTrk*));
    b->scratch_prev = (int32_t*)malloc(sizeof(int32_t) * 3 * (size_t)A * E);
    b->scratch_cur = (int32_t*)malloc(sizeof(int32_t) * 3 * (size_t)A * E);
    for (int e = 0; e < E; e++) {
        b->envs[e] = or_env_new(grid, H, W, A, P, T, mc, dr, dl, seed_base + (uint32_t)e);  /* VectorizedEnv seed+idx */
        or_env_reset(b->envs[e]);                                                            /* vec_env.reset() */
        b->trk[e] = or_trk_new(P);
        or_trk_update_from_env(b->trk[e], b->envs[e]);
    }
    return b;
}

void or_batch_free(OBatch* b) {
    if (!b) return;
    for (int e = 0; e < b->E; e++) { or_env_free(b->envs[e]); or_trk_free(b->trk[e]); }
    free(b->envs); free(b->trk); free(b->scratch_prev); free(b->scratch_cur); free(b);
}

OEnv* or_batch_env(OBatch* b, int e) { return b->envs[e]; }
OTrk* or_batch_trk(OBatch* b, int e) { return b->trk[e]; }

void or_batch_step(OBatch* b, const uint8_t* actions_int, int auto_reset, const double* consts, double* r_env,
                   float* r_shaped, uint8_t* done, int n_threads) {
    (void)n_threads;
#pragma omp parallel for schedule(static) num_threads(n_threads > 0 ? n_threads : 1) if (n_threads > 1)
    for (int e = 0; e < b->E; e++) {
        OEnv* env = b->envs[e];
        int A = b->A;
        uint8_t mv[64], op[64];
        uint8_t* mvp = A <= 64 ? mv : (uint8_t*)malloc((size_t)A);
        uint8_t* opp = A <= 64 ? op : (uint8_t*)malloc((size_t)A);
        for (int a = 0; a < A; a++) {
            int x = actions_int[(size_t)e * A + a];
            mvp[a] = TRAINER_MOVE[x % 5];
            int o = x / 5;
            opp[a] = (uint8_t)(o >= 3 ? 0 : o);
        }
        int32_t* prev1 = b->scratch_prev + (size_t)3 * A * e;
        int32_t* cur1 = b->scratch_cur + (size_t)3 * A * e;
        env_robots1(env, prev1);
        int prev_t = env->t;
        double r;
        int r_int;
        int d = or_env_step(env, mvp, opp, &r, &r_int);
        env_robots1(env, cur1);
        float sh = or_compute_shaped_rewards(r, prev_t, prev1, env->t, cur1, mvp, opp, b->trk[e]->rows, b->trk[e]->n,
                                             A, consts);
        if (d && auto_reset) {
            or_env_reset(env);
            if (b->tracker_clear_on_reset) or_trk_clear(b->trk[e]);
        }
        or_trk_update_from_env(b->trk[e], env);
        r_env[e] = r;
        r_shaped[e] = sh;
        done[e] = (uint8_t)d;
        if (mvp != mv) free(mvp);
        if (opp != op) free(opp);
    }
}

/* The observations the MAPPO rollout builds after every step (MAPPO/trainer.py:261-280):      */
/* convert_global_state, then convert_observation and generate_vector_features per agent, of  */
/* every env's current state and tracker.  Outputs [E][A][6][H][W], [E][A][Dv], [E][4][H][W], */
/* [E][Dg]; any may be NULL.  The CPU leg of bench.py --config 3.                              */
void or_batch_obs(OBatch* b, int T, int MO, int MP, int MR, int MPs, float* amap, float* avec, float* cmap,
                  float* cvec, int n_threads) {
    (void)n_threads;
    const int A = b->A;
    const int H = b->envs[0]->H, W = b->envs[0]->W, HW = H * W;
    const size_t dv = 6 + 5 * (size_t)MO + 5 * (size_t)MP + 1, dg = 6 * (size_t)MR + 7 * (size_t)MPs + 1;
    float* gm_scratch = (float*)malloc(sizeof(float) * 4 * (size_t)HW * (n_threads > 0 ? n_threads : 1));
#pragma omp parallel for schedule(static) num_threads(n_threads > 0 ? n_threads : 1) if (n_threads > 1)
    for (int e = 0; e < b->E; e++) {
        const OEnv* env = b->envs[e];
        const OTrk* k = b->trk[e];
        int32_t rb[3 * 64];
        int32_t* r1 = A <= 64 ? rb : (int32_t*)malloc(sizeof(int32_t) * 3 * (size_t)A);
        env_robots1(env, r1);
        float* gm = cmap ? cmap + (size_t)e * 4 * HW : NULL;
        float* gv = cvec ? cvec + (size_t)e * dg : NULL;
        if (gm || gv) {
            int tid = 0;
#ifdef _OPENMP
            tid = omp_get_thread_num();
#endif
            float* gm_tmp = gm_scratch + (size_t)tid * 4 * HW;
            float* gv_tmp = gv ? gv : (float*)malloc(sizeof(float) * dg);
            or_convert_global_state(env->grid, H, W, env->t, A, r1, k->rows, k->n, T, MR, MPs, gm ? gm : gm_tmp,
                                    gv_tmp);
            if (!gv) free(gv_tmp);
        }
        for (int a = 0; a < A; a++) {
            if (amap)
                or_convert_observation(env->grid, H, W, env->t, A, r1, k->rows, k->n, a,
                                       amap + ((size_t)e * A + a) * 6 * HW);
            if (avec)
                or_generate_vector_features(H, W, env->t, A, r1, k->rows, k->n, a, T, MO, MP,
                                            avec + ((size_t)e * A + a) * dv);
        }
        if (r1 != rb) free(r1);
    }
    free(gm_scratch);
}

/* ----------------------------------------------------------------------- */
/* GreedyAgents (greedyagent.py), literal: BFS from the goal on every call, */
/* the package list exactly as the agent builds it (init_agents and the     */
/* first get_actions both append the t=0 spawns, so they appear twice, and  */
/* packages[id-1] / packages_free[id-1] index that list by id).             */
/* ----------------------------------------------------------------------- */
typedef struct {
    int A, P, n, is_init;
    int* list;          /* package ids in append order (greedyagent.py:60,135) */
    uint8_t* free_;     /* packages_free */
    int* target;        /* robots_target: 0 = 'free', else package id */
    ORobot* robots;     /* inner robots (0-indexed r, c, carrying) */
    int* bd;            /* BFS scratch: distances, queue */
    int* bq;
} OGreedy;

OGreedy* or_greedy_new(int A, int P, int H, int W) {
    OGreedy* g = (OGreedy*)calloc(1, sizeof(OGreedy));
    g->A = A; g->P = P;
    g->list = (int*)calloc((size_t)(2 * P + 1), sizeof(int));
    g->free_ = (uint8_t*)calloc((size_t)(2 * P + 1), 1);
    g->target = (int*)calloc((size_t)(A + 1), sizeof(int));
    g->robots = (ORobot*)calloc((size_t)(A + 1), sizeof(ORobot));
    g->bd = (int*)malloc(sizeof(int) * (size_t)H * W);
    g->bq = (int*)malloc(sizeof(int) * (size_t)H * W);
    return g;
}

void or_greedy_free(OGreedy* g) {
    if (!g) return;
    free(g->list); free(g->free_); free(g->target); free(g->robots); free(g->bd); free(g->bq); free(g);
}

/* state['packages'] = this step's spawns (env.py:133-137), appended in id order */
static void greedy_append(OGreedy* g, const OEnv* e) {
    for (int i = 0; i < e->P; i++)
        if (e->pkgs[i].start_time == e->t) {
            g->list[g->n] = e->pkgs[i].id;
            g->free_[g->n] = 1;
            g->n++;
        }
}

/* greedyagent.py:54-64 init_agents */
void or_greedy_init(OGreedy* g, const OEnv* e) {
    g->n = 0;
    g->is_init = 0;
    for (int i = 0; i < g->A; i++) {
        g->robots[i].r = e->robots[i].r;
        g->robots[i].c = e->robots[i].c;
        g->robots[i].carrying = 0;
        g->target[i] = 0;
    }
    greedy_append(g, e);
}

/* greedyagent.py:6-41 run_bfs(map, start, goal): returns the move, *dist = d after the move */
static int greedy_bfs(OGreedy* g, const OEnv* e, int sr, int sc, int gr, int gc, int* dist) {
    const int H = e->H, W = e->W;
    for (int i = 0; i < H * W; i++) g->bd[i] = -1;
    int qh = 0, qt = 0;
    g->bd[gr * W + gc] = 0;
    g->bq[qt++] = gr * W + gc;
    static const int DR[4] = {-1, 1, 0, 0}, DC[4] = {0, 0, -1, 1};
    while (qh < qt) {
        int cur = g->bq[qh++];
        int r = cur / W, c = cur % W;
        for (int k = 0; k < 4; k++) {
            int nr = r + DR[k], nc = c + DC[k];
            if (nr < 0 || nr >= H || nc < 0 || nc >= W) continue;
            if (g->bd[nr * W + nc] < 0 && e->grid[nr * W + nc] == 0) {
                g->bd[nr * W + nc] = g->bd[cur] + 1;
                g->bq[qt++] = nr * W + nc;
            }
        }
    }
    int ds = g->bd[sr * W + sc];
    if (ds < 0) { *dist = 100000; return MV_S; }
    static const int MOVES[4] = {MV_U, MV_D, MV_L, MV_R};   /* actions = ['U','D','L','R'] */
    for (int k = 0; k < 4; k++) {
        int nr = sr + DR[k], nc = sc + DC[k];
        if (nr < 0 || nr >= H || nc < 0 || nc >= W) continue;
        int dn = g->bd[nr * W + nc];
        if (dn >= 0 && dn == ds - 1) { *dist = dn; return MOVES[k]; }
    }
    *dist = ds;
    return MV_S;
}

/* greedyagent.py:66-102 update_move_to_target(robot, target_package_id = list index, phase) */
static void greedy_move_to(OGreedy* g, const OEnv* e, int i, int idx, int phase_target, uint8_t* mv, uint8_t* op) {
    const OPkg* p = &e->pkgs[g->list[idx] - 1];   /* self.packages[target_package_id] */
    int pr = phase_target ? p->tr : p->sr, pc = phase_target ? p->tc : p->sc;
    int distance = abs(pr - g->robots[i].r) + abs(pc - g->robots[i].c);
    int pkg_act = 0, move = MV_S;
    if (distance >= 1) {
        int d2;
        move = greedy_bfs(g, e, g->robots[i].r, g->robots[i].c, pr, pc, &d2);
        if (d2 == 0) pkg_act = phase_target ? 2 : 1;
    } else {
        pkg_act = phase_target ? 2 : 1;
    }
    mv[i] = (uint8_t)move;
    op[i] = (uint8_t)pkg_act;
}

/* greedyagent.py:104-170 update_inner_state + get_actions; mv/op: MV_* codes and 0/1/2 */
void or_greedy_actions(OGreedy* g, const OEnv* e, uint8_t* mv, uint8_t* op) {
    g->is_init = 1;
    for (int i = 0; i < g->A; i++) {                       /* update_inner_state */
        int prev_carry = g->robots[i].carrying;
        g->robots[i].r = e->robots[i].r;
        g->robots[i].c = e->robots[i].c;
        g->robots[i].carrying = e->robots[i].carrying;
        if (prev_carry != 0) g->target[i] = e->robots[i].carrying == 0 ? 0 : e->robots[i].carrying;
    }
    greedy_append(g, e);
    for (int i = 0; i < g->A; i++) {
        if (g->target[i] != 0) {
            int pid = g->target[i];
            greedy_move_to(g, e, i, pid - 1, g->robots[i].carrying != 0, mv, op);
        } else {
            int closest = 0, best = 1000000;
            for (int j = 0; j < g->n; j++) {
                if (!g->free_[j]) continue;
                const OPkg* p = &e->pkgs[g->list[j] - 1];
                int d = abs(p->sr - g->robots[i].r) + abs(p->sc - g->robots[i].c);
                if (d < best) { best = d; closest = g->list[j]; }
            }
            if (closest != 0) {
                g->free_[closest - 1] = 0;
                g->target[i] = closest;
                greedy_move_to(g, e, i, closest - 1, 0, mv, op);
            } else {
                mv[i] = MV_S;
                op[i] = 0;
            }
        }
    }
}

/* ----------------------------------------------------------------------- */
/* IDQ / qmix featurizers, literal.  Tracker rows are    */
/* (id, status 1 waiting / 2 in_transit, sr, sc, tr, tc, start, deadline),  */
/* robots1 are the state's (r+1, c+1, carrying).                            */
/* ----------------------------------------------------------------------- */
static double urgency_of(int t, int st, int dl) {
    double u = 0.0;
    if (dl > st) {
        u = (double)(t - st) / (double)(dl - st);
        u = u > 0.0 ? u : 0.0;
        u = u < 1.0 ? u : 1.0;
    } else if (dl == st) {
        u = t >= st ? 1.0 : 0.0;
    }
    return u;
}

/* IDQ/networks.py:112-217 convert_state (qmix/networks.py:243-348 is the same code) */
void or_idq_convert_state(const uint8_t* grid, int H, int W, int t, int A, const int32_t* robots1,
                          const int32_t* trk, int n, int idx, float* out) {
    memset(out, 0, sizeof(float) * 6 * (size_t)H * W);
    for (int i = 0; i < H * W; i++) out[i] = (float)grid[i];
    if (idx < 0 || idx >= A) return;
    int carried = robots1[3 * idx + 2];
    if (carried == 0) {
        for (int k = 0; k < n; k++) {
            const int32_t* p = trk + 8 * k;
            if (p[1] != 1) continue;                       /* status == 'waiting' */
            int sr = p[2], sc = p[3], st = p[6], dl = p[7];
            if (t >= st) {
                float u = (float)urgency_of(t, st, dl);
                if (sr >= 0 && sr < H && sc >= 0 && sc < W) {
                    float* c1 = &out[1 * H * W + sr * W + sc];
                    if (u > *c1) *c1 = u;                      /* max(tensor, urgency) */
                    out[2 * H * W + sr * W + sc] = 1.0f;
                }
            }
        }
    }
    for (int i = 0; i < A; i++) {
        if (i == idx) continue;
        int r = robots1[3 * i] - 1, c = robots1[3 * i + 1] - 1;
        if (r >= 0 && r < H && c >= 0 && c < W) out[3 * H * W + r * W + c] = 1.0f;
    }
    {
        int r = robots1[3 * idx] - 1, c = robots1[3 * idx + 1] - 1;
        if (r >= 0 && r < H && c >= 0 && c < W) out[4 * H * W + r * W + c] = 1.0f;
    }
    if (carried != 0) {
        for (int k = 0; k < n; k++) {
            const int32_t* p = trk + 8 * k;
            if (p[0] != carried) continue;                 /* carried id in persistent_packages */
            int tr = p[4], tc = p[5];
            if (tr >= 0 && tr < H && tc >= 0 && tc < W) out[5 * H * W + tr * W + tc] = 1.0f;
            break;
        }
    }
}

/* qmix/networks.py:350-468 convert_global_state_to_tensor, shape (7, oh, ow) */
void or_qmix_global_tensor(const uint8_t* grid, int H, int W, int t, int A, const int32_t* robots1,
                           const int32_t* trk, int n, int oh, int ow, float* out) {
    const size_t S = (size_t)oh * ow;
    memset(out, 0, sizeof(float) * 7 * S);
    int sr0 = H > oh ? (H - oh) / 2 : 0, sc0 = W > ow ? (W - ow) / 2 : 0;
    int rows = H < oh ? H : oh, cols = W < ow ? W : ow;
    int tro = (oh - rows) / 2, tco = (ow - cols) / 2;
    for (int r = 0; r < rows; r++)
        for (int c = 0; c < cols; c++) out[(size_t)(tro + r) * ow + tco + c] = (float)grid[(sr0 + r) * W + sc0 + c];
    for (int i = 0; i < A; i++) {
        int r = robots1[3 * i] - 1, c = robots1[3 * i + 1] - 1, cy = robots1[3 * i + 2];
        if (r >= 0 && r < oh && c >= 0 && c < ow) {
            out[1 * S + (size_t)r * ow + c] = 1.0f;
            if (cy != 0) out[2 * S + (size_t)r * ow + c] = 1.0f;
        }
    }
    for (int k = 0; k < n; k++) {
        const int32_t* p = trk + 8 * k;
        int sr = p[2], sc = p[3], tr = p[4], tc = p[5], st = p[6], dl = p[7];
        if (!(t >= st)) continue;
        if (p[1] == 1) {
            if (sr >= 0 && sr < oh && sc >= 0 && sc < ow) out[3 * S + (size_t)sr * ow + sc] = 1.0f;
            if (sr >= 0 && sr < oh && sc >= 0 && sc < ow) {
                double u = 0.0;
                if (dl > st) {
                    u = (double)(t - st) / (double)(dl - st);
                    u = u > 0.0 ? u : 0.0;
                    u = u < 1.0 ? u : 1.0;
                } else if (dl == st) {
                    u = 1.0;
                }
                float* c6 = &out[6 * S + (size_t)sr * ow + sc];
                if ((float)u > *c6) *c6 = (float)u;
            }
            if (tr >= 0 && tr < oh && tc >= 0 && tc < ow) out[4 * S + (size_t)tr * ow + tc] = 1.0f;
        } else if (p[1] == 2) {
            if (tr >= 0 && tr < oh && tc >= 0 && tc < ow) out[5 * S + (size_t)tr * ow + tc] = 1.0f;
        }
    }
}

/* IDQ/networks.py:228-349 reward_shaping.  ops: the actions' package ops as ints 0..3;
 * ops_are_ints = 0 reproduces IDQ/trainer.py's call with string ops ('1' != 1: no op branch). */
void or_idq_reward_shaping(int prev_t, const int32_t* prev1, int cur_t, const int32_t* cur1, const uint8_t* ops,
                           int ops_are_ints, const int32_t* trk, int n, int A, double* out) {
    for (int i = 0; i < A; i++) {
        double r = 0.0;
        int pr = prev1[3 * i] - 1, pc = prev1[3 * i + 1] - 1, pcy = prev1[3 * i + 2];
        int cr = cur1[3 * i] - 1, cc = cur1[3 * i + 1] - 1, ccy = cur1[3 * i + 2];
        if (pr == cr && pc == cc) r += -0.1;                             /* SHAPING_STAY_PENALTY */
        int op = ops_are_ints ? ops[i] : -1;
        if (op == 1) {
            if (pcy == 0 && ccy != 0) r += 2;                            /* successful pickup */
            else if (pcy != 0) r += -0.1;
            else if (pcy == 0 && ccy == 0) {
                int avail = 0;
                for (int k = 0; k < n; k++) {
                    const int32_t* p = trk + 8 * k;
                    if (p[1] == 1 && p[2] == pr && p[3] == pc && p[6] <= prev_t) { avail = 1; break; }
                }
                if (!avail) r += -0.1;
            }
        } else if (op == 2) {
            if (pcy != 0 && ccy == 0) {
                for (int k = 0; k < n; k++) {
                    const int32_t* p = trk + 8 * k;
                    if (p[0] != pcy) continue;
                    if (cr == p[4] && cc == p[5]) {
                        r += 10;                                          /* delivery bonus */
                        if (cur_t > p[7]) r += -5;                        /* late */
                    }
                    break;
                }
            } else if (pcy == 0) {
                r += 0;                                                   /* SHAPING_WASTED_DROP_PENALTY */
            }
        }
        out[i] = r;
    }
}
