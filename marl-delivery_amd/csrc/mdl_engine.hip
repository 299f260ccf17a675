// mdl_engine.hip -- host side of the C ABI declared in include/mdl_engine.h.
//
// Owns the engine's SoA state in HBM (hipMalloc), validates configurations the
// reference would reject (or loop forever on), builds the per-map tables
// (row-major free-cell lists for the reset draws, fp64 distance-rank tables
// for the feature sorts) and launches the kernels of mdl_kernels.hip.
#include "mdl_engine.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mdl_kernels.hpp"

namespace {
thread_local std::string g_err;
}  // namespace

// the library-wide error slot behind mdl_last_error() (mdl_kernels.hpp)
void mdl::set_error(const char* msg) { g_err = msg; }

namespace {

int fail(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return -1;
}

#define HIPCHK(x)                                                                       \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) return fail("%s failed: %s", #x, hipGetErrorString(e_)); \
    } while (0)

constexpr size_t LDS_BUDGET = 64 * 1024;  // dynamic LDS per 256-thread workgroup

// CPython float_pow(x, 2.0) -> libm pow(|x|, 2.0) (special cases 0 and 1).
// Called through a volatile pointer so the compiler cannot fold it to x*x:
// the reference's sort keys are exactly these doubles (MAPPO/helper.py:139,158).
double (*volatile g_pow)(double, double) = pow;
double py_sq(double x) {
    if (x == 0.0) return 0.0;
    if (x < 0) x = -x;
    if (x == 1.0) return 1.0;
    return g_pow(x, 2.0);
}

// rank[(dr+H-1)*(2W-1) + dc+W-1] = rank of (dr/H)**2 + (dc/W)**2 among all
// distinct values (equal doubles share a rank).
void build_rank(int H, int W, std::vector<uint16_t>& out) {
    const int R = 2 * H - 1, C = 2 * W - 1;
    std::vector<double> key((size_t)R * C);
    for (int dr = -(H - 1); dr <= H - 1; dr++)
        for (int dc = -(W - 1); dc <= W - 1; dc++)
            key[(size_t)(dr + H - 1) * C + (dc + W - 1)] = py_sq((double)dr / (double)H) + py_sq((double)dc / (double)W);
    std::vector<double> u = key;
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    out.resize(key.size());
    for (size_t i = 0; i < key.size(); i++)
        out[i] = (uint16_t)(std::lower_bound(u.begin(), u.end(), key[i]) - u.begin());
}

struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// Waves per workgroup of the step kernel for a launch over n envs: 4 (capped by the LDS budget,
// the reset scratch per wave).  Round 2 ran a chip-filling batch as ONE workgroup per CU (config
// 2's 4096 envs = 16 waves on each of 256 CUs: 4.47 -> 4.40 us per step then); with the
// XCD-contiguous slots (xcd_block) 4-wave workgroups are faster again: config 2 4.34-4.35 ->
// 4.22-4.25 us same box, 2- and 1-wave workgroups 4.24-4.27 / 4.38-4.40, config 5 unchanged
// (profiles/r03/step_wpb_ab.txt).
int step_wpb(int n, int n_cu, size_t lds_per_wave, int P) {
    (void)n;
    (void)n_cu;
    (void)P;
    int w = 4;
    if (lds_per_wave > 0) {
        const int cap = (int)(LDS_BUDGET / lds_per_wave);
        if (w > cap) w = cap;
    }
    return w < 1 ? 1 : w;
}

int waves_per_block(size_t lds_per_wave) {
    if (lds_per_wave == 0) return 4;
    size_t w = LDS_BUDGET / lds_per_wave;
    if (w > 4) w = 4;
    return (int)w;
}

// elements of padding after the package table, state words and tracker (see mdl_create)
constexpr size_t PKG_PAD = 256;

}  // namespace

struct MdlEngine {
    MdlConfig cfg{};
    int device = 0;
    mdl::DevParams p{};
    std::vector<int> mapH, mapW;
    std::vector<void*> allocs;
    size_t lds_step = 0, lds_obs = 0;
    bool step_rows = false;   // k_step_rows applies (A <= 8, P <= 64) and the layout allows it
    bool rows_forced = false; // MDL_STEP_LAYOUT_ROWS: at every batch size
    size_t lds_rows = 0;
    bool step_halves = false;   // k_step_halves applies (A == 16, P <= 128) and the layout allows it
    bool halves_forced = false; // MDL_STEP_LAYOUT_HALVES: at every batch size
    size_t lds_halves = 0;
    // Whether a full-batch step over n envs runs four envs per wavefront.  AUTO: from ROWS_MIN_ENVS
    // envs on.  Below that the step is latency bound -- one wave's dependent chain is longer for
    // k_step_rows, whose wave does four envs' work -- and one wave per env wins (4,096 envs: 4.19
    // vs 4.44 us per step, 6,144: 4.99 vs 5.32); above it the step is issue bound and the rows
    // layout's ~2x fewer instructions per env win (8,192 envs 5.83 vs 5.45 us, 10,240 6.75 vs 6.38,
    // config 4's 65,536 28.7 vs 21.1; profiles/r05/rows_ab.txt).
    static constexpr int ROWS_MIN_ENVS = 7168;
    bool rows_for(int n) const { return step_rows && (rows_forced || n >= ROWS_MIN_ENVS); }
    // Two envs per wavefront (k_step_halves, A == 16, P <= 128) from HALVES_MIN_ENVS envs on (AUTO):
    // below it one wave per env is as fast (8,192 envs: 8.56 vs 8.67 us per step), from 16,384 on the
    // halves layout is faster (13.65 vs 14.08, 65,536: 41.3 vs 45.6, config 5's 131,072: 76.1 vs
    // 84.1; profiles/r06/ab3/ab.txt).
    static constexpr int HALVES_MIN_ENVS = 12288;
    bool halves_for(int n) const { return step_halves && (halves_forced || n >= HALVES_MIN_ENVS); }
    // the layout mdl_step launches for a call over n envs (with an id list: always one wave per env)
    int32_t layout_for(int n, bool ids) const {
        if (ids) return MDL_STEP_LAYOUT_WAVE;
        if (rows_for(n)) return MDL_STEP_LAYOUT_ROWS;
        if (halves_for(n)) return MDL_STEP_LAYOUT_HALVES;
        return MDL_STEP_LAYOUT_WAVE;
    }
    size_t lds_for(int32_t layout) const {
        return layout == MDL_STEP_LAYOUT_ROWS ? lds_rows : layout == MDL_STEP_LAYOUT_HALVES ? lds_halves : lds_step;
    }
    int32_t last_step_layout = 0;   // MDL_STEP_LAYOUT_* of the last mdl_step launch (0: none yet)
    // A synchronous host-mapped call whose wait timed out leaves its launch queued on `hung`: until that
    // stream has drained, no call may rewrite the mailbox / arena inputs that launch still reads.
    bool poisoned = false;
    hipStream_t hung = nullptr;
    int wpb_step = 1, wpb_obs = 1;
    int obs_rank_lds = 0;   // small builder: LDS bytes of the largest map's rank table (0: ranks read from L2)
    int n_cu = 0;   // compute units of the device (step_wpb)
    int maxHW = 0;
    bool seeded = false;
    uint64_t map_fp = 0;  // FNV-1a of every map's (H, W, cells, env_map): checkpoint compatibility
    uint64_t cfg_fp = 0;  // FNV-1a of the reward / shaping constants and observation dims: checkpoint compatibility
    // shape_run_end[e]: end (exclusive) of env e's run of consecutive envs whose maps share one
    // (H, W); an observation range must lie inside one run (its output tensors have one shape)
    std::vector<int32_t> shape_run_end;
    // greedy baseline (mdl_greedy_*): BFS tables per map and one agent record per env, made on first use
    uint16_t* gtab = nullptr;
    unsigned char* gstate = nullptr;
    mdl::GreedyLayout glay{};
    bool greedy_stale = false;  // set by loading a checkpoint that has no greedy section
    // dict-API mailbox (mdl_mailbox / mdl_mail_*): one host-mapped allocation, made on first use
    void* mail = nullptr;
    MdlMailbox mbox{};
    unsigned* mail_ctr = nullptr;      // device: waves of every export so far (mod 2^32)
    unsigned mail_waves = 0;           // host mirror of *mail_ctr once the last export ended
    int32_t mail_seq = 0;              // last completion value published
    std::vector<uint8_t> mail_seen;    // duplicate-id check of a call
    // host-mapped arena of the helper-compatible calls (mdl_host_arena / mdl_host_wait)
    void* arena = nullptr;
    size_t arena_bytes = 0;
    int32_t arena_seq = 0;
    unsigned* arena_ctr = nullptr;     // device: waves of every self-publishing helper launch (mod 2^32)
    unsigned arena_waves = 0;          // host mirror of *arena_ctr once the last such launch ended

    // (device pointer, bytes) of every state buffer, in checkpoint order
    // (the greedy agents' records follow when with_greedy: they exist once mdl_greedy_init ran)
    std::vector<std::pair<void*, size_t>> state_sections(bool with_greedy) const {
        const size_t E = p.E, A = p.A, P = p.P;
        std::vector<std::pair<void*, size_t>> v = {
            {p.rob, E * A * 4},   {p.pkg, E * P * 8},        {p.pstate, E * P * 2},
            {p.es, E * 16},       {p.mt, E * mdl::MT_N * 4}, {p.mt_pos, E * 4},
            {p.trk, p.stale ? E * P * 8 : 0}, {p.ep_total, E * 8}, {p.ep_len, E * 4}};
        if (with_greedy) v.push_back({gstate, E * (size_t)greedy_stride()});
        return v;
    }
    // bytes per env of the greedy agent record (the layout greedy_alloc sets up)
    int greedy_stride() const {
        const int cap = 3 * p.P + 64, list_off = (8 + 4 * p.A + 3) & ~3;
        return (list_off + 2 * cap + cap + 15) & ~15;
    }
    bool has_greedy() const { return gstate != nullptr && !greedy_stale; }
    // Every observation build goes through here: the env range must lie inside one run of
    // same-shape envs (the small builder copies the rank table of the range's first env's map
    // into LDS for the whole launch, mdl_obs_small.hpp k_obs_small; the outputs have one H x W).
    hipError_t launch_obs(int env_begin, int n, float* am, float* av, float* cm, float* cv, hipStream_t s) const {
        if (env_begin < 0 || n <= 0 || env_begin + n > p.E || shape_run_end[env_begin] < env_begin + n)
            return hipErrorInvalidValue;
        return mdl::launch_obs(p, env_begin, n, am, av, cm, cv, wpb_obs, lds_obs, s, obs_rank_lds);
    }

    template <class T>
    int alloc(T** ptr, size_t count) {
        void* v = nullptr;
        const size_t bytes = count * sizeof(T) > 0 ? count * sizeof(T) : 16;
        hipError_t e = hipMalloc(&v, bytes);
        if (e != hipSuccess) return fail("hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
        allocs.push_back(v);
        e = hipMemset(v, 0, bytes);
        if (e != hipSuccess) return fail("hipMemset failed: %s", hipGetErrorString(e));
        *ptr = (T*)v;
        return 0;
    }
    ~MdlEngine() {
        for (void* v : allocs) (void)hipFree(v);
        if (mail) (void)hipHostFree(mail);
        if (arena) (void)hipHostFree(arena);
    }
};

extern "C" {

const char* mdl_last_error(void) { return g_err.c_str(); }
const char* mdl_version(void) { return "mdl-engine 0.1 gfx950"; }

int mdl_create(const MdlConfig* cfg, const uint8_t* grids, const int32_t* map_hw, int32_t n_maps,
               const int32_t* env_map, int32_t device, MdlEngine** out) {
    if (!cfg || !grids || !map_hw || !out) return fail("mdl_create: null argument");
    *out = nullptr;
    const MdlConfig& c = *cfg;
    if (c.n_envs < 1 || c.n_envs >= (1 << 24)) return fail("n_envs must be in [1, 2^24)");
    if (c.n_robots < 1 || c.n_robots > MDL_MAX_ROBOTS) return fail("n_robots must be in [1, %d]", MDL_MAX_ROBOTS);
    if (c.n_packages < 1 || c.n_packages > MDL_MAX_PACKAGES)
        return fail("n_packages must be in [1, %d]", MDL_MAX_PACKAGES);
    if (c.max_time_steps < 1) return fail("max_time_steps must be >= 1");
    if (n_maps < 1 || n_maps > mdl::MAX_MAPS) return fail("n_maps must be in [1, %d]", mdl::MAX_MAPS);
    if (c.tracker_mode != MDL_TRACKER_FRESH && c.tracker_mode != MDL_TRACKER_MAPPO_STALE)
        return fail("unknown tracker_mode %d", c.tracker_mode);
    if (c.max_other_robots < 0 || c.max_packages_obs < 0 || c.max_robots_state < 0 || c.max_packages_state < 0)
        return fail("observation slot counts must be >= 0");
    // env.py:113-116: start_time = randint(1, T) for packages beyond min(A,20)+1 -> needs T >= 2
    const int lim = c.n_robots < 20 ? c.n_robots : 20;
    if (c.n_packages > lim + 1 && c.max_time_steps < 2)
        return fail("max_time_steps must be >= 2 when n_packages > min(n_robots,20)+1 (numpy randint(1, T))");

    MdlEngine* eng = new MdlEngine();
    eng->cfg = c;
    eng->device = device;
    DeviceGuard dg(device);
    if (!dg.ok) {
        delete eng;
        return fail("hipSetDevice(%d) failed", device);
    }

    // ---- maps ----
    std::vector<uint8_t> allgrid, allvalid, allvalidc;
    int rank_max = 0;
    long dl_max = 0;
    std::vector<uint32_t> allbits;
    std::vector<uint16_t> allfree, allrank;
    mdl::DevParams& p = eng->p;
    size_t goff = 0;
    for (int m = 0; m < n_maps; m++) {
        const int H = map_hw[2 * m], W = map_hw[2 * m + 1];
        if (H < 1 || W < 1 || H > 255 || W > 255 || H * W > MDL_MAX_CELLS) {
            delete eng;
            return fail("map %d: H, W must be in [1,255] with H*W <= %d", m, MDL_MAX_CELLS);
        }
        const uint8_t* g = grids + goff;
        mdl::MapDesc& md = p.maps[m];
        md.H = H;
        md.W = W;
        md.grid_off = (int)allgrid.size();
        md.free_off = (int)allfree.size();
        md.rank_off = (int)allrank.size();
        md.inv_hw = 1.0f / (float)(H * W);
        md.bits_off = (int)allbits.size();
        md.mvc_off = (int)allvalidc.size();
        allvalidc.resize(allvalidc.size() + (size_t)256 * W, 0);
        for (int w = 0; w < (H * W + 31) / 32; w++) {
            uint32_t b = 0;
            for (int k = 0; k < 32; k++)
                if (w * 32 + k < H * W && grids[goff + w * 32 + k]) b |= 1u << k;
            allbits.push_back(b);
        }
        int nf = 0;
        for (int i = 0; i < H * W; i++) {
            if (g[i] > 1) {
                delete eng;
                return fail("map %d: cells must be 0 or 1", m);
            }
            allgrid.push_back(g[i]);
            // valid_position (env.py:336-345) of each move, bit = move code L1 R2 U3 D4
            const int r = i / W, col = i % W;
            uint8_t vm = 0;
            if (col - 1 >= 0 && g[i - 1] != 1) vm |= 1u << 1;
            if (col + 1 < W && g[i + 1] != 1) vm |= 1u << 2;
            if (r - 1 >= 0 && g[i - W] != 1) vm |= 1u << 3;
            if (r + 1 < H && g[i + W] != 1) vm |= 1u << 4;
            allvalid.push_back(vm);
            allvalidc[(size_t)md.mvc_off + ((size_t)col << 8 | (size_t)r)] = vm;
            if (g[i] == 0) {
                allfree.push_back((uint16_t)((i / W) | ((i % W) << 8)));
                nf++;
            }
        }
        md.nfree = nf;
        if (nf < c.n_robots) {
            delete eng;
            return fail("map %d has %d free cells < n_robots %d (numpy randint(0, 0) raises)", m, nf, c.n_robots);
        }
        if (nf < 2) {
            delete eng;
            return fail("map %d needs >= 2 free cells (start != target loop, env.py:107-111)", m);
        }
        if ((long)c.max_time_steps - 1 + 10 + 3L * H > 65535) {
            delete eng;
            return fail("deadlines must fit 16 bits (T + 3H + 9 <= 65535)");
        }
        std::vector<uint16_t> rk;
        build_rank(H, W, rk);
        for (uint16_t v : rk) rank_max = std::max<int>(rank_max, v);
        dl_max = std::max<long>(dl_max, (long)c.max_time_steps - 1 + 10 + 3L * H);
        allrank.insert(allrank.end(), rk.begin(), rk.end());
        eng->mapH.push_back(H);
        eng->mapW.push_back(W);
        eng->maxHW = std::max(eng->maxHW, H * W);
        goff += (size_t)H * W;
    }
    std::vector<uint8_t> em;
    if (env_map && n_maps == 1) env_map = nullptr;  // single map: no per-env lookup in the kernels
    if (env_map) {
        em.resize(c.n_envs);
        for (int e = 0; e < c.n_envs; e++) {
            if (env_map[e] < 0 || env_map[e] >= n_maps) {
                delete eng;
                return fail("env_map[%d] = %d out of range", e, env_map[e]);
            }
            em[e] = (uint8_t)env_map[e];
        }
    }

    p.E = c.n_envs;
    p.A = c.n_robots;
    p.P = c.n_packages;
    p.T = c.max_time_steps;
    p.move_cost = c.move_cost;
    p.delivery_reward = c.delivery_reward;
    p.delay_reward = c.delay_reward;
    {
        double acc = 0.0;   // ((0.0 + move_cost) + move_cost) ... k times: env.py:252-257's fold
        for (int k = 0; k < 65; k++) {
            if (k < 9) p.cost_sum[k] = acc;
            p.cost_fold[k] = acc;
            acc += c.move_cost;
        }
    }
    for (int i = 0; i < 9; i++) p.shaping[i] = (float)c.shaping[i];  // NEP 50: constants rounded to float32
    p.stale = c.tracker_mode == MDL_TRACKER_MAPPO_STALE;
    p.obsT = c.obs_max_time_steps;
    p.MO = c.max_other_robots;
    p.MP = c.max_packages_obs;
    p.MR = c.max_robots_state;
    p.MPs = c.max_packages_state;
    p.n_maps = n_maps;
    {   // 32-bit obs sort keys: order (11 bits) | rank << 11 | max(0, dl - t) << (11 + rank bits)
        auto bits = [](long v) { int b = 0; while (v > 0) { b++; v >>= 1; } return b; };
        const int rb = bits(rank_max), db = bits(dl_max);
        p.key32_dsh = (11 + rb + db <= 32) ? 11 + rb : 0;
        p.key7_dsh = (7 + rb + db <= 32) ? 7 + rb : 0;
    }

    const size_t E = c.n_envs, A = c.n_robots, P = c.n_packages;
    uint8_t *d_grid = nullptr, *d_valid = nullptr;
    uint32_t* d_bits = nullptr;
    uint16_t *d_free = nullptr, *d_rank = nullptr;
    uint8_t* d_em = nullptr;
    int rc = 0;
    rc |= eng->alloc(&d_grid, allgrid.size());
    rc |= eng->alloc(&d_valid, allvalid.size());
    uint8_t* d_validc = nullptr;
    rc |= eng->alloc(&d_validc, allvalidc.size());
    rc |= eng->alloc(&d_bits, allbits.size());
    rc |= eng->alloc(&d_free, allfree.size());
    rc |= eng->alloc(&d_rank, allrank.size());
    // fp64 reciprocals for the observation builders' divisions (qdiv_r)
    std::vector<double> recip;
    for (int m = 0; m < n_maps; m++) {
        recip.push_back(1.0 / (double)eng->mapH[m]);
        recip.push_back(1.0 / (double)eng->mapW[m]);
    }
    recip.push_back(c.obs_max_time_steps > 0 ? 1.0 / (double)c.obs_max_time_steps : 0.0);
    recip.push_back(c.max_robots_state > 1 ? 1.0 / (double)(c.max_robots_state - 1) : 0.0);
    double* d_recip = nullptr;
    rc |= eng->alloc(&d_recip, recip.size());
    if (env_map) rc |= eng->alloc(&d_em, E);
    rc |= eng->alloc(&p.rob, E * A);
    // the package buffers end in 256 slots of padding: the multi-env step kernels load every lane's
    // slot past an env's P without clamping (k_step_halves: up to the last env's slot 127)
    rc |= eng->alloc(&p.pkg, E * P + PKG_PAD);
    rc |= eng->alloc(&p.pstate, E * P + PKG_PAD);
    rc |= eng->alloc(&p.es, E);
    rc |= eng->alloc(&p.mt, E * mdl::MT_N);
    rc |= eng->alloc(&p.mt_pos, E);
    rc |= eng->alloc(&p.trk, (p.stale ? E : 1) * P + PKG_PAD);
    rc |= eng->alloc(&p.ep_total, E);
    rc |= eng->alloc(&p.ep_len, E);
    if (rc) {
        std::string msg = g_err;
        delete eng;
        return fail("%s", msg.c_str());
    }
    if (hipMemcpy(d_grid, allgrid.data(), allgrid.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_valid, allvalid.data(), allvalid.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_validc, allvalidc.data(), allvalidc.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_bits, allbits.data(), allbits.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_free, allfree.data(), allfree.size() * 2, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_rank, allrank.data(), allrank.size() * 2, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_recip, recip.data(), recip.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
        (env_map && hipMemcpy(d_em, em.data(), E, hipMemcpyHostToDevice) != hipSuccess)) {
        delete eng;
        return fail("hipMemcpy of map tables failed");
    }
    p.grids = d_grid;
    p.movevalid = d_valid;
    p.movevalid_cell = d_validc;
    p.gridbits = d_bits;
    p.free_cells = d_free;
    p.rank = d_rank;
    p.obs_recip = d_recip;
    p.env_map = d_em;
    {
        uint64_t h = 1469598103934665603ull;
        auto mix = [&h](uint64_t v) {
            for (int b = 0; b < 8; b++) {
                h ^= (v >> (8 * b)) & 0xff;
                h *= 1099511628211ull;
            }
        };
        for (int m = 0; m < n_maps; m++) mix(((uint64_t)eng->mapH[m] << 32) | (uint32_t)eng->mapW[m]);
        for (uint8_t v : allgrid) mix(v);
        for (uint8_t v : em) mix(v);
        eng->map_fp = h;
        h = 1469598103934665603ull;
        auto mixd = [&mix](double d) { uint64_t v; memcpy(&v, &d, 8); mix(v); };
        mixd(c.move_cost);
        mixd(c.delivery_reward);
        mixd(c.delay_reward);
        for (int i = 0; i < 9; i++) mixd(c.shaping[i]);
        mix((uint64_t)(uint32_t)c.obs_max_time_steps);
        mix(((uint64_t)(uint32_t)c.max_other_robots << 32) | (uint32_t)c.max_packages_obs);
        mix(((uint64_t)(uint32_t)c.max_robots_state << 32) | (uint32_t)c.max_packages_state);
        eng->cfg_fp = h;
    }
    eng->shape_run_end.assign(c.n_envs, c.n_envs);
    for (int e = c.n_envs - 2; e >= 0; e--) {
        const int m0 = env_map ? env_map[e] : 0, m1 = env_map ? env_map[e + 1] : 0;
        const bool same = eng->mapH[m0] == eng->mapH[m1] && eng->mapW[m0] == eng->mapW[m1];
        eng->shape_run_end[e] = same ? eng->shape_run_end[e + 1] : e + 1;
    }

    eng->lds_step = mdl::step_lds((int)P);
    eng->wpb_step = waves_per_block(eng->lds_step);
    if (c.step_layout != MDL_STEP_LAYOUT_AUTO && c.step_layout != MDL_STEP_LAYOUT_WAVE &&
        c.step_layout != MDL_STEP_LAYOUT_ROWS && c.step_layout != MDL_STEP_LAYOUT_HALVES)
        return fail("unknown step_layout %d", c.step_layout);
    if (c.step_layout == MDL_STEP_LAYOUT_ROWS && !mdl::step_rows_ok((int)A, (int)P))
        return fail("step_layout ROWS needs A <= 8 and P <= 64 (A=%d P=%d)", (int)A, (int)P);
    if (c.step_layout == MDL_STEP_LAYOUT_HALVES && !mdl::step_halves_ok((int)A, (int)P))
        return fail("step_layout HALVES needs A == 16 and P <= 128 (A=%d P=%d)", (int)A, (int)P);
    const bool auto_l = c.step_layout == MDL_STEP_LAYOUT_AUTO;
    eng->step_rows = (auto_l || c.step_layout == MDL_STEP_LAYOUT_ROWS) && mdl::step_rows_ok((int)A, (int)P);
    eng->rows_forced = c.step_layout == MDL_STEP_LAYOUT_ROWS;
    eng->lds_rows = mdl::step_rows_lds((int)P);
    eng->step_halves = (auto_l || c.step_layout == MDL_STEP_LAYOUT_HALVES) && mdl::step_halves_ok((int)A, (int)P);
    eng->halves_forced = c.step_layout == MDL_STEP_LAYOUT_HALVES;
    eng->lds_halves = mdl::step_halves_lds((int)P);
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess) eng->n_cu = prop.multiProcessorCount;
    }
    p.obs_plane_words = mdl::obs_plane_words((int)A, eng->maxHW);
    if (c.obs_builder != MDL_OBS_BUILDER_AUTO && c.obs_builder != MDL_OBS_BUILDER_GENERIC)
        return fail("unknown obs_builder %d", c.obs_builder);
    p.obs_small = mdl::obs_use_small((int)A, (int)P, p.key7_dsh, eng->maxHW, p.MO, p.MP) &&
                  c.obs_builder == MDL_OBS_BUILDER_AUTO;
    eng->lds_obs = p.obs_small ? mdl::obs_lds_small((int)A, eng->maxHW, (int)P, p.MO, p.MP)
                               : mdl::obs_lds((int)A, (int)P, eng->maxHW, p.MO, p.MP, p.MR, p.MPs);
    eng->wpb_obs = waves_per_block(eng->lds_obs);
    // Worth it when the actor vectors take several tuple passes (each gathers ranks): config 3b
    // (MO = MP = 100) 141-143 -> 135-137 us per build; with one pass (config 3) the block's table copy
    // and barrier cost more than the two gathers they save (74.5 -> 76 us; profiles/r04/obs_rank_lds_ab.txt)
    const int MPc_ = p.MP < (int)P ? p.MP : (int)P;
    if (p.obs_small && (int)(A * A + A * MPc_ + A) > 64) {
        for (int m = 0; m < n_maps; m++)
            eng->obs_rank_lds = std::max(eng->obs_rank_lds, (int)(((2 * eng->mapH[m] - 1) * (2 * eng->mapW[m] - 1) * 2 + 15) & ~15));
        // a workgroup's LDS: the table + wpb slices, within the per-CU budget of the builder's occupancy
        if ((size_t)eng->obs_rank_lds + eng->lds_obs * eng->wpb_obs > LDS_BUDGET || eng->obs_rank_lds > 8192)
            eng->obs_rank_lds = 0;
    }
    if (eng->wpb_step < 1 || eng->wpb_obs < 1) {
        delete eng;
        return fail("configuration needs more than %zu bytes of LDS per env", LDS_BUDGET);
    }
    *out = eng;
    return 0;
}

int mdl_destroy(MdlEngine* eng) {
    if (!eng) return 0;
    DeviceGuard dg(eng->device);
    (void)hipDeviceSynchronize();
    delete eng;
    return 0;
}

int mdl_seed(MdlEngine* eng, const uint32_t* seeds, void* stream) {
    if (!eng || !seeds) return fail("mdl_seed: null argument");
    DeviceGuard dg(eng->device);
    hipStream_t s = (hipStream_t)stream;
    uint32_t* d = nullptr;
    const size_t bytes = sizeof(uint32_t) * eng->p.E;
    HIPCHK(hipMalloc(&d, bytes));
    hipError_t e = hipMemcpyAsync(d, seeds, bytes, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = mdl::launch_seed(eng->p, d, eng->wpb_step, eng->lds_step, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(d);
    if (e != hipSuccess) return fail("mdl_seed: %s", hipGetErrorString(e));
    eng->seeded = true;
    return 0;
}

int mdl_reset(MdlEngine* eng, const int32_t* env_ids, int32_t n, void* stream) {
    if (!eng) return fail("mdl_reset: null engine");
    if (!eng->seeded) return fail("mdl_reset: engine not seeded (call mdl_seed first)");
    if (!env_ids) n = eng->p.E;
    if (n < 0 || n > eng->p.E) return fail("mdl_reset: n=%d out of range", n);
    if (n == 0) return 0;
    DeviceGuard dg(eng->device);
    HIPCHK(mdl::launch_reset(eng->p, env_ids, n, eng->wpb_step, eng->lds_step, (hipStream_t)stream));
    return 0;
}

int mdl_tracker_clear(MdlEngine* eng, const int32_t* env_ids, int32_t n, void* stream) {
    if (!eng) return fail("mdl_tracker_clear: null engine");
    if (!eng->p.stale) return 0;  // fresh tracker has no storage
    if (!env_ids) n = eng->p.E;
    if (n < 0 || n > eng->p.E) return fail("mdl_tracker_clear: n=%d out of range", n);
    if (n == 0) return 0;
    DeviceGuard dg(eng->device);
    HIPCHK(mdl::launch_tracker_clear(eng->p, env_ids, n, (hipStream_t)stream));
    return 0;
}

int mdl_step(MdlEngine* eng, const uint8_t* actions, int32_t action_format, const int32_t* env_ids, int32_t n,
             int32_t auto_reset, double* r_env, float* r_shaped, uint8_t* done, void* stream) {
    if (!eng || !actions) return fail("mdl_step: null argument");
    if (!eng->seeded) return fail("mdl_step: engine not seeded (call mdl_seed first)");
    if (action_format != MDL_ACTION_TRAINER_INT && action_format != MDL_ACTION_CODES)
        return fail("mdl_step: unknown action_format %d", action_format);
    if (!env_ids) n = eng->p.E;
    if (n < 0 || n > eng->p.E) return fail("mdl_step: n=%d out of range", n);
    if (n == 0) return 0;
    DeviceGuard dg(eng->device);
    const int32_t layout = eng->layout_for(n, env_ids != nullptr);
    eng->last_step_layout = layout;
    if (layout == MDL_STEP_LAYOUT_ROWS) {
        HIPCHK(mdl::launch_step_rows(eng->p, actions, action_format, n, auto_reset, r_env, r_shaped, done,
                                     step_wpb(n, eng->n_cu, eng->lds_rows, eng->p.P), eng->lds_rows,
                                     (hipStream_t)stream));
        return 0;
    }
    if (layout == MDL_STEP_LAYOUT_HALVES) {
        HIPCHK(mdl::launch_step_halves(eng->p, actions, action_format, n, auto_reset, r_env, r_shaped, done,
                                       step_wpb(n, eng->n_cu, eng->lds_halves, eng->p.P), eng->lds_halves,
                                       (hipStream_t)stream));
        return 0;
    }
    HIPCHK(mdl::launch_step(eng->p, actions, action_format, env_ids, n, auto_reset, r_env, r_shaped, done,
                            step_wpb(n, eng->n_cu, eng->lds_step, eng->p.P), eng->lds_step, (hipStream_t)stream));
    return 0;
}

int mdl_step_floor(MdlEngine* eng, int32_t n, void* stream) {
    if (!eng) return fail("mdl_step_floor: null engine");
    if (n < 1 || n > eng->p.E) return fail("mdl_step_floor: n=%d out of range", n);
    DeviceGuard dg(eng->device);
    // the launch shape of a full-batch mdl_step over n envs (the layout mdl_step takes for it)
    const int32_t layout = eng->layout_for(n, false);
    const size_t lds = eng->lds_for(layout);
    const int epw = layout == MDL_STEP_LAYOUT_ROWS ? 4 : layout == MDL_STEP_LAYOUT_HALVES ? 2 : 1;
    HIPCHK(mdl::launch_step_floor(eng->p, n, step_wpb(n, eng->n_cu, lds, eng->p.P), lds, (hipStream_t)stream, epw));
    return 0;
}

int mdl_step_obs(MdlEngine* eng, const uint8_t* actions, int32_t action_format, int32_t auto_reset, double* r_env,
                 float* r_shaped, uint8_t* done, float* actor_map, float* actor_vec, float* critic_map,
                 float* critic_vec, void* stream) {
    if (!eng || !actions) return fail("mdl_step_obs: null argument");
    if (!eng->seeded) return fail("mdl_step_obs: engine not seeded (call mdl_seed first)");
    if (action_format != MDL_ACTION_TRAINER_INT && action_format != MDL_ACTION_CODES)
        return fail("mdl_step_obs: unknown action_format %d", action_format);
    const int E = eng->p.E;
    if (eng->shape_run_end[0] < E)
        return fail("mdl_step_obs: the envs mix map shapes (same-shape run ends at %d); use mdl_step + mdl_build_obs "
                    "per group", eng->shape_run_end[0]);
    DeviceGuard dg(eng->device);
    hipStream_t s = (hipStream_t)stream;
    if (eng->p.obs_small && eng->p.A <= 8 && eng->p.P <= 64) {
        const size_t lds = std::max(eng->lds_step, eng->lds_obs);   // one slice: reset scratch, then the planes
        if (lds <= LDS_BUDGET) {   // else: the two-launch path below
            const int wpb = step_wpb(E, eng->n_cu, lds, eng->p.P);
            HIPCHK(mdl::launch_step_obs(eng->p, actions, action_format, E, auto_reset, r_env, r_shaped, done,
                                        actor_map, actor_vec, critic_map, critic_vec, wpb, lds, s));
            return 0;
        }
    }
    HIPCHK(mdl::launch_step(eng->p, actions, action_format, nullptr, E, auto_reset, r_env, r_shaped, done,
                            step_wpb(E, eng->n_cu, eng->lds_step, eng->p.P), eng->lds_step, s));
    HIPCHK(eng->launch_obs(0, E, actor_map, actor_vec, critic_map, critic_vec, s));
    return 0;
}

int mdl_step_fused(MdlEngine* eng, const uint8_t* actions, int32_t action_format, const int32_t* env_ids, int32_t n,
                   int32_t k_steps, int32_t auto_reset, double* r_env, float* r_shaped, uint8_t* done, void* stream) {
    if (!eng || !actions) return fail("mdl_step_fused: null argument");
    if (!eng->seeded) return fail("mdl_step_fused: engine not seeded (call mdl_seed first)");
    if (action_format != MDL_ACTION_TRAINER_INT && action_format != MDL_ACTION_CODES)
        return fail("mdl_step_fused: unknown action_format %d", action_format);
    if (!env_ids) n = eng->p.E;
    if (n < 0 || n > eng->p.E) return fail("mdl_step_fused: n=%d out of range", n);
    if (k_steps < 1) return fail("mdl_step_fused: k_steps=%d must be >= 1", k_steps);
    if (n == 0) return 0;
    DeviceGuard dg(eng->device);
    HIPCHK(mdl::launch_step_fused(eng->p, actions, action_format, env_ids, n, k_steps, auto_reset, r_env, r_shaped,
                                  done, step_wpb(n, eng->n_cu, eng->lds_step, eng->p.P), eng->lds_step, (hipStream_t)stream));
    return 0;
}

// ---- dict-API mailbox: Environment.step / reset with one launch pair and no copies ----
static_assert(mdl::RT_MOVE == MDL_RTERM_MOVE && mdl::RT_ONTIME == MDL_RTERM_ONTIME && mdl::RT_LATE == MDL_RTERM_LATE,
              "reward-term bits of the header and the kernels");
int mdl_mailbox(MdlEngine* eng, MdlMailbox* out) {
    if (!eng || !out) return fail("mdl_mailbox: null argument");
    if (!eng->mail) {
        DeviceGuard dg(eng->device);
        const size_t E = eng->p.E, A = eng->p.A, P = eng->p.P;
        // 16-byte aligned sections: seq | codes | ids | r_env | r_shaped | done | robots | pkgs | t | total | rterms
        const size_t sz[11] = {16, E * A, E * 4, E * 8, E * 4, E, E * A * 12, E * P * 32, E * 4, E * 8, E * 4};
        size_t off[11], tot = 0;
        for (int i = 0; i < 11; i++) {
            off[i] = tot;
            tot += (sz[i] + 15) & ~(size_t)15;
        }
        // fine-grained (coherent) and mapped: the kernels read the inputs and write the rows in place,
        // the host reads them as soon as the completion word changes
        // the completion counter first: a mailbox exists only with everything it needs
        if (!eng->mail_ctr && eng->alloc(&eng->mail_ctr, 1)) return -1;
        HIPCHK(hipHostMalloc(&eng->mail, tot, hipHostMallocCoherent | hipHostMallocMapped));
        memset(eng->mail, 0, tot);
        char* b = (char*)eng->mail;
        MdlMailbox& m = eng->mbox;
        m.seq = (int32_t*)(b + off[0]);
        m.codes = (uint8_t*)(b + off[1]);
        m.ids = (int32_t*)(b + off[2]);
        m.r_env = (double*)(b + off[3]);
        m.r_shaped = (float*)(b + off[4]);
        m.done = (uint8_t*)(b + off[5]);
        m.robots = (int32_t*)(b + off[6]);
        m.pkgs = (int32_t*)(b + off[7]);
        m.t = (int32_t*)(b + off[8]);
        m.total_reward = (double*)(b + off[9]);
        m.rterms = (int32_t*)(b + off[10]);
        eng->mail_seen.assign(E, 0);
    }
    *out = eng->mbox;
    return 0;
}

namespace {
// The ids of a mailbox call (host memory, so checked here): in [0, E), no repeats.
int mail_check_ids(MdlEngine* eng, int32_t n, int32_t use_ids, const char* who) {
    if (!eng->mail) return fail("%s: call mdl_mailbox first", who);
    if (n < 0 || n > eng->p.E || (!use_ids && n != eng->p.E))
        return fail("%s: n=%d (use_ids=%d) out of range for %d envs", who, n, use_ids, eng->p.E);
    if (!use_ids) return 0;
    const int32_t* ids = eng->mbox.ids;
    int rc = 0;
    for (int i = 0; i < n && !rc; i++) {
        const int32_t e = ids[i];
        if (e < 0 || e >= eng->p.E) rc = fail("%s: env id %d out of range [0, %d)", who, e, eng->p.E);
        else if (eng->mail_seen[e]) rc = fail("%s: env id %d listed twice", who, e);
        else eng->mail_seen[e] = 1;
    }
    for (int i = 0; i < n; i++)
        if (ids[i] >= 0 && ids[i] < eng->p.E) eng->mail_seen[ids[i]] = 0;
    return rc;
}

// Spin until the device publishes `want` in the host-mapped word `seq` (written last, with a
// system-scope release, by the final kernel of the call): no stream synchronisation, whose
// wake-up costs microseconds more.  A failed launch never publishes, so the stream is asked now
// and then.
// The synchronous dict-API calls spin here (the callers hold the GIL: a call is microseconds to a
// few milliseconds), so a GPU that never publishes must not hang the process: past
// SPIN_LIMIT_S seconds with the stream still busy the call fails instead of spinning on.
constexpr double SPIN_LIMIT_S = 60.0;
// Refuses host-mapped I/O while a timed-out call's launch may still be queued (spin_wait): that
// launch reads the mailbox / arena inputs and publishes a sequence value, so a new call could hand
// it new inputs or misread its completion.  Cleared once the stream it was queued on has drained.
int host_io_ok(MdlEngine* eng, const char* who) {
    if (!eng->poisoned) return 0;
    const hipError_t q = hipStreamQuery(eng->hung);
    if (q == hipSuccess) {
        eng->poisoned = false;
        return 0;
    }
    return fail("%s: an earlier synchronous call on this engine timed out with its launch still queued (%s); "
                "refused until that stream has drained", who, q == hipErrorNotReady ? "still running" : hipGetErrorString(q));
}
int spin_wait(MdlEngine* eng, volatile const int32_t* seq, int32_t want, hipStream_t s, const char* who) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned long spins = 1;; spins++) {
        if (*seq == want) return 0;
        __builtin_ia32_pause();
        if ((spins & 0xffff) == 0) {
            const hipError_t q = hipStreamQuery(s);
            if (q != hipSuccess && q != hipErrorNotReady) return fail("%s: %s", who, hipGetErrorString(q));
            if (q == hipSuccess && *seq != want) return fail("%s: the call finished without publishing", who);
            const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (el > SPIN_LIMIT_S) {
                eng->poisoned = true;   // the launch may still read the host-mapped inputs: see host_io_ok
                eng->hung = s;
                return fail("%s: no completion after %.0f s (stream still busy): giving up the wait; host-mapped "
                            "calls on this engine are refused until that stream has drained", who, el);
            }
        }
    }
}

// export the call's rows into the mailbox, then wait (spinning) for the completion word
int mail_finish(MdlEngine* eng, int32_t n, int32_t use_ids, hipStream_t s, const char* who) {
    const MdlMailbox& m = eng->mbox;
    const int32_t want = eng->mail_seq = (eng->mail_seq % 0x7ffffff0) + 1;
    mdl::MailRows rows{m.seq, m.robots, m.pkgs, m.t, m.total_reward, m.rterms};
    const unsigned base = eng->mail_waves;
    HIPCHK(mdl::launch_mail_export(eng->p, use_ids ? m.ids : nullptr, n, rows, eng->mail_ctr, base, want, s));
    eng->mail_waves += mdl::mail_export_waves(n);   // the device counter's value after this launch
    return spin_wait(eng, m.seq, want, s, who);
}
}  // namespace

int mdl_mail_step(MdlEngine* eng, int32_t n, int32_t use_ids, int32_t auto_reset, void* stream) {
    if (!eng) return fail("mdl_mail_step: null engine");
    if (!eng->seeded) return fail("mdl_mail_step: engine not seeded (call mdl_seed first)");
    if (mail_check_ids(eng, n, use_ids, "mdl_mail_step")) return -1;
    if (host_io_ok(eng, "mdl_mail_step")) return -1;
    if (n == 0) return 0;
    DeviceGuard dg(eng->device);
    hipStream_t s = (hipStream_t)stream;
    const MdlMailbox& m = eng->mbox;
    // one launch: the step, its rows into the mailbox, the completion word (k_step_mail)
    const int32_t want = eng->mail_seq = (eng->mail_seq % 0x7ffffff0) + 1;
    const mdl::MailRows rows{m.seq, m.robots, m.pkgs, m.t, m.total_reward, m.rterms};
    HIPCHK(mdl::launch_step_mail(eng->p, m.codes, use_ids ? m.ids : nullptr, n, auto_reset, m.r_env, m.r_shaped,
                                 m.done, step_wpb(n, eng->n_cu, eng->lds_step, eng->p.P), eng->lds_step, rows,
                                 eng->mail_ctr, eng->mail_waves, want, s));
    eng->mail_waves += (unsigned)n;   // the n waves of rows [0, n) counted themselves
    return spin_wait(eng, m.seq, want, s, "mdl_mail_step");
}

int mdl_mail_reset(MdlEngine* eng, int32_t n, int32_t use_ids, void* stream) {
    if (!eng) return fail("mdl_mail_reset: null engine");
    if (!eng->seeded) return fail("mdl_mail_reset: engine not seeded (call mdl_seed first)");
    if (mail_check_ids(eng, n, use_ids, "mdl_mail_reset")) return -1;
    if (host_io_ok(eng, "mdl_mail_reset")) return -1;
    if (n == 0) return 0;
    DeviceGuard dg(eng->device);
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(mdl::launch_reset(eng->p, use_ids ? eng->mbox.ids : nullptr, n, eng->wpb_step, eng->lds_step, s));
    return mail_finish(eng, n, use_ids, s, "mdl_mail_reset");
}

int mdl_host_arena(MdlEngine* eng, int64_t bytes, void** out) {
    if (!eng || !out || bytes < 0) return fail("mdl_host_arena: bad argument");
    if (host_io_ok(eng, "mdl_host_arena")) return -1;   // a queued launch may still use the arena
    if (!eng->arena || (size_t)bytes > eng->arena_bytes) {
        size_t cap = 64 * 1024;
        while (cap < (size_t)bytes) cap *= 2;
        DeviceGuard dg(eng->device);
        if (eng->arena) {   // every call on it has returned (the waits are synchronous)
            (void)hipHostFree(eng->arena);
            eng->arena = nullptr;
        }
        if (!eng->arena_ctr && eng->alloc(&eng->arena_ctr, 1)) return -1;
        void* a = nullptr;
        HIPCHK(hipHostMalloc(&a, cap + 256, hipHostMallocCoherent | hipHostMallocMapped));
        memset(a, 0, 256);
        eng->arena = a;
        eng->arena_bytes = cap;
        eng->arena_seq = 0;
    }
    *out = (char*)eng->arena + 256;   // the first 256 bytes hold the completion word
    return 0;
}

int mdl_host_wait(MdlEngine* eng, void* stream) {
    if (!eng) return fail("mdl_host_wait: null engine");
    if (!eng->arena) return fail("mdl_host_wait: call mdl_host_arena first");
    if (host_io_ok(eng, "mdl_host_wait")) return -1;
    DeviceGuard dg(eng->device);
    hipStream_t s = (hipStream_t)stream;
    int32_t* seq = (int32_t*)eng->arena;
    const int32_t want = eng->arena_seq = (eng->arena_seq % 0x7ffffff0) + 1;
    HIPCHK(mdl::launch_publish(seq, want, s));
    return spin_wait(eng, seq, want, s, "mdl_host_wait");
}

int mdl_mail_export(MdlEngine* eng, int32_t n, int32_t use_ids, void* stream) {
    if (!eng) return fail("mdl_mail_export: null engine");
    if (mail_check_ids(eng, n, use_ids, "mdl_mail_export")) return -1;
    if (host_io_ok(eng, "mdl_mail_export")) return -1;
    if (n == 0) return 0;
    DeviceGuard dg(eng->device);
    return mail_finish(eng, n, use_ids, (hipStream_t)stream, "mdl_mail_export");
}

// ---- greedy baseline ----
namespace {
// BFS tables per map and the per-env agent records, made on first use (or by a checkpoint load)
int greedy_alloc(MdlEngine* eng, hipStream_t s) {
    if (eng->gtab) return 0;
    mdl::GreedyLayout& g = eng->glay;
    g.A = eng->p.A;
    g.cap = 3 * eng->p.P + 64;
    g.list_off = (8 + 4 * g.A + 3) & ~3;
    g.free_off = g.list_off + 2 * g.cap;
    g.stride = eng->greedy_stride();
    g.lds_stride = (3 * g.cap + 15) & ~15;
    if (4 * (size_t)g.lds_stride > LDS_BUDGET) return fail("mdl_greedy_init: too many packages for the greedy agent");
    int64_t tab = 0;
    for (int m = 0; m < eng->p.n_maps; m++) {
        const int64_t hw = (int64_t)eng->mapH[m] * eng->mapW[m];
        if (hw > 4096) return fail("mdl_greedy_init: map %d has %lld cells (the BFS tables need <= 4096)", m,
                                   (long long)hw);
        g.tab_off[m] = tab;
        tab += hw * hw;
    }
    if (eng->alloc(&eng->gtab, (size_t)tab) || eng->alloc(&eng->gstate, (size_t)eng->p.E * g.stride)) return -1;
    for (int m = 0; m < eng->p.n_maps; m++)
        HIPCHK(mdl::launch_bfs_table(eng->p.grids + eng->p.maps[m].grid_off, eng->mapH[m], eng->mapW[m],
                                     eng->gtab + g.tab_off[m], s));
    return 0;
}
}  // namespace

int mdl_greedy_init(MdlEngine* eng, const int32_t* env_ids, int32_t n, void* stream) {
    if (!eng) return fail("mdl_greedy_init: null engine");
    if (!eng->seeded) return fail("mdl_greedy_init: engine not seeded");
    if (!env_ids) n = eng->p.E;
    if (n < 0 || n > eng->p.E) return fail("mdl_greedy_init: n=%d out of range", n);
    DeviceGuard dg(eng->device);
    hipStream_t s = (hipStream_t)stream;
    if (greedy_alloc(eng, s)) return -1;
    if (n == 0) return 0;
    HIPCHK(mdl::launch_greedy_init(eng->p, eng->glay, eng->gstate, env_ids, n, s));
    // every env re-initialised only without an id list: a device id list is not read back, and one
    // of length E may repeat ids or hold ids the kernel skips
    if (!env_ids) eng->greedy_stale = false;
    return 0;
}

int mdl_greedy_actions(MdlEngine* eng, const int32_t* env_ids, int32_t n, uint8_t* actions, void* stream) {
    if (!eng || !actions) return fail("mdl_greedy_actions: null argument");
    if (!eng->gstate) return fail("mdl_greedy_actions: call mdl_greedy_init first");
    if (eng->greedy_stale)
        return fail("mdl_greedy_actions: the greedy agents' state predates mdl_load_state of a checkpoint without "
                    "it; call mdl_greedy_init without an id list");
    if (!env_ids) n = eng->p.E;
    if (n < 0 || n > eng->p.E) return fail("mdl_greedy_actions: n=%d out of range", n);
    if (n == 0) return 0;
    DeviceGuard dg(eng->device);
    HIPCHK(mdl::launch_greedy_act(eng->p, eng->glay, eng->gstate, eng->gtab, env_ids, n, actions,
                                  (hipStream_t)stream));
    return 0;
}

// ---- checkpoint ----
namespace {
constexpr uint32_t CKPT_VERSION = 2;
constexpr uint32_t CKPT_GREEDY = 1u;  // flags: the greedy agents' records follow the env state
struct CkptHeader {
    char magic[8];  // "MDLSTATE"
    uint32_t version, tracker_mode;
    int32_t E, A, P, T, n_maps, seeded;
    uint64_t map_fp, payload_bytes;
    uint64_t cfg_fp;  // reward / shaping constants, observation dims
    uint32_t flags, reserved;
};
static_assert(sizeof(CkptHeader) == 72, "checkpoint header layout");

size_t payload(const MdlEngine* eng, bool with_greedy) {
    size_t n = 0;
    for (auto& s : eng->state_sections(with_greedy)) n += s.second;
    return n;
}
}  // namespace

int mdl_state_bytes(MdlEngine* eng, int64_t* bytes) {
    if (!eng || !bytes) return fail("mdl_state_bytes: null argument");
    *bytes = (int64_t)(sizeof(CkptHeader) + payload(eng, eng->has_greedy()));
    return 0;
}

int mdl_save_state(MdlEngine* eng, void* buf, int64_t bytes, void* stream) {
    int64_t need = 0;
    if (mdl_state_bytes(eng, &need)) return -1;
    if (!buf || bytes < need) return fail("mdl_save_state: buffer of %lld bytes, need %lld", (long long)bytes,
                                          (long long)need);
    DeviceGuard dg(eng->device);
    hipStream_t s = (hipStream_t)stream;
    const bool g = eng->has_greedy();
    CkptHeader h{};
    memcpy(h.magic, "MDLSTATE", 8);
    h.version = CKPT_VERSION;
    h.tracker_mode = (uint32_t)eng->cfg.tracker_mode;
    h.E = eng->p.E; h.A = eng->p.A; h.P = eng->p.P; h.T = eng->p.T;
    h.n_maps = eng->p.n_maps;
    h.seeded = eng->seeded ? 1 : 0;
    h.map_fp = eng->map_fp;
    h.cfg_fp = eng->cfg_fp;
    h.flags = g ? CKPT_GREEDY : 0u;
    h.payload_bytes = (uint64_t)payload(eng, g);
    memcpy(buf, &h, sizeof h);
    char* o = (char*)buf + sizeof h;
    for (auto& sec : eng->state_sections(g)) {
        if (sec.second) HIPCHK(hipMemcpyAsync(o, sec.first, sec.second, hipMemcpyDeviceToHost, s));
        o += sec.second;
    }
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

int mdl_load_state(MdlEngine* eng, const void* buf, int64_t bytes, void* stream) {
    if (!eng) return fail("mdl_load_state: null engine");
    if (!buf || bytes < (int64_t)sizeof(CkptHeader)) return fail("mdl_load_state: truncated checkpoint");
    CkptHeader h;
    memcpy(&h, buf, sizeof h);
    if (memcmp(h.magic, "MDLSTATE", 8) != 0) return fail("mdl_load_state: not an engine checkpoint");
    if (h.version != CKPT_VERSION)
        return fail("mdl_load_state: checkpoint version %u, this engine reads version %u", h.version, CKPT_VERSION);
    if (h.E != eng->p.E || h.A != eng->p.A || h.P != eng->p.P || h.T != eng->p.T ||
        h.tracker_mode != (uint32_t)eng->cfg.tracker_mode || h.n_maps != eng->p.n_maps || h.map_fp != eng->map_fp)
        return fail("mdl_load_state: checkpoint of a different configuration (E=%d A=%d P=%d T=%d, maps %llx)", h.E, h.A,
                    h.P, h.T, (unsigned long long)h.map_fp);
    if (h.cfg_fp != eng->cfg_fp)
        return fail("mdl_load_state: checkpoint of an engine with other reward / shaping constants or observation "
                    "dimensions");
    if (h.flags & ~CKPT_GREEDY) return fail("mdl_load_state: unknown checkpoint flags %#x", h.flags);
    const bool g = (h.flags & CKPT_GREEDY) != 0;
    const int64_t need = (int64_t)(sizeof h + payload(eng, g));
    if (bytes < need || h.payload_bytes != (uint64_t)(need - (int64_t)sizeof h))
        return fail("mdl_load_state: checkpoint of %lld bytes, need %lld", (long long)bytes, (long long)need);
    DeviceGuard dg(eng->device);
    hipStream_t s = (hipStream_t)stream;
    if (g && greedy_alloc(eng, s)) return -1;
    const char* in = (const char*)buf + sizeof h;
    for (auto& sec : eng->state_sections(g)) {
        if (sec.second) HIPCHK(hipMemcpyAsync(sec.first, in, sec.second, hipMemcpyHostToDevice, s));
        in += sec.second;
    }
    HIPCHK(hipStreamSynchronize(s));
    eng->seeded = h.seeded != 0;
    // greedy records not in the checkpoint describe the engine's pre-load episodes: refuse them
    eng->greedy_stale = !g && eng->gstate != nullptr;
    if (g) eng->greedy_stale = false;
    return 0;
}

int mdl_build_obs(MdlEngine* eng, int32_t env_begin, int32_t n, float* actor_map, float* actor_vec,
                  float* critic_map, float* critic_vec, void* stream) {
    if (!eng) return fail("mdl_build_obs: null engine");
    if (env_begin < 0 || n < 0 || env_begin + n > eng->p.E) return fail("mdl_build_obs: env range out of bounds");
    if (n == 0) return 0;
    if (eng->shape_run_end[env_begin] < env_begin + n)
        return fail("mdl_build_obs: envs [%d, %d) mix map shapes (same-shape run ends at %d)", env_begin,
                    env_begin + n, eng->shape_run_end[env_begin]);
    DeviceGuard dg(eng->device);
    HIPCHK(eng->launch_obs(env_begin, n, actor_map, actor_vec, critic_map, critic_vec, (hipStream_t)stream));
    return 0;
}

int mdl_read_state(MdlEngine* eng, int32_t* robots, int32_t* pkgs, int32_t* t, double* total_reward,
                   int32_t* tracker, int32_t* tracker_data, void* stream) {
    if (!eng) return fail("mdl_read_state: null engine");
    DeviceGuard dg(eng->device);
    HIPCHK(mdl::launch_export(eng->p, robots, pkgs, t, total_reward, tracker, tracker_data, (hipStream_t)stream));
    return 0;
}

namespace {
// Helper calls that finish themselves (mdl_host_views_*): the launch's own waves publish the
// arena's completion word, the host spins on it -- one launch, no k_publish behind it.
struct HostCall {
    MdlEngine* eng;
    bool on;
    mdl::Publish pb;
    unsigned waves = 0;
    HostCall(MdlEngine* e, bool publish) : eng(e), on(publish) {}
    // the Publish of a launch of `launch_waves` waves
    // (a one-wave launch publishes without the counter)
    const mdl::Publish& arm(unsigned launch_waves) {
        if (on) {
            waves = launch_waves > 1 ? launch_waves : 0;
            pb = mdl::Publish{(int32_t*)eng->arena, launch_waves > 1 ? eng->arena_ctr : nullptr, eng->arena_waves,
                              (eng->arena_seq % 0x7ffffff0) + 1};
        }
        return pb;
    }
    // after a successful launch: account for its waves, then wait for its word
    int finish(hipStream_t s, const char* who) {
        if (!on) return 0;
        eng->arena_seq = pb.value;
        eng->arena_waves += waves;
        return spin_wait(eng, pb.seq, pb.value, s, who);
    }
};

int views_features(MdlEngine* eng, const int32_t* views, const int64_t* offsets, int32_t n_views, int32_t max_slots,
                   const int32_t* agent_idx, int32_t T, int32_t MO, int32_t MP, int32_t MR, int32_t MPs, float* obs,
                   float* vec, float* gmap, float* gvec, void* stream, bool host, const char* who) {
    if (!eng || !views || !offsets) return fail("%s: null argument", who);
    if (host && !eng->arena) return fail("%s: call mdl_host_arena first", who);
    if (host && host_io_ok(eng, who)) return -1;
    if (n_views < 0 || max_slots < 0 || max_slots > 4096) return fail("%s: bad sizes", who);
    if (MO < 0 || MP < 0 || MR < 0 || MPs < 0) return fail("%s: negative slot count", who);
    if (n_views == 0) return 0;
    const int MPc = std::min(MP, max_slots), MPsc = std::min(MPs, max_slots);
    const size_t lds = mdl::views_lds(max_slots, eng->maxHW, MO, MPc, MR, MPsc);
    const int wpb = waves_per_block(lds);
    if (wpb < 1) return fail("%s: needs %zu bytes of LDS per view", who, lds);
    DeviceGuard dg(eng->device);
    HostCall hc(eng, host);
    const hipStream_t s = (hipStream_t)stream;
    HIPCHK(mdl::launch_views_features(eng->p, views, offsets, n_views, agent_idx, T, MO, MP, MR, MPs, MPc, MPsc,
                                      max_slots, eng->maxHW, obs, vec, gmap, gvec, wpb, lds, s, hc.arm(mdl::grid_waves(n_views, wpb))));
    return hc.finish(s, who);
}

int views_shaped(MdlEngine* eng, const int32_t* prev_views, const int64_t* prev_offsets, int32_t max_slots,
                 const int32_t* cur, const int64_t* cur_offsets, const uint8_t* actions, const int64_t* act_offsets,
                 const double* g, int32_t n, const double* consts, float* out, void* stream, bool host,
                 const char* who) {
    if (!eng || !prev_views || !prev_offsets || !cur || !cur_offsets || !actions || !act_offsets || !g || !out)
        return fail("%s: null argument", who);
    if (host && !eng->arena) return fail("%s: call mdl_host_arena first", who);
    if (host && host_io_ok(eng, who)) return -1;
    if (n < 0 || max_slots < 0 || max_slots > 4096) return fail("%s: bad sizes", who);
    if (n == 0) return 0;
    mdl::ShapingConsts C;
    for (int i = 0; i < 9; i++) C.c[i] = consts ? (float)consts[i] : eng->p.shaping[i];
    const size_t lds = mdl::views_shaped_lds(max_slots);
    const int wpb = waves_per_block(lds);
    DeviceGuard dg(eng->device);
    HostCall hc(eng, host);
    const hipStream_t s = (hipStream_t)stream;
    HIPCHK(mdl::launch_views_shaped(eng->p, prev_views, prev_offsets, cur, cur_offsets, actions, act_offsets, g, n, C,
                                    out, wpb, lds, max_slots, s, hc.arm(mdl::grid_waves(n, wpb))));
    return hc.finish(s, who);
}
}  // namespace

static_assert(mdl::VIEW_INLINE_WORDS == MDL_VIEW_INLINE_WORDS, "inline view capacity of the header and kernels");

int mdl_host_view_features(MdlEngine* eng, const int32_t* rec, int32_t words, int32_t agent_index, int32_t T,
                           int32_t MO, int32_t MP, int32_t MR, int32_t MPs, float* obs, float* vec, float* gmap,
                           float* gvec, void* stream) {
    const char* who = "mdl_host_view_features";
    if (!eng || !rec) return fail("%s: null argument", who);
    if (!eng->arena) return fail("%s: call mdl_host_arena first", who);
    if (host_io_ok(eng, who)) return -1;
    if (words < 4 || words > MDL_VIEW_INLINE_WORDS)
        return fail("%s: a record of %d words (inline records hold 4..%d)", who, words, MDL_VIEW_INLINE_WORDS);
    const int A = rec[1], ns = rec[2], map = rec[3];
    if (A < 0 || A > MDL_MAX_ROBOTS || ns < 0 || 4 + 3 * A + 8 * ns > words)
        return fail("%s: a record of %d words cannot hold %d robots and %d slots", who, words, A, ns);
    if (map < 0 || map >= eng->p.n_maps) return fail("%s: map index %d out of range", who, map);
    if (MO < 0 || MP < 0 || MR < 0 || MPs < 0) return fail("%s: negative slot count", who);
    const int MPc = std::min(MP, ns), MPsc = std::min(MPs, ns);
    const size_t lds = mdl::views_lds(ns, eng->maxHW, MO, MPc, MR, MPsc);
    if (waves_per_block(lds) < 1) return fail("%s: needs %zu bytes of LDS", who, lds);
    DeviceGuard dg(eng->device);
    HostCall hc(eng, true);
    const hipStream_t s = (hipStream_t)stream;
    HIPCHK(mdl::launch_view_features_inline(eng->p, rec, words, agent_index, T, MO, MP, MR, MPs, MPc, MPsc, ns,
                                            eng->maxHW, obs, vec, gmap, gvec, lds, s, hc.arm(1)));
    return hc.finish(s, who);
}

int mdl_host_view_shaped_reward(MdlEngine* eng, const int32_t* prev_view, int32_t prev_words, const int32_t* cur,
                                int32_t cur_words, const uint8_t* actions, int32_t n_actions, double g,
                                const double* consts, float* out, void* stream) {
    const char* who = "mdl_host_view_shaped_reward";
    if (!eng || !prev_view || !cur || (!actions && n_actions > 0) || !out) return fail("%s: null argument", who);
    if (!eng->arena) return fail("%s: call mdl_host_arena first", who);
    if (host_io_ok(eng, who)) return -1;
    if (prev_words < 4 || cur_words < 2 || n_actions < 0) return fail("%s: bad sizes", who);
    const int A = prev_view[1], ns = prev_view[2];
    if (A < 0 || A > MDL_MAX_ROBOTS || ns < 0 || 4 + 3 * A + 8 * ns > prev_words)
        return fail("%s: a record of %d words cannot hold %d robots and %d slots", who, prev_words, A, ns);
    if (cur[1] < A || 2 + 3 * A > cur_words || n_actions < A)
        return fail("%s: %d robots before the step, but %d after and %d actions", who, A, cur[1], n_actions);
    const int co = prev_words, ao = co + cur_words, words = ao + (n_actions + 3) / 4;
    if (words > MDL_VIEW_INLINE_WORDS)
        return fail("%s: %d words of inputs (inline records hold %d)", who, words, MDL_VIEW_INLINE_WORDS);
    int32_t buf[MDL_VIEW_INLINE_WORDS];
    memcpy(buf, prev_view, 4 * (size_t)prev_words);
    memcpy(buf + co, cur, 4 * (size_t)cur_words);
    buf[words - 1] = 0;
    memcpy(buf + ao, actions, (size_t)n_actions);
    mdl::ShapingConsts C;
    for (int i = 0; i < 9; i++) C.c[i] = consts ? (float)consts[i] : eng->p.shaping[i];
    const size_t lds = mdl::views_shaped_lds(ns);
    DeviceGuard dg(eng->device);
    HostCall hc(eng, true);
    const hipStream_t s = (hipStream_t)stream;
    HIPCHK(mdl::launch_view_shaped_inline(buf, words, co, ao, g, C, ns, lds, s, hc.arm(1)));
    if (hc.finish(s, who)) return -1;
    memcpy(out, (const int32_t*)eng->arena + 1, 4);   // the result, published beside the completion word
    return 0;
}

int mdl_views_features(MdlEngine* eng, const int32_t* views, const int64_t* offsets, int32_t n_views,
                       int32_t max_slots, const int32_t* agent_idx, int32_t T, int32_t MO, int32_t MP, int32_t MR,
                       int32_t MPs, float* obs, float* vec, float* gmap, float* gvec, void* stream) {
    return views_features(eng, views, offsets, n_views, max_slots, agent_idx, T, MO, MP, MR, MPs, obs, vec, gmap,
                          gvec, stream, false, "mdl_views_features");
}

int mdl_host_views_features(MdlEngine* eng, const int32_t* views, const int64_t* offsets, int32_t n_views,
                            int32_t max_slots, const int32_t* agent_idx, int32_t T, int32_t MO, int32_t MP,
                            int32_t MR, int32_t MPs, float* obs, float* vec, float* gmap, float* gvec, void* stream) {
    return views_features(eng, views, offsets, n_views, max_slots, agent_idx, T, MO, MP, MR, MPs, obs, vec, gmap,
                          gvec, stream, true, "mdl_host_views_features");
}

int mdl_views_shaped_reward(MdlEngine* eng, const int32_t* prev_views, const int64_t* prev_offsets,
                            int32_t max_slots, const int32_t* cur, const int64_t* cur_offsets, const uint8_t* actions,
                            const int64_t* act_offsets, const double* g, int32_t n, const double* consts, float* out,
                            void* stream) {
    return views_shaped(eng, prev_views, prev_offsets, max_slots, cur, cur_offsets, actions, act_offsets, g, n, consts,
                        out, stream, false, "mdl_views_shaped_reward");
}

int mdl_host_views_shaped_reward(MdlEngine* eng, const int32_t* prev_views, const int64_t* prev_offsets,
                                 int32_t max_slots, const int32_t* cur, const int64_t* cur_offsets,
                                 const uint8_t* actions, const int64_t* act_offsets, const double* g, int32_t n,
                                 const double* consts, float* out, void* stream) {
    return views_shaped(eng, prev_views, prev_offsets, max_slots, cur, cur_offsets, actions, act_offsets, g, n, consts,
                        out, stream, true, "mdl_host_views_shaped_reward");
}

// ---- IDQ / qmix featurizers and IDQ reward shaping ----
int mdl_build_obs_alt(MdlEngine* eng, int32_t env_begin, int32_t n, float* idq_obs, float* qmix_state, int32_t out_h,
                      int32_t out_w, void* stream) {
    if (!eng) return fail("mdl_build_obs_alt: null engine");
    if (env_begin < 0 || n < 0 || env_begin + n > eng->p.E) return fail("mdl_build_obs_alt: env range out of bounds");
    if (qmix_state && (out_h < 1 || out_w < 1 || out_h > 4096 || out_w > 4096))
        return fail("mdl_build_obs_alt: bad state tensor shape (%d, %d)", out_h, out_w);
    if (n == 0) return 0;
    if (eng->shape_run_end[env_begin] < env_begin + n)
        return fail("mdl_build_obs_alt: envs [%d, %d) mix map shapes (same-shape run ends at %d)", env_begin,
                    env_begin + n, eng->shape_run_end[env_begin]);
    const size_t lds = mdl::alt_obs_lds(eng->p.P, eng->maxHW);
    const int wpb = waves_per_block(lds);
    if (wpb < 1) return fail("mdl_build_obs_alt: needs %zu bytes of LDS per env", lds);
    DeviceGuard dg(eng->device);
    HIPCHK(mdl::launch_alt_obs(eng->p, env_begin, n, idq_obs, qmix_state, out_h, out_w, wpb, lds,
                               (hipStream_t)stream));
    return 0;
}

int mdl_views_alt_features(MdlEngine* eng, const int32_t* views, const int64_t* offsets, int32_t n_views,
                           int32_t max_slots, const int32_t* agent_idx, float* idq_obs, float* qmix_state,
                           int32_t out_h, int32_t out_w, void* stream) {
    if (!eng || !views || !offsets) return fail("mdl_views_alt_features: null argument");
    if (n_views < 0 || max_slots < 0 || max_slots > 4096) return fail("mdl_views_alt_features: bad sizes");
    if (qmix_state && (out_h < 1 || out_w < 1 || out_h > 4096 || out_w > 4096))
        return fail("mdl_views_alt_features: bad state tensor shape (%d, %d)", out_h, out_w);
    if (n_views == 0) return 0;
    const size_t lds = mdl::views_alt_lds(max_slots, eng->maxHW);
    const int wpb = waves_per_block(lds);
    if (wpb < 1) return fail("mdl_views_alt_features: needs %zu bytes of LDS per view", lds);
    DeviceGuard dg(eng->device);
    HIPCHK(mdl::launch_views_alt(eng->p, views, offsets, n_views, agent_idx, idq_obs, qmix_state, out_h, out_w, wpb,
                                 lds, max_slots, (hipStream_t)stream));
    return 0;
}

int mdl_views_idq_reward(MdlEngine* eng, const int32_t* prev_views, const int64_t* prev_offsets, int32_t max_slots,
                         const int32_t* cur, const int64_t* cur_offsets, const uint8_t* ops, const int64_t* op_offsets,
                         int32_t ops_are_ints, int32_t n, double* out, void* stream) {
    if (!eng || !prev_views || !prev_offsets || !cur || !cur_offsets || !ops || !op_offsets || !out)
        return fail("mdl_views_idq_reward: null argument");
    if (n < 0 || max_slots < 0 || max_slots > 4096) return fail("mdl_views_idq_reward: bad sizes");
    if (n == 0) return 0;
    const size_t lds = mdl::views_shaped_lds(max_slots);
    const int wpb = waves_per_block(lds);
    DeviceGuard dg(eng->device);
    HIPCHK(mdl::launch_views_idq_reward(prev_views, prev_offsets, cur, cur_offsets, ops, op_offsets, ops_are_ints, n,
                                        out, wpb, lds, max_slots, (hipStream_t)stream));
    return 0;
}

int mdl_rank_table(int32_t H, int32_t W, uint16_t* out) {
    if (!out || H < 1 || W < 1 || H > 255 || W > 255) return fail("mdl_rank_table: bad arguments");
    std::vector<uint16_t> rk;
    build_rank(H, W, rk);
    std::memcpy(out, rk.data(), rk.size() * sizeof(uint16_t));
    return 0;
}

int mdl_get_config(const MdlEngine* eng, MdlConfig* out) {
    if (!eng || !out) return fail("mdl_get_config: null argument");
    *out = eng->cfg;
    return 0;
}

int mdl_step_layout(const MdlEngine* eng, int32_t n, int32_t use_ids, int32_t* layout) {
    if (!eng || !layout) return fail("mdl_step_layout: null argument");
    if (n < 0 || n > eng->p.E) return fail("mdl_step_layout: n=%d out of range", n);
    *layout = eng->layout_for(use_ids ? n : eng->p.E, use_ids != 0);
    return 0;
}

int mdl_step_kernel_name(const MdlEngine* eng, int32_t layout, int32_t with_obs, char* out, int32_t cap) {
    if (!eng || !out || cap < 1) return fail("mdl_step_kernel_name: bad argument");
    if (layout != MDL_STEP_LAYOUT_WAVE && layout != MDL_STEP_LAYOUT_ROWS && layout != MDL_STEP_LAYOUT_HALVES)
        return fail("mdl_step_kernel_name: layout %d is not WAVE, ROWS or HALVES", layout);
    if ((layout == MDL_STEP_LAYOUT_ROWS && (with_obs || !eng->step_rows)) ||
        (layout == MDL_STEP_LAYOUT_HALVES && (with_obs || !eng->step_halves)))
        return fail("mdl_step_kernel_name: no launch in layout %d in this configuration", layout);
    // mdl_step_obs's one-launch form (else it is mdl_step's wave kernel + the builder)
    const bool obs = with_obs && eng->p.obs_small && eng->p.A <= 8 && eng->p.P <= 64 &&
                     std::max(eng->lds_step, eng->lds_obs) <= LDS_BUDGET;
    const int epw = layout == MDL_STEP_LAYOUT_ROWS ? 4 : layout == MDL_STEP_LAYOUT_HALVES ? 2 : 1;
    const int k = mdl::step_kernel_name(eng->p, epw, obs, out, cap);
    if (k < 0 || k >= cap) return fail("mdl_step_kernel_name: buffer of %d bytes too small", cap);
    return 0;
}

int mdl_last_step_layout(const MdlEngine* eng, int32_t* layout) {
    if (!eng || !layout) return fail("mdl_last_step_layout: null argument");
    *layout = eng->last_step_layout;
    return 0;
}

int mdl_obs_dims(const MdlEngine* eng, int32_t* actor_vec_dim, int32_t* critic_vec_dim) {
    if (!eng) return fail("mdl_obs_dims: null engine");
    if (actor_vec_dim) *actor_vec_dim = 6 + 5 * eng->p.MO + 5 * eng->p.MP + 1;
    if (critic_vec_dim) *critic_vec_dim = 6 * eng->p.MR + 7 * eng->p.MPs + 1;
    return 0;
}

}  // extern "C"
