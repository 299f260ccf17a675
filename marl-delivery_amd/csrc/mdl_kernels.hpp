// mdl_kernels.hpp -- host-visible launchers of the gfx950 kernels (mdl_kernels.hip).
#pragma once
#include "mdl_device.hpp"

namespace mdl {

// sets the thread-local message mdl_last_error() returns (mdl_engine.hip)
void set_error(const char* msg);

struct ShapingConsts {
    float c[9];
};

hipError_t launch_seed(const DevParams& p, const uint32_t* seeds, int wpb, size_t lds, hipStream_t s);
hipError_t launch_reset(const DevParams& p, const int* ids, int n, int wpb, size_t lds, hipStream_t s);
hipError_t launch_tracker_clear(const DevParams& p, const int* ids, int n, hipStream_t s);
hipError_t launch_step(const DevParams& p, const uint8_t* actions, int fmt, const int* ids, int n, int auto_reset,
                       double* r, float* sh, uint8_t* done, int wpb, size_t lds, hipStream_t s);
// k_step_rows (mdl_step_rows.hpp): a full-batch step with four envs per wavefront, one per 16-lane
// row; A <= 8, P <= 64 (step_rows_ok).  lds: the per-wave slice (step_rows_lds).
bool step_rows_ok(int A, int P);
// The symbol (as rocprof names it) of the step kernel a launch takes: launch_step_rows
// (envs_per_wave 4), launch_step_halves (2), launch_step_obs (obs: the fused step + observation
// kernel) or launch_step (1).  Mirrors their dispatch; bench.py labels its roofline record with it.
// Returns snprintf's count.
int step_kernel_name(const DevParams& p, int envs_per_wave, bool obs, char* out, int cap);
size_t step_rows_lds(int P);
// k_step_halves (mdl_step_halves.hpp): a full-batch step with two envs per wavefront, one per 32-lane
// half; A == 16, P <= 128 (step_halves_ok).  lds: the per-wave slice (step_halves_lds).
bool step_halves_ok(int A, int P);
size_t step_halves_lds(int P);
hipError_t launch_step_halves(const DevParams& p, const uint8_t* actions, int fmt, int n, int auto_reset, double* r,
                              float* sh, uint8_t* done, int wpb, size_t lds, hipStream_t s);
hipError_t launch_step_rows(const DevParams& p, const uint8_t* actions, int fmt, int n, int auto_reset, double* r,
                            float* sh, uint8_t* done, int wpb, size_t lds, hipStream_t s);
// the step's launch shape (grid, workgroup, LDS, kernel arguments) with an empty kernel; rows: the
// grid of the layout's envs per wave (1: k_step, 2: k_step_halves, 4: k_step_rows)
hipError_t launch_step_floor(const DevParams& p, int n, int wpb, size_t lds, hipStream_t s, int envs_per_wave = 1);
hipError_t launch_step_fused(const DevParams& p, const uint8_t* actions, int fmt, const int* ids, int n, int K,
                             int auto_reset, double* r, float* sh, uint8_t* done, int wpb, size_t lds,
                             hipStream_t s);
hipError_t launch_step_obs(const DevParams& p, const uint8_t* actions, int fmt, int n, int auto_reset, double* r,
                           float* sh, uint8_t* done, float* amap, float* avec, float* cmap, float* cvec, int wpb,
                           size_t lds, hipStream_t s);
// rank_lds > 0 (small builder): bytes of LDS in front of the per-wave slices holding the launch's
// distance-rank table (mdl_obs_small.hpp k_obs_small).  PRECONDITION: envs [env_begin, env_begin+n)
// share one map shape -- the table copied is env_begin's map's.  The engine checks it
// (MdlEngine::launch_obs, mdl_engine.hip) before every call.
hipError_t launch_obs(const DevParams& p, int env_begin, int n, float* amap, float* avec, float* cmap, float* cvec,
                      int wpb, size_t lds, hipStream_t s, int rank_lds = 0);
// A launch's own completion word (host-mapped): every wave of its grid counts itself in the
// running device counter `ctr` (never reset: `base` is its value before the launch) after a
// system-scope release of its stores; the last one writes `value` to `seq`.  seq == nullptr: none;
// ctr == nullptr: a one-wave launch, which writes `value` straight after its release.
struct Publish {
    int32_t* seq = nullptr;
    unsigned* ctr = nullptr;
    unsigned base = 0;
    int32_t value = 0;
    unsigned expect = 0;   // > 0: the number of waves that count themselves (not the whole grid)
};
// A view record carried in the kernel arguments (mdl_host_view_*): two capacity classes, the larger
// sized so the kernel's whole argument block stays well inside the 4 KiB kernarg limit.
constexpr int VIEW_INLINE_SMALL = 256, VIEW_INLINE_WORDS = 768;
template <int CAP>
struct ViewInline {
    int32_t w[CAP];
};
hipError_t launch_view_features_inline(const DevParams& p, const int32_t* rec, int words, int a, int T, int MO,
                                      int MP, int MR, int MPs, int MPc, int MPsc, int NSmax, int HW, float* obs,
                                      float* vec, float* gmap, float* gvec, size_t lds, hipStream_t s,
                                      const Publish& pb);
// the result comes back in the completion word's second half (pb.seq 8-byte aligned)
hipError_t launch_view_shaped_inline(const int32_t* rec, int words, int co, int ao, double g, const ShapingConsts& C,
                                     int NSmax, size_t lds, hipStream_t s, const Publish& pb);
unsigned grid_waves(int n, int wpb);   // waves of a 256-thread-block launch of wpb views per block
hipError_t launch_views_features(const DevParams& p, const int32_t* views, const int64_t* offs, int n,
                                 const int32_t* agent_idx, int T, int MO, int MP, int MR, int MPs, int MPc, int MPsc,
                                 int NSmax, int HW, float* obs, float* vec, float* gmap, float* gvec, int wpb,
                                 size_t lds, hipStream_t s, const Publish& pb = Publish{});
hipError_t launch_views_shaped(const DevParams& p, const int32_t* prev, const int64_t* prev_offs, const int32_t* cur,
                               const int64_t* cur_offs, const uint8_t* acts, const int64_t* act_offs, const double* g,
                               int n, const ShapingConsts& C, float* out, int wpb, size_t lds, int NSmax,
                               hipStream_t s, const Publish& pb = Publish{});
// the dict-API mailbox's output rows (host-mapped memory; row w = the w-th env of a call)
struct MailRows {
    int32_t* seq;      // completion word, written last
    int32_t* robots;   // [E][A][3]
    int32_t* pkgs;     // [E][P][8]
    int32_t* t;        // [E]
    double* total;     // [E]
    int32_t* rterms;   // [E] RT_* bits
};
hipError_t launch_publish(int32_t* seq, int32_t value, hipStream_t s);
// mdl_mail_step in one launch: the step (action codes, rows [0, n) = envs ids[w] or w), its rows
// into the mailbox, the completion word `seq` once all n waves have counted themselves in `ctr`
hipError_t launch_step_mail(const DevParams& p, const uint8_t* codes, const int* ids, int n, int auto_reset, double* r,
                            float* sh, uint8_t* done, int wpb, size_t lds, const MailRows& m, unsigned* ctr,
                            unsigned base, int32_t seq, hipStream_t s);
unsigned mail_export_waves(int n);   // waves of one k_mail_export launch over n envs
hipError_t launch_mail_export(const DevParams& p, const int32_t* ids, int n, const MailRows& m, unsigned* ctr,
                              unsigned base, int32_t seq, hipStream_t s);
hipError_t launch_export(const DevParams& p, int32_t* robots, int32_t* pkgs, int32_t* t, double* total,
                         int32_t* tracker, int32_t* tracker_data, hipStream_t s);

// Greedy agent record layout (mdl_greedy.hip): per env `stride` bytes.
struct GreedyLayout {
    int A, cap, stride, list_off, free_off, lds_stride;
    int64_t tab_off[MAX_MAPS];  // BFS table of map m: tables + tab_off[m], [HW goal][HW cell] u16
};
hipError_t launch_bfs_table(const uint8_t* grid, int H, int W, uint16_t* table, hipStream_t s);
hipError_t launch_greedy_init(const DevParams& p, const GreedyLayout& g, unsigned char* gs, const int* ids, int n,
                              hipStream_t s);
hipError_t launch_greedy_act(const DevParams& p, const GreedyLayout& g, unsigned char* gs, const uint16_t* tables,
                             const int* ids, int n, uint8_t* actions, hipStream_t s);

hipError_t launch_alt_obs(const DevParams& p, int env_begin, int n, float* idq, float* qst, int oh, int ow, int wpb,
                          size_t lds, hipStream_t s);
hipError_t launch_views_alt(const DevParams& p, const int32_t* views, const int64_t* offs, int n,
                            const int32_t* agent_idx, float* idq, float* qst, int oh, int ow, int wpb, size_t lds,
                            int NSmax, hipStream_t s);
hipError_t launch_views_idq_reward(const int32_t* prev, const int64_t* prev_offs, const int32_t* cur,
                                   const int64_t* cur_offs, const uint8_t* ops, const int64_t* op_offs,
                                   int ops_are_ints, int n, double* out, int wpb, size_t lds, int NSmax,
                                   hipStream_t s);
size_t alt_obs_lds(int P, int HW);
size_t views_alt_lds(int NSmax, int HW);

size_t step_lds(int P);
size_t obs_lds(int A, int P, int HW, int MO, int MP, int MR, int MPs);
int obs_plane_words(int A, int HW);
size_t obs_lds_small(int A, int HW, int P, int MO, int MP);
bool obs_use_small(int A, int P, int key7_dsh, int maxHW, int MO, int MP);
size_t views_lds(int NSmax, int HW, int MO, int MPc, int MR, int MPsc);
size_t views_shaped_lds(int NSmax);

}  // namespace mdl
