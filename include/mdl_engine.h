/*
 * mdl_engine.h -- C ABI of the MI355X-native marl-delivery batched step engine.
 *
 * One engine = E independent grid-world instances resident in HBM on one GPU.
 * All compute runs as gfx950 HIP kernels, one wavefront per env instance.
 * Entry points are extern "C", take plain pointers and sizes, and return an
 * int status (0 = ok, <0 = error; mdl_last_error() gives a thread-local
 * message).  No exception crosses the ABI.  Every call that takes a `stream`
 * (a hipStream_t passed as void*, NULL = default stream) is asynchronous on
 * that stream; device pointers are caller-owned unless documented otherwise.
 * One engine per device; calls on one handle are not thread-safe.
 *
 * The reference has no FFI (it is pure Python); each entry point below names
 * the Python interface it replaces (path:line under the reference tree).
 * INTEGRATION.md shows the ctypes binding a maintainer of the reference
 * would add.
 */
#ifndef MDL_ENGINE_H
#define MDL_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MDL_MAX_ROBOTS 64      /* one wavefront lane per robot */
#define MDL_MAX_PACKAGES 1024  /* Group-Project.pdf p.3 bounds G <= 1000 */
#define MDL_MAX_CELLS 16384    /* H*W <= 128*128; H, W <= 255 */

/* tracker semantics of the persistent-package dict */
#define MDL_TRACKER_FRESH 0        /* == env truth; QMIX/trainer.py:523-526 clears it on reset */
#define MDL_TRACKER_MAPPO_STALE 1  /* MAPPO/trainer.py:232-233 never clears it on auto-reset */

/* action byte formats for mdl_step */
#define MDL_ACTION_TRAINER_INT 0   /* int a: move=['D','L','R','S','U'][a%5], op=a//5 (>=3 -> 0); MAPPO/trainer.py:198-205 */
#define MDL_ACTION_CODES 1         /* move code | op code << 3; move 0..5 = S,L,R,U,D,<other string>; op 0..3 = '0','1','2',<other int> */

typedef struct MdlEngine MdlEngine;

/* Environment(...) constructor arguments (env.py:20-22) + the featurizer /
 * shaping configuration of the trainers (MAPPO/trainer.py:39-64,
 * MAPPO/helper.py:68-70,167-169,271-279, QMIX/config.yaml). */
typedef struct {
    int32_t n_envs;            /* E */
    int32_t n_robots;          /* A, 1..64 */
    int32_t n_packages;        /* P, 1..1024 */
    int32_t max_time_steps;    /* T */
    double move_cost;          /* env.py:21 defaults -0.01 */
    double delivery_reward;    /* 10.0 */
    double delay_reward;       /* 1.0 */
    int32_t tracker_mode;      /* MDL_TRACKER_* */
    double shaping[9];         /* pickup, on_time, late, closer, wasted_pick, wasted_drop, stuck, idle, away */
    int32_t obs_max_time_steps;/* T passed to the feature builders */
    int32_t max_other_robots;  /* MO  (generate_vector_features) */
    int32_t max_packages_obs;  /* MP */
    int32_t max_robots_state;  /* MR  (convert_global_state) */
    int32_t max_packages_state;/* MPs */
    int32_t obs_builder;       /* MDL_OBS_BUILDER_*: which observation kernel mdl_build_obs uses (same outputs) */
    int32_t step_layout;       /* MDL_STEP_LAYOUT_*: how mdl_step maps envs onto wavefronts (same outputs) */
} MdlConfig;

/* MdlConfig.obs_builder.  AUTO: the small builder (flat bit images, one tuple per lane) where it
 * applies (A <= 8, P <= 64, 32-bit sort keys), the general builder otherwise.  GENERIC: always the
 * general builder (any A, P).  Both produce the same floats; GENERIC exists so tests can compare
 * the two on one configuration. */
#define MDL_OBS_BUILDER_AUTO 0
#define MDL_OBS_BUILDER_GENERIC 1

/* MdlConfig.step_layout.  ROWS: a full-batch mdl_step (env_ids NULL) runs four envs per wavefront,
 * one per 16-lane row (A <= 8, P <= 64; mdl_create fails otherwise).  HALVES: two envs per
 * wavefront, one per 32-lane half (A == 16, P <= 128).  WAVE: one env per wavefront always.  AUTO:
 * ROWS where it applies and the batch has at least 7,168 envs, HALVES where it applies and the
 * batch has at least 12,288 envs (the measured crossovers on MI355X), WAVE otherwise.  Subset steps (env_ids),
 * mdl_step_fused, mdl_step_obs and the mailbox step always use one wave per env.  Every layout
 * produces the same state and outputs; the explicit layouts exist so tests can compare them on one
 * configuration. */
#define MDL_STEP_LAYOUT_AUTO 0
#define MDL_STEP_LAYOUT_WAVE 1
#define MDL_STEP_LAYOUT_ROWS 2
#define MDL_STEP_LAYOUT_HALVES 3

/* Create an engine on `device`.  grids: n_maps row-major 0/1 maps packed back
 * to back; map_hw: 2*n_maps (H, W); env_map: E map indices (NULL = all map 0).
 * Replaces Environment.__init__ / load_map (env.py:20-57) and
 * VectorizedEnv.__init__ (MAPPO/env_vectorized.py:2-11) minus seeding. */
int mdl_create(const MdlConfig* cfg, const uint8_t* grids, const int32_t* map_hw, int32_t n_maps,
               const int32_t* env_map, int32_t device, MdlEngine** out);
int mdl_destroy(MdlEngine* eng);

/* RandomState(seed) (env.py:40) for every env -- seeds: E host uint32 -- then
 * the constructor's layout draw (env.py:41).  VectorizedEnv passes seed+i
 * (MAPPO/env_vectorized.py:8-9). */
int mdl_seed(MdlEngine* eng, const uint32_t* seeds, void* stream);

/* Environment.reset() (env.py:81-125) for env_ids[0..n) (device int32; NULL =
 * all E envs, n ignored).  VectorizedEnv.reset(indices) (QMIX/env_vectorized.py:13-21).
 * In MDL_TRACKER_FRESH mode the tracker is implicitly cleared; in
 * MDL_TRACKER_MAPPO_STALE mode it is updated with the reset state, not cleared
 * (MAPPO/trainer.py:232-233); mdl_tracker_clear() clears it explicitly. */
int mdl_reset(MdlEngine* eng, const int32_t* env_ids, int32_t n, void* stream);
int mdl_tracker_clear(MdlEngine* eng, const int32_t* env_ids, int32_t n, void* stream);

/* env_ids (here and in mdl_reset / mdl_tracker_clear / mdl_step_fused / the greedy entry
 * points): a DEVICE int32 array of n ids, each processed once and in parallel, so the ids
 * must be unique and in [0, E); an id outside [0, E) is skipped by the kernels (it cannot
 * touch another env or allocation), duplicates race.  NULL = all E envs in order.  The
 * Python layer checks host-side id lists (list semantics, duplicates refused) before upload.
 *
 * One transition for env_ids[0..n) (NULL = all E in order).
 * Environment.step (env.py:173-306) + compute_shaped_rewards
 * (MAPPO/helper.py:257-369, evaluated with the pre-step tracker) + the
 * tracker update (MAPPO/trainer.py:95-130) + optional reset-on-done
 * (MAPPO/trainer.py:229-257).  actions: device uint8 [n][A] in
 * `action_format`.  Outputs (device, [n], any may be NULL): r_env = the float
 * reward env.step returns (fp64, bit-exact), r_shaped = the float32 value
 * compute_shaped_rewards returns, done = check_terminate (env.py:308-316). */
int mdl_step(MdlEngine* eng, const uint8_t* actions, int32_t action_format, const int32_t* env_ids, int32_t n,
             int32_t auto_reset, double* r_env, float* r_shaped, uint8_t* done, void* stream);

/* mdl_step for all E envs followed by mdl_build_obs(eng, 0, E, ...) of the new state --
 * the trainer's per-step sequence (MAPPO/trainer.py:229-286: env.step, reset on done,
 * tracker update, then convert_observation x A, generate_vector_features x A and
 * convert_global_state of the next state).  Same outputs as the two calls (bit-exact);
 * for A <= 8, P <= 64 they run as ONE kernel that builds the observations from the
 * state the step leaves in registers (no second launch, no state reload), otherwise
 * as the two launches.  The E envs must share one map shape; any output may be NULL. */
int mdl_step_obs(MdlEngine* eng, const uint8_t* actions, int32_t action_format, int32_t auto_reset, double* r_env,
                 float* r_shaped, uint8_t* done, float* actor_map, float* actor_vec, float* critic_map,
                 float* critic_vec, void* stream);

/* Bench mode: k_steps consecutive mdl_step calls fused
 * into one launch, each env's state held in registers between steps.  Same
 * results as k_steps mdl_step calls with actions[k] (bit-exact); actions are
 * [k_steps][n][A], r_env / r_shaped / done are [k_steps][n].  Not part of the
 * reference interface: a trainer needs the policy between steps. */
int mdl_step_fused(MdlEngine* eng, const uint8_t* actions, int32_t action_format, const int32_t* env_ids, int32_t n,
                   int32_t k_steps, int32_t auto_reset, double* r_env, float* r_shaped, uint8_t* done, void* stream);

/* Measurement aid (no reference counterpart): the launch floor of mdl_step over n envs -- one
 * launch of an EMPTY kernel with mdl_step's grid, workgroup size, LDS request and kernel-argument
 * layout (so the same preloaded argument registers and kernarg segment).  bench.py replays it the
 * way it replays mdl_step and reports the step's time above this floor.  Touches no state. */
int mdl_step_floor(MdlEngine* eng, int32_t n, void* stream);

/* ---- IDQ / qmix featurizers and IDQ reward shaping ----
 * mdl_build_obs_alt, for envs [env_begin, env_begin+n) sharing one map shape (H, W):
 *   idq_obs    f32 [n][A][6][H][W]       convert_state                IDQ/networks.py:112-217
 *                                        (qmix/networks.py:243-348 is the same function)
 *   qmix_state f32 [n][7][out_h][out_w]  convert_global_state_to_tensor qmix/networks.py:350-468
 *                                        with state_tensor_shape (7, out_h, out_w); the trainers pass (7, H, W)
 * Either pointer may be NULL.  The IDQ / qmix trainers clear their tracker per episode: build the
 * engine with MDL_TRACKER_FRESH for them.
 * mdl_views_alt_features: the same on packed dict views (as mdl_views_features).
 * mdl_views_idq_reward: reward_shaping (IDQ/networks.py:228-349) per agent, fp64, out[op_offsets[w]+a];
 * ops_are_ints = 0 reproduces IDQ/trainer.py, which passes string ops (so no op branch fires). */
int mdl_build_obs_alt(MdlEngine* eng, int32_t env_begin, int32_t n, float* idq_obs, float* qmix_state, int32_t out_h,
                      int32_t out_w, void* stream);
int mdl_views_alt_features(MdlEngine* eng, const int32_t* views, const int64_t* offsets, int32_t n_views,
                           int32_t max_slots, const int32_t* agent_idx, float* idq_obs, float* qmix_state,
                           int32_t out_h, int32_t out_w, void* stream);
int mdl_views_idq_reward(MdlEngine* eng, const int32_t* prev_views, const int64_t* prev_offsets, int32_t max_slots,
                         const int32_t* cur, const int64_t* cur_offsets, const uint8_t* ops, const int64_t* op_offsets,
                         int32_t ops_are_ints, int32_t n, double* out, void* stream);

/* ---- greedy baseline: greedyagent.py batched on the device ----
 * mdl_greedy_init = GreedyAgents() + init_agents(state) for the listed envs (call it right
 * after their reset, as evaluation.py:29-35 does); the first call also builds run_bfs's
 * distance field for every cell of every map (maps of <= 4096 cells).
 * mdl_greedy_actions = one get_actions(state) per listed env (call once per step, before
 * mdl_step), written as MDL_ACTION_CODES bytes [n][A].  Bug-compatible with the reference
 * agent (duplicated t=0 package entries, id-1 list indexing).  After mdl_load_state of a
 * checkpoint without greedy records, only a call without an id list (env_ids == NULL: every env)
 * makes mdl_greedy_actions usable again. */
int mdl_greedy_init(MdlEngine* eng, const int32_t* env_ids, int32_t n, void* stream);
int mdl_greedy_actions(MdlEngine* eng, const int32_t* env_ids, int32_t n, uint8_t* actions, void* stream);

/* ---- dict-API mailbox: the per-call path of Environment.step / reset on single envs ----
 * Environment.step (env.py:173-306) and VectorizedEnv.step / reset(indices) (QMIX/env_vectorized.py:13-37)
 * return Python dicts per call, so their cost is the host <-> GPU round trip, not the step.  The mailbox
 * is ONE engine-owned host allocation, fine-grained and mapped into the device: the caller writes action
 * codes (and env ids) into it, the step kernel reads them from there, an export kernel writes the touched
 * envs' rows and a completion word into it, and the call spins on that word (no device staging buffers,
 * no copy-engine transfers, no stream synchronisation).  Row w of every output = the w-th env of the call
 * (ids[w] with use_ids, else env w).  The pointers stay valid until mdl_destroy; the outputs of a call
 * are overwritten by the next one.  Calls are synchronous (they return once the rows are in the mailbox). */
typedef struct {
    int32_t* seq;          /* completion word (device-written) */
    uint8_t* codes;        /* in:  [E][A] MDL_ACTION_CODES bytes */
    int32_t* ids;          /* in:  [E] env ids of the call (unique, in [0, E)) */
    double* r_env;         /* out: [E] env.step's reward (fp64) */
    float* r_shaped;       /* out: [E] compute_shaped_rewards (engine tracker) */
    uint8_t* done;         /* out: [E] */
    int32_t* robots;       /* out: [E][A][3] (row, col, carrying), 0-indexed */
    int32_t* pkgs;         /* out: [E][P][8] as mdl_read_state */
    int32_t* t;            /* out: [E] */
    double* total_reward;  /* out: [E] */
    int32_t* rterms;       /* out: [E] reward terms the step added: MDL_RTERM_* bits (0 after a reset) */
} MdlMailbox;
#define MDL_RTERM_MOVE 1    /* a move cost (env.py:256) */
#define MDL_RTERM_ONTIME 2  /* an on-time delivery reward (env.py:288) */
#define MDL_RTERM_LATE 4    /* a late delivery reward (env.py:291) */
/* Allocates the mailbox on first use (E-sized sections) and returns its pointers. */
int mdl_mailbox(MdlEngine* eng, MdlMailbox* out);
/* mdl_step(codes, MDL_ACTION_CODES, ids or all E) on the mailbox's inputs, then the rows of those envs. */
int mdl_mail_step(MdlEngine* eng, int32_t n, int32_t use_ids, int32_t auto_reset, void* stream);
/* mdl_reset of those envs (Environment.reset, env.py:81-125), then their rows. */
int mdl_mail_reset(MdlEngine* eng, int32_t n, int32_t use_ids, void* stream);
/* The rows of those envs only (after other engine calls on `stream`). */
int mdl_mail_export(MdlEngine* eng, int32_t n, int32_t use_ids, void* stream);

/* Host-mapped scratch for the helper-compatible calls on single dicts (convert_observation,
 * generate_vector_features, convert_global_state, compute_shaped_rewards: MAPPO/helper.py:6-369):
 * the caller packs the view records into it and passes its addresses to mdl_views_* as both the
 * inputs and the outputs -- the kernels read and write host memory directly -- then calls
 * mdl_host_wait, which returns once everything queued on `stream` before it has finished (a
 * one-wave kernel publishes a completion word the call spins on).  mdl_host_arena returns at least
 * `bytes` of it (16-byte aligned; a larger request replaces the arena, so earlier addresses die). */
int mdl_host_arena(MdlEngine* eng, int64_t bytes, void** out);
int mdl_host_wait(MdlEngine* eng, void* stream);
/* mdl_views_features / mdl_views_shaped_reward with their inputs and outputs in the arena, and
 * synchronous: the launch's own waves publish the arena's completion word when the last of them
 * has written its outputs (no mdl_host_wait launch behind it), and the call returns once it has
 * seen it.  `stream` need not be the caller's compute stream: nothing on the device waits for or
 * on these calls.  (The helper functions of marl_gpu.helper call these from C, _mdl_pack.) */
int mdl_host_views_features(MdlEngine* eng, const int32_t* views, const int64_t* offsets, int32_t n_views,
                            int32_t max_slots, const int32_t* agent_idx, int32_t T, int32_t MO, int32_t MP,
                            int32_t MR, int32_t MPs, float* obs, float* vec, float* gmap, float* gvec, void* stream);
int mdl_host_views_shaped_reward(MdlEngine* eng, const int32_t* prev_views, const int64_t* prev_offsets,
                                 int32_t max_slots, const int32_t* cur, const int64_t* cur_offsets,
                                 const uint8_t* actions, const int64_t* act_offsets, const double* g, int32_t n,
                                 const double* consts, float* out, void* stream);
/* One view / one transition with its inputs in the caller's host memory (any: they are copied
 * into the kernel's arguments at launch, so the wave reads them without round trips to host
 * memory) and its outputs in the arena; synchronous as above.  rec: one view record (layout of
 * mdl_views_features) of `words` <= MDL_VIEW_INLINE_WORDS words.  For the shaped reward the
 * previous view, the current record and the action codes together must fit that capacity
 * (prev_words + cur_words + ceil(n_actions / 4)); n_actions >= the view's robots.  Larger
 * inputs take the arena entries above.  The shaped reward comes back beside the completion word,
 * so `out` may be any host memory.  The single-call paths of marl_gpu.helper. */
#define MDL_VIEW_INLINE_WORDS 768
int mdl_host_view_features(MdlEngine* eng, const int32_t* rec, int32_t words, int32_t agent_index, int32_t T,
                           int32_t MO, int32_t MP, int32_t MR, int32_t MPs, float* obs, float* vec, float* gmap,
                           float* gvec, void* stream);
int mdl_host_view_shaped_reward(MdlEngine* eng, const int32_t* prev_view, int32_t prev_words, const int32_t* cur,
                                int32_t cur_words, const uint8_t* actions, int32_t n_actions, double g,
                                const double* consts, float* out, void* stream);

/* ---- checkpoint of the engine state ----
 * A versioned host blob: a 56-byte header (magic "MDLSTATE", version, E, A, P, T, tracker mode,
 * map fingerprint) then every state buffer (robots, packages, state words, env records,
 * MT19937 states, tracker data, episode results).  Loading it into an engine of the same
 * configuration resumes every env's stream exactly, RNG included; any other engine refuses it.
 * save / load are synchronous on `stream`; the buffer is host memory. */
int mdl_state_bytes(MdlEngine* eng, int64_t* bytes);
int mdl_save_state(MdlEngine* eng, void* host_buf, int64_t bytes, void* stream);
int mdl_load_state(MdlEngine* eng, const void* host_buf, int64_t bytes, void* stream);

/* ---- rollout glue: keeps MAPPO/trainer.py:133-290 on the device ---- */

/* Categorical(logits=...).sample() and .log_prob() (MAPPO/trainer.py:141-143) for n_rows rows of
 * n_actions float32 logits (row-major, contiguous).  Inverse CDF of softmax(logits) on a
 * Philox4x32-10 uniform keyed by (seed, offset, row): deterministic for a given (seed, offset),
 * independent of launch shape; a caller advances `offset` once per call.  actions: uint8 [n_rows]
 * (the trainer-int action, ready for mdl_step); log_probs: float32 [n_rows] or NULL. */
int mdl_sample_actions(const float* logits, int64_t n_rows, int32_t n_actions, uint64_t seed, uint64_t offset,
                       uint8_t* actions, float* log_probs, void* stream);

/* The same draw with the offset read on the device: offset = *offset_dev + offset_add, so a
 * captured hipGraph of a whole rollout replays with fresh offsets (MAPPO/trainer.py:141-143:
 * each rollout samples new actions).  Identical results to mdl_sample_actions at that offset. */
int mdl_sample_actions_dev(const float* logits, int64_t n_rows, int32_t n_actions, uint64_t seed,
                           const uint64_t* offset_dev, uint64_t offset_add, uint8_t* actions, float* log_probs,
                           void* stream);

/* *counter += value on the device (stream-ordered; advances offset_dev inside a graph). */
int mdl_counter_add(uint64_t* counter, uint64_t value, void* stream);

/* Generalised advantage estimation exactly as MAPPO/trainer.py:266-276 computes it in float32
 * (same operation order): rewards, values, dones [T][n] (dones uint8), next_value [n];
 * gamma = float32(GAMMA), gamma_lambda = float32(GAMMA * GAE_LAMBDA) with the product in double.
 * Writes advantages and returns (= advantages + values) [T][n]. */
int mdl_gae(const float* rewards, const float* values, const float* next_value, const uint8_t* dones, int32_t T,
            int64_t n, float gamma, float gamma_lambda, float* advantages, float* returns, void* stream);

/* Observation builders for envs [env_begin, env_begin+n), which must share one
 * map shape (H, W), from the current state + tracker:
 *   actor_map  f32 [n][A][6][H][W]          convert_observation       MAPPO/helper.py:6-66
 *   actor_vec  f32 [n][A][6+5MO+5MP+1]      generate_vector_features  MAPPO/helper.py:68-165
 *   critic_map f32 [n][4][H][W]             convert_global_state[0]   MAPPO/helper.py:167-198
 *   critic_vec f32 [n][6MR+7MPs+1]          convert_global_state[1]   MAPPO/helper.py:199-255
 * Any output pointer may be NULL. */
int mdl_build_obs(MdlEngine* eng, int32_t env_begin, int32_t n, float* actor_map, float* actor_vec,
                  float* critic_map, float* critic_vec, void* stream);

/* State snapshot into caller DEVICE buffers (async on `stream`).  Any pointer may be NULL.
 *   robots   int32 [E][A][3]  (row, col, carrying), 0-indexed
 *   pkgs     int32 [E][P][8]  (sr, sc, tr, tc, start_time, deadline, id, status 0 None/1 waiting/2 in_transit/3 delivered)
 *   t        int32 [E];  total_reward f64 [E]
 *   tracker  int32 [E][P][4]  per id 1..P: (present, in_transit, order, _) ; data rows in tracker_data int32 [E][P][6]
 * Backs the dict view of Environment.get_state (env.py:127-147). */
int mdl_read_state(MdlEngine* eng, int32_t* robots, int32_t* pkgs, int32_t* t, double* total_reward,
                   int32_t* tracker, int32_t* tracker_data, void* stream);

/* Helper-compatible builders on arbitrary state dicts ("views"): the same
 * device code as mdl_build_obs / the fused shaping, fed from a packed int32
 * record per view instead of engine state.  View record layout (int32):
 *   [0] t  [1] A  [2] n_slots  [3] map index
 *   then A x (row, col, carrying)           0-indexed robot rows (state['robots'] minus 1)
 *   then n_slots x (id, status 1|2, sr, sc, tr, tc, start_time, deadline)  tracker in dict order
 * views: device int32 blob; offsets: device int64 [n_views] record starts;
 * max_slots: the largest n_slots of any record (sizes the LDS slice).
 * Robot and package cells must lie inside the view's map.
 * agent_idx: device int32 [n_views] (may be out of range -> reference's
 * early-return outputs).  Outputs per view: obs [6][H][W], vec [6+5MO+5MP+1],
 * gmap [4][H][W], gvec [6MR+7MPs+1] (NULL to skip).  T/MO/MP/MR/MPs are call
 * arguments here.  Replaces convert_observation / generate_vector_features /
 * convert_global_state called on dicts (MAPPO/helper.py:6-255). */
int mdl_views_features(MdlEngine* eng, const int32_t* views, const int64_t* offsets, int32_t n_views,
                       int32_t max_slots, const int32_t* agent_idx, int32_t T, int32_t MO, int32_t MP, int32_t MR, int32_t MPs,
                       float* obs, float* vec, float* gmap, float* gvec, void* stream);

/* compute_shaped_rewards (MAPPO/helper.py:257-369) on dict inputs: prev view
 * record (state + tracker_prev as above), current robots int32 [A][3]
 * (0-indexed) and time, actions uint8 [A] in MDL_ACTION_CODES, global reward
 * (fp64).  cur: device int32 blob, cur_offsets: int64 [n] (record = [t, A,
 * then A x 3]); actions: uint8 blob with act_offsets int64 [n]; g: f64 [n];
 * consts: host double[9] (NULL = engine's).  Output: f32 [n]. */
int mdl_views_shaped_reward(MdlEngine* eng, const int32_t* prev_views, const int64_t* prev_offsets, int32_t max_slots,
                            const int32_t* cur, const int64_t* cur_offsets, const uint8_t* actions,
                            const int64_t* act_offsets, const double* g, int32_t n, const double* consts,
                            float* out, void* stream);

/* Host-only (no GPU needed): the distance-rank table the feature sorts use.
 * out[(dr+H-1)*(2W-1) + dc+W-1] = rank of the fp64 key (dr/H)**2 + (dc/W)**2
 * (CPython float_pow -> libm pow) among all distinct keys of the map shape;
 * equal doubles share a rank.  out holds (2H-1)*(2W-1) entries.  This is the
 * order of others.sort / pkgs.sort in MAPPO/helper.py:139,158. */
int mdl_rank_table(int32_t H, int32_t W, uint16_t* out);

/* Introspection */
int mdl_get_config(const MdlEngine* eng, MdlConfig* out);
/* The step layout (MDL_STEP_LAYOUT_WAVE, _ROWS or _HALVES) mdl_step launches for a call over n envs
 * (use_ids = 0: the full batch, n ignored as in mdl_step; use_ids = 1: an env_ids subset of n,
 * always WAVE) -- the engine's own decision, the one mdl_step takes. */
int mdl_step_layout(const MdlEngine* eng, int32_t n, int32_t use_ids, int32_t* layout);
/* The layout of the last mdl_step launch on this engine (0 before the first one). */
int mdl_last_step_layout(const MdlEngine* eng, int32_t* layout);
/* The symbol (as rocprof reports it, e.g. "mdl::k_step<true, 1, false, 5>") of the kernel mdl_step
 * launches in `layout` (WAVE / ROWS / HALVES), or, with with_obs, of mdl_step_obs's step launch (its fused
 * step + observation kernel where it applies).  NUL-terminated into out[cap]. */
int mdl_step_kernel_name(const MdlEngine* eng, int32_t layout, int32_t with_obs, char* out, int32_t cap);
int mdl_obs_dims(const MdlEngine* eng, int32_t* actor_vec_dim, int32_t* critic_vec_dim);
const char* mdl_last_error(void);
const char* mdl_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MDL_ENGINE_H */
