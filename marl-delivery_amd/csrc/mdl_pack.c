/*
 * mdl_pack.c -- CPython extension: the helper functions' dict -> view-record packing in C.
 *
 * The helper-compatible functions (marl_gpu.helper: convert_observation, generate_vector_features,
 * convert_global_state, compute_shaped_rewards on one state dict, MAPPO/helper.py:6-369) hand the
 * device one int32 "view" record per call (include/mdl_engine.h, mdl_views_features):
 *     [t, A, n_slots, map] + A x (row, col, carrying) 0-indexed + n_slots x (id, status 1|2, sr, sc, tr, tc, st, dl)
 * Built from Python objects with numpy that took tens of microseconds per call -- more than the
 * reference's whole CPU helper; this walks the dicts once and writes the words straight into the
 * engine's host-mapped arena (an address the caller passes), so the kernel reads them from there.
 *
 * features() / shaped() go one step further for the single-view helper calls: pack, launch through
 * the engine's self-publishing entries (mdl_host_views_features / mdl_host_views_shaped_reward,
 * whose addresses bind() receives once), wait, and return the numpy outputs -- no ctypes call and
 * no Python-level buffer handling per call.
 *
 * The GIL stays held across each call: the mailbox, the arena and their host-side counters are
 * shared per engine, so two threads stepping envs of one engine (or calling helpers on one map)
 * must not interleave -- the GIL serialises them (the calls are microseconds long).
 *
 * Host plumbing only (no GPU code, no reference semantics beyond the record layout).  The tracker
 * dict is read in insertion order (PyDict_Next), the order the reference iterates
 * persistent_packages.values() in (MAPPO/trainer.py:95-130); 'status' == 'in_transit' -> 2, else 1.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#include <numpy/arrayobject.h>
#include <numpy/arrayscalars.h>

#include "mdl_engine.h"   /* MDL_VIEW_INLINE_WORDS */

static int get_int(PyObject* o, long* out) {
    long v = PyLong_AsLong(o);
    if (v == -1 && PyErr_Occurred()) return -1;
    *out = v;
    return 0;
}

/* item k of a sequence (tuple / list fast paths) as a long */
static int seq_int(PyObject* seq, Py_ssize_t k, long* out) {
    PyObject* it;
    if (PyTuple_Check(seq)) {
        if (k >= PyTuple_GET_SIZE(seq)) goto short_seq;
        return get_int(PyTuple_GET_ITEM(seq, k), out);
    }
    if (PyList_Check(seq)) {
        if (k >= PyList_GET_SIZE(seq)) goto short_seq;
        return get_int(PyList_GET_ITEM(seq, k), out);
    }
    it = PySequence_GetItem(seq, k);
    if (!it) return -1;
    {
        const int rc = get_int(it, out);
        Py_DECREF(it);
        return rc;
    }
short_seq:
    PyErr_SetString(PyExc_ValueError, "sequence too short");
    return -1;
}

/* interned keys (their hashes are cached: a lookup costs no string construction) */
static PyObject *s_in_transit, *k_id, *k_status, *k_start_pos, *k_target_pos, *k_start_time, *k_deadline;

static PyObject* dict_get(PyObject* d, PyObject* key) {
    PyObject* v = PyDict_Check(d) ? PyDict_GetItemWithError(d, key) : NULL;   /* borrowed */
    if (!v && !PyErr_Occurred()) {
        if (PyDict_Check(d)) PyErr_SetObject(PyExc_KeyError, key);
        else PyErr_SetString(PyExc_TypeError, "tracker entries must be dicts");
    }
    return v;
}

static int dict_int(PyObject* d, PyObject* key, long* out) {
    PyObject* v = dict_get(d, key);
    return v ? get_int(v, out) : -1;
}

static int dict_pair(PyObject* d, PyObject* key, long* a, long* b) {
    PyObject* v = dict_get(d, key);
    if (!v) return -1;
    if (seq_int(v, 0, a) || seq_int(v, 1, b)) return -1;
    return 0;
}

/* The view record [t, A, n, map] + A x (row, col, carrying) 0-indexed + n x (id, status, sr, sc, tr, tc,
 * st, dl) at w (cap words), from the first `amax` robots (amax < 0: all).  robots: sequence of
 * (row, col, carrying) 1-indexed; tracker: dict id -> entry dict in insertion order
 * (MAPPO/trainer.py:95-130 layout), or a sequence of rows.  Returns the words written, or -1 with an
 * exception set. */
static Py_ssize_t do_pack_view(int32_t* w, Py_ssize_t cap, long t, PyObject* robots, PyObject* tracker, long H,
                               long W, long map_index, Py_ssize_t amax) {
    PyObject* rs = PySequence_Fast(robots, "robots must be a sequence");
    if (!rs) return -1;
    Py_ssize_t A = PySequence_Fast_GET_SIZE(rs);
    if (amax >= 0 && amax < A) A = amax;
    const int is_dict = PyDict_Check(tracker);
    PyObject* ts = NULL;
    Py_ssize_t n;
    if (is_dict) {
        n = PyDict_Size(tracker);
    } else {
        ts = PySequence_Fast(tracker, "tracker must be a dict or a sequence of rows");
        if (!ts) {
            Py_DECREF(rs);
            return -1;
        }
        n = PySequence_Fast_GET_SIZE(ts);
    }
    Py_ssize_t ret = -1;
    if (A > 64) {
        PyErr_SetString(PyExc_ValueError, "at most 64 robots per view");
        goto done;
    }
    if (4 + 3 * A + 8 * n > cap) {
        PyErr_SetString(PyExc_ValueError, "view record larger than the arena");
        goto done;
    }
    w[0] = (int32_t)t;
    w[1] = (int32_t)A;
    w[2] = (int32_t)n;
    w[3] = (int32_t)map_index;
    int32_t* o = w + 4;
    for (Py_ssize_t i = 0; i < A; i++) {
        long r, c, cy;
        PyObject* rb = PySequence_Fast_GET_ITEM(rs, i);
        if (seq_int(rb, 0, &r) || seq_int(rb, 1, &c) || seq_int(rb, 2, &cy)) goto done;
        r -= 1;
        c -= 1;
        if (r < 0 || r >= H || c < 0 || c >= W) {
            PyErr_SetString(PyExc_ValueError, "robot positions must lie inside the map");
            goto done;
        }
        o[0] = (int32_t)r;
        o[1] = (int32_t)c;
        o[2] = (int32_t)cy;
        o += 3;
    }
    Py_ssize_t pos = 0, k = 0;
    PyObject *key, *v;
    while (k < n) {
        long id, st, sr, sc, tr, tc, t0, dl;
        if (is_dict) {
            if (!PyDict_Next(tracker, &pos, &key, &v)) break;
            PyObject* sv = dict_get(v, k_status);
            if (!sv) goto done;
            const int eq = sv == s_in_transit ? 1 : PyObject_RichCompareBool(sv, s_in_transit, Py_EQ);
            if (eq < 0) goto done;
            st = eq ? 2 : 1;
            if (dict_int(v, k_id, &id) || dict_pair(v, k_start_pos, &sr, &sc) || dict_pair(v, k_target_pos, &tr, &tc) ||
                dict_int(v, k_start_time, &t0) || dict_int(v, k_deadline, &dl))
                goto done;
        } else {
            v = PySequence_Fast_GET_ITEM(ts, k);
            if (seq_int(v, 0, &id) || seq_int(v, 1, &st) || seq_int(v, 2, &sr) || seq_int(v, 3, &sc) ||
                seq_int(v, 4, &tr) || seq_int(v, 5, &tc) || seq_int(v, 6, &t0) || seq_int(v, 7, &dl))
                goto done;
        }
        if (sr < 0 || sr >= H || sc < 0 || sc >= W || tr < 0 || tr >= H || tc < 0 || tc >= W) {
            PyErr_SetString(PyExc_ValueError, "package cells must lie inside the map");
            goto done;
        }
        if (t0 < 0 || t0 > 65535 || dl < 0 || dl > 65535) {
            PyErr_SetString(PyExc_ValueError, "start_time / deadline must fit 16 bits");
            goto done;
        }
        o[0] = (int32_t)id;
        o[1] = (int32_t)st;
        o[2] = (int32_t)sr;
        o[3] = (int32_t)sc;
        o[4] = (int32_t)tr;
        o[5] = (int32_t)tc;
        o[6] = (int32_t)t0;
        o[7] = (int32_t)dl;
        o += 8;
        k++;
    }
    ret = 4 + 3 * A + 8 * n;
done:
    Py_DECREF(rs);
    Py_XDECREF(ts);
    return ret;
}

/* pack_view(addr, cap_words, t, robots, tracker, H, W, map_index) -> words written. */
static PyObject* pack_view(PyObject* self, PyObject* args) {
    unsigned long long addr;
    Py_ssize_t cap;
    long t, H, W, map_index;
    PyObject *robots, *tracker;
    (void)self;
    if (!PyArg_ParseTuple(args, "KnlOOlll", &addr, &cap, &t, &robots, &tracker, &H, &W, &map_index)) return NULL;
    const Py_ssize_t nw = do_pack_view((int32_t*)(uintptr_t)addr, cap, t, robots, tracker, H, W, map_index, -1);
    return nw < 0 ? NULL : PyLong_FromSsize_t(nw);
}

/* [t, A] + A x (row, col, carrying) 0-indexed at w from the first `amax` robots (amax < 0: all)
 * (the "current state" record of mdl_views_shaped_reward).  Returns the words, or -1. */
static Py_ssize_t do_pack_robots(int32_t* w, Py_ssize_t cap, long t, PyObject* robots, Py_ssize_t amax) {
    PyObject* rs = PySequence_Fast(robots, "robots must be a sequence");
    if (!rs) return -1;
    Py_ssize_t A = PySequence_Fast_GET_SIZE(rs);
    if (amax >= 0 && amax < A) A = amax;
    if (2 + 3 * A > cap) {
        Py_DECREF(rs);
        PyErr_SetString(PyExc_ValueError, "record larger than the arena");
        return -1;
    }
    w[0] = (int32_t)t;
    w[1] = (int32_t)A;
    for (Py_ssize_t i = 0; i < A; i++) {
        long r, c, cy;
        PyObject* rb = PySequence_Fast_GET_ITEM(rs, i);
        if (seq_int(rb, 0, &r) || seq_int(rb, 1, &c) || seq_int(rb, 2, &cy)) {
            Py_DECREF(rs);
            return -1;
        }
        w[2 + 3 * i] = (int32_t)(r - 1);
        w[3 + 3 * i] = (int32_t)(c - 1);
        w[4 + 3 * i] = (int32_t)cy;
    }
    Py_DECREF(rs);
    return 2 + 3 * A;
}

/* pack_robots(addr, cap_words, t, robots) -> words */
static PyObject* pack_robots(PyObject* self, PyObject* args) {
    unsigned long long addr;
    Py_ssize_t cap;
    long t;
    PyObject* robots;
    (void)self;
    if (!PyArg_ParseTuple(args, "KnlO", &addr, &cap, &t, &robots)) return NULL;
    const Py_ssize_t nw = do_pack_robots((int32_t*)(uintptr_t)addr, cap, t, robots, -1);
    return nw < 0 ? NULL : PyLong_FromSsize_t(nw);
}

/* ---- one-call helpers ---- */
typedef int (*views_features_fn)(void* eng, const int32_t* views, const int64_t* offsets, int32_t n_views,
                                 int32_t max_slots, const int32_t* agent_idx, int32_t T, int32_t MO, int32_t MP,
                                 int32_t MR, int32_t MPs, float* obs, float* vec, float* gmap, float* gvec,
                                 void* stream);
typedef int (*views_shaped_fn)(void* eng, const int32_t* prev_views, const int64_t* prev_offsets, int32_t max_slots,
                               const int32_t* cur, const int64_t* cur_offsets, const uint8_t* actions,
                               const int64_t* act_offsets, const double* g, int32_t n, const double* consts,
                               float* out, void* stream);
typedef int (*view_features_fn)(void* eng, const int32_t* rec, int32_t words, int32_t agent_index, int32_t T,
                                int32_t MO, int32_t MP, int32_t MR, int32_t MPs, float* obs, float* vec, float* gmap,
                                float* gvec, void* stream);
typedef int (*view_shaped_fn)(void* eng, const int32_t* prev_view, int32_t prev_words, const int32_t* cur,
                              int32_t cur_words, const uint8_t* actions, int32_t n_actions, double g,
                              const double* consts, float* out, void* stream);
typedef const char* (*last_error_fn)(void);
static views_features_fn f_features;
static views_shaped_fn f_shaped;
static view_features_fn f_features1;
static view_shaped_fn f_shaped1;
static last_error_fn f_last_error;
static PyObject* exc_type;   /* marl_gpu._lib.MdlError */

/* bind(addr mdl_host_views_features, addr mdl_host_views_shaped_reward, addr mdl_host_view_features,
 *      addr mdl_host_view_shaped_reward, addr mdl_last_error, MdlError) */
static PyObject* bind(PyObject* self, PyObject* args) {
    unsigned long long a, b, a1, b1, c;
    PyObject* exc;
    (void)self;
    if (!PyArg_ParseTuple(args, "KKKKKO", &a, &b, &a1, &b1, &c, &exc)) return NULL;
    f_features = (views_features_fn)(uintptr_t)a;
    f_shaped = (views_shaped_fn)(uintptr_t)b;
    f_features1 = (view_features_fn)(uintptr_t)a1;
    f_shaped1 = (view_shaped_fn)(uintptr_t)b1;
    f_last_error = (last_error_fn)(uintptr_t)c;
    Py_INCREF(exc);
    Py_XSETREF(exc_type, exc);
    Py_RETURN_NONE;
}

static PyObject* lib_error(const char* what) {
    PyErr_Format(exc_type ? exc_type : PyExc_RuntimeError, "%s: %s", what, f_last_error ? f_last_error() : "?");
    return NULL;
}

static Py_ssize_t align16(Py_ssize_t x) { return (x + 15) & ~(Py_ssize_t)15; }

static Py_ssize_t seq_len(PyObject* o) {
    if (PyDict_Check(o)) return PyDict_Size(o);
    return PyObject_Length(o);
}

/* features(eng, stream, arena, cap_bytes, t, robots, tracker, H, W, agent_index, T, MO, MP, MR, MPs, want)
 *   -> tuple of float32 arrays for the bits of `want` (1 obs [6,H,W], 2 vec [6+5MO+5MP+1],
 *      4 gmap [4,H,W], 8 gvec [6MR+7MPs+1]), or the arena bytes needed (int) when cap_bytes is short.
 * A record of at most MDL_VIEW_INLINE_WORDS words travels in the kernel arguments
 * (mdl_host_view_features) and the arena holds only the outputs; a larger one goes through the
 * arena: view record | int64 offset 0 | agent index | outputs (16-byte aligned). */
static PyObject* features(PyObject* self, PyObject* args) {
    unsigned long long eng, stream, arena;
    Py_ssize_t cap;
    long t, H, W, idx, T, MO, MP, MR, MPs, want;
    PyObject *robots, *tracker;
    (void)self;
    if (!PyArg_ParseTuple(args, "KKKnlOOlllllllll", &eng, &stream, &arena, &cap, &t, &robots, &tracker, &H, &W, &idx,
                          &T, &MO, &MP, &MR, &MPs, &want))
        return NULL;
    if (!f_features) {
        PyErr_SetString(PyExc_RuntimeError, "_mdl_pack.bind() not called");
        return NULL;
    }
    const Py_ssize_t A = seq_len(robots), ns = seq_len(tracker);
    if (A < 0 || ns < 0) return NULL;
    const Py_ssize_t HW = H * W;
    const Py_ssize_t sz[4] = {6 * HW, 6 + 5 * MO + 5 * MP + 1, 4 * HW, 6 * MR + 7 * MPs + 1};
    const Py_ssize_t vw = 4 + 3 * A + 8 * ns;
    const int inl = vw <= MDL_VIEW_INLINE_WORDS;
    const Py_ssize_t o_off = align16(4 * vw), o_idx = align16(o_off + 8);
    Py_ssize_t pos = inl ? 0 : align16(o_idx + 4), o_out[4];
    int nout = 0;
    for (int k = 0; k < 4; k++) {
        o_out[k] = -1;
        if (want & (1 << k)) {
            o_out[k] = pos;
            pos = align16(pos + 4 * sz[k]);
            nout++;
        }
    }
    if (pos > cap) return PyLong_FromSsize_t(pos);
    char* b = (char*)(uintptr_t)arena;
    float* outp[4];
    for (int k = 0; k < 4; k++) outp[k] = o_out[k] >= 0 ? (float*)(b + o_out[k]) : NULL;
    int rc;
    if (inl) {
        int32_t rec[MDL_VIEW_INLINE_WORDS];
        if (do_pack_view(rec, vw, t, robots, tracker, H, W, 0, -1) < 0) return NULL;
        rc = f_features1((void*)(uintptr_t)eng, rec, (int32_t)vw, (int32_t)idx, (int32_t)T, (int32_t)MO, (int32_t)MP,
                         (int32_t)MR, (int32_t)MPs, outp[0], outp[1], outp[2], outp[3], (void*)(uintptr_t)stream);
        if (rc) return lib_error("mdl_host_view_features");
    } else {
        if (do_pack_view((int32_t*)b, vw, t, robots, tracker, H, W, 0, -1) < 0) return NULL;
        *(int64_t*)(b + o_off) = 0;
        *(int32_t*)(b + o_idx) = (int32_t)idx;
        rc = f_features((void*)(uintptr_t)eng, (const int32_t*)b, (const int64_t*)(b + o_off), 1, (int32_t)ns,
                        (const int32_t*)(b + o_idx), (int32_t)T, (int32_t)MO, (int32_t)MP, (int32_t)MR, (int32_t)MPs,
                        outp[0], outp[1], outp[2], outp[3], (void*)(uintptr_t)stream);
        if (rc) return lib_error("mdl_host_views_features");
    }
    PyObject* tup = PyTuple_New(nout);
    if (!tup) return NULL;
    int j = 0;
    for (int k = 0; k < 4; k++) {
        if (!outp[k]) continue;
        npy_intp dims[3] = {k == 0 ? 6 : 4, H, W};
        if (k == 1 || k == 3) dims[0] = sz[k];
        PyObject* arr = PyArray_SimpleNew((k == 1 || k == 3) ? 1 : 3, dims, NPY_FLOAT32);
        if (!arr) {
            Py_DECREF(tup);
            return NULL;
        }
        memcpy(PyArray_DATA((PyArrayObject*)arr), outp[k], 4 * (size_t)sz[k]);
        PyTuple_SET_ITEM(tup, j++, arr);
    }
    return tup;
}

/* MOVE_CODES / OP_CODES of marl_gpu.compat: one-character strings, anything else 5 / 3 */
static int move_code(PyObject* o) {
    if (PyUnicode_Check(o) && PyUnicode_GET_LENGTH(o) == 1) {
        switch (PyUnicode_READ_CHAR(o, 0)) {
            case 'S': return 0;
            case 'L': return 1;
            case 'R': return 2;
            case 'U': return 3;
            case 'D': return 4;
        }
    }
    return 5;
}

static int op_code(PyObject* o) {
    if (PyUnicode_Check(o) && PyUnicode_GET_LENGTH(o) == 1) {
        const Py_UCS4 c = PyUnicode_READ_CHAR(o, 0);
        if (c >= '0' && c <= '2') return (int)(c - '0');
    }
    return 3;
}

/* shaped(eng, stream, arena, cap_bytes, g, prev_t, prev_robots, cur_t, cur_robots, actions, num_agents, tracker,
 *        H, W, consts_addr) -> numpy.float32, or the arena bytes needed (int) when cap_bytes is short.
 * actions: (move, op) pairs (compat._code's mapping) or bytes of MDL_ACTION_CODES.
 * The first num_agents robots / actions of each (list(...)[:num_agents], MAPPO/helper.py:257-369).
 * Arena layout: prev view | cur record | action codes | int64 offset 0 | pad | g (f64) | out (f32). */
static PyObject* shaped(PyObject* self, PyObject* args) {
    unsigned long long eng, stream, arena, consts;
    Py_ssize_t cap, na;
    double g;
    long pt, ct, H, W;
    PyObject *prev_r, *cur_r, *actions, *tracker;
    (void)self;
    if (!PyArg_ParseTuple(args, "KKKndlOlOOnOllK", &eng, &stream, &arena, &cap, &g, &pt, &prev_r, &ct, &cur_r,
                          &actions, &na, &tracker, &H, &W, &consts))
        return NULL;
    if (!f_shaped) {
        PyErr_SetString(PyExc_RuntimeError, "_mdl_pack.bind() not called");
        return NULL;
    }
    Py_ssize_t Ap = seq_len(prev_r), Ac = seq_len(cur_r), ns = seq_len(tracker);
    if (Ap < 0 || Ac < 0 || ns < 0) return NULL;
    /* (move, op) pairs, or code bytes (MDL_ACTION_CODES) */
    const int as_codes = PyBytes_Check(actions);
    PyObject* acts = as_codes ? (Py_INCREF(actions), actions) : PySequence_Fast(actions, "actions must be a sequence");
    if (!acts) return NULL;
    Py_ssize_t Na = as_codes ? PyBytes_GET_SIZE(acts) : PySequence_Fast_GET_SIZE(acts);
    /* Python's [:num_agents] */
    const Py_ssize_t lim_p = na >= 0 ? na : Ap + na, lim_c = na >= 0 ? na : Ac + na, lim_a = na >= 0 ? na : Na + na;
    Ap = lim_p < 0 ? 0 : (lim_p < Ap ? lim_p : Ap);
    Ac = lim_c < 0 ? 0 : (lim_c < Ac ? lim_c : Ac);
    Na = lim_a < 0 ? 0 : (lim_a < Na ? lim_a : Na);
    const Py_ssize_t vw = 4 + 3 * Ap + 8 * ns, cw = 2 + 3 * Ac;
    /* inline (mdl_host_view_shaped_reward): the inputs in the kernel arguments, the output at arena
     * offset 0; else the arena layout above */
    const int inl = vw + cw + (Na + 3) / 4 <= MDL_VIEW_INLINE_WORDS;
    const Py_ssize_t o_c = align16(4 * vw), o_a = align16(o_c + 4 * cw), o_off = align16(o_a + Na);
    const Py_ssize_t o_out = inl ? 0 : o_off + 24, need = inl ? 16 : o_off + 48;
    int32_t rec[MDL_VIEW_INLINE_WORDS];
    PyObject* ret = NULL;
    if (Na < Ap || Ac < Ap) {   /* the reference indexes all three per agent (IndexError) */
        PyErr_Format(PyExc_IndexError, "%zd robots before the step, but %zd after and %zd actions", Ap, Ac, Na);
        goto done;
    }
    if (need > cap) {
        ret = PyLong_FromSsize_t(need);
        goto done;
    }
    char* b = (char*)(uintptr_t)arena;
    char* in = inl ? (char*)rec : b;   /* where the inputs are packed */
    const Py_ssize_t i_c = inl ? 4 * vw : o_c, i_a = inl ? 4 * (vw + cw) : o_a;
    if (do_pack_view((int32_t*)in, vw, pt, prev_r, tracker, H, W, 0, Ap) < 0) goto done;
    if (do_pack_robots((int32_t*)(in + i_c), cw, ct, cur_r, Ac) < 0) goto done;
    if (as_codes) memcpy(in + i_a, PyBytes_AS_STRING(acts), (size_t)Na);
    for (Py_ssize_t i = 0; i < Na && !as_codes; i++) {
        PyObject* pr = PySequence_Fast(PySequence_Fast_GET_ITEM(acts, i), "each action must be a (move, op) pair");
        if (!pr) goto done;
        if (PySequence_Fast_GET_SIZE(pr) != 2) {
            Py_DECREF(pr);
            PyErr_SetString(PyExc_ValueError, "each action must be a (move, op) pair");
            goto done;
        }
        in[i_a + i] = (char)(move_code(PySequence_Fast_GET_ITEM(pr, 0)) | (op_code(PySequence_Fast_GET_ITEM(pr, 1)) << 3));
        Py_DECREF(pr);
    }
    int rc;
    const double* cp = consts ? (const double*)(uintptr_t)consts : NULL;
    if (inl) {
        rc = f_shaped1((void*)(uintptr_t)eng, rec, (int32_t)vw, rec + vw, (int32_t)cw, (const uint8_t*)(rec + vw + cw),
                       (int32_t)Na, g, cp, (float*)(b + o_out), (void*)(uintptr_t)stream);
    } else {
        *(int64_t*)(b + o_off) = 0;
        *(int64_t*)(b + o_off + 8) = 0;
        *(double*)(b + o_off + 16) = g;
        rc = f_shaped((void*)(uintptr_t)eng, (const int32_t*)b, (const int64_t*)(b + o_off), (int32_t)ns,
                      (const int32_t*)(b + o_c), (const int64_t*)(b + o_off), (const uint8_t*)(b + o_a),
                      (const int64_t*)(b + o_off), (const double*)(b + o_off + 16), 1, cp, (float*)(b + o_out),
                      (void*)(uintptr_t)stream);
    }
    if (rc) {
        lib_error(inl ? "mdl_host_view_shaped_reward" : "mdl_host_views_shaped_reward");
        goto done;
    }
    ret = PyArrayScalar_New(Float);
    if (ret) PyArrayScalar_ASSIGN(ret, Float, *(const float*)(b + o_out));
done:
    Py_DECREF(acts);
    return ret;
}

/* ---- Environment.step on the mailbox in one C call ---- */
typedef int (*mail_step_fn)(void* eng, int32_t n, int32_t use_ids, int32_t auto_reset, void* stream);
typedef struct {
    mail_step_fn step;
    void* eng;
    uint8_t* codes;
    int32_t* ids;
    const double* r_env;
    const uint8_t* done;
    const int32_t* robots;
    const int32_t* pkgs;
    const int32_t* t;
    const double* total;
    const int32_t* rterms;
    int A, P;
} MailCtx;

static void mail_ctx_free(PyObject* cap) { PyMem_Free(PyCapsule_GetPointer(cap, "mdl.mailctx")); }

/* mail_ctx(addr mdl_mail_step, eng, codes, ids, r_env, done, robots, pkgs, t, total, rterms, A, P) -> capsule */
static PyObject* mail_ctx(PyObject* self, PyObject* args) {
    unsigned long long f, eng, codes, ids, r_env, done, robots, pkgs, t, total, rterms;
    int A, P;
    (void)self;
    if (!PyArg_ParseTuple(args, "KKKKKKKKKKKii", &f, &eng, &codes, &ids, &r_env, &done, &robots, &pkgs, &t, &total,
                          &rterms, &A, &P))
        return NULL;
    MailCtx* c = (MailCtx*)PyMem_Malloc(sizeof(MailCtx));
    if (!c) return PyErr_NoMemory();
    c->step = (mail_step_fn)(uintptr_t)f;
    c->eng = (void*)(uintptr_t)eng;
    c->codes = (uint8_t*)(uintptr_t)codes;
    c->ids = (int32_t*)(uintptr_t)ids;
    c->r_env = (const double*)(uintptr_t)r_env;
    c->done = (const uint8_t*)(uintptr_t)done;
    c->robots = (const int32_t*)(uintptr_t)robots;
    c->pkgs = (const int32_t*)(uintptr_t)pkgs;
    c->t = (const int32_t*)(uintptr_t)t;
    c->total = (const double*)(uintptr_t)total;
    c->rterms = (const int32_t*)(uintptr_t)rterms;
    c->A = A;
    c->P = P;
    PyObject* cap = PyCapsule_New(c, "mdl.mailctx", mail_ctx_free);
    if (!cap) PyMem_Free(c);
    return cap;
}

/* get_state's dict from mailbox row 0 (env.py:127-147): 1-indexed robots, the packages whose
 * start_time is t as (id, sr+1, sc+1, tr+1, tc+1, start_time, deadline) */
static PyObject* state_dict(const MailCtx* c, int w, PyObject* grid) {
    const int A = c->A, P = c->P, t = c->t[w];
    const int32_t* robots = c->robots + (size_t)w * A * 3;
    const int32_t* pkgs = c->pkgs + (size_t)w * P * 8;
    PyObject* rl = PyList_New(A);
    if (!rl) return NULL;
    for (int i = 0; i < A; i++) {
        const int32_t* r = robots + 3 * i;
        PyObject* tp = Py_BuildValue("(iii)", r[0] + 1, r[1] + 1, r[2]);
        if (!tp) {
            Py_DECREF(rl);
            return NULL;
        }
        PyList_SET_ITEM(rl, i, tp);
    }
    PyObject* pl = PyList_New(0);
    if (!pl) {
        Py_DECREF(rl);
        return NULL;
    }
    for (int j = 0; j < P; j++) {
        const int32_t* q = pkgs + 8 * j;
        if (q[4] != t) continue;
        PyObject* tp = Py_BuildValue("(iiiiiii)", q[6], q[0] + 1, q[1] + 1, q[2] + 1, q[3] + 1, q[4], q[5]);
        if (!tp || PyList_Append(pl, tp) < 0) {
            Py_XDECREF(tp);
            Py_DECREF(rl);
            Py_DECREF(pl);
            return NULL;
        }
        Py_DECREF(tp);
    }
    PyObject* d = Py_BuildValue("{s:i,s:O,s:N,s:N}", "time_step", t, "map", grid, "robots", rl, "packages", pl);
    return d;
}

/* the codes of one env's actions into row w of the mailbox (compat._code's mapping); a count other
 * than n_robots raises env.py:182-183's ValueError */
static int encode_into(uint8_t* row, int A, PyObject* actions, int n_robots) {
    PyObject* acts = PySequence_Fast(actions, "actions must be a sequence");
    if (!acts) return -1;
    const Py_ssize_t na = PySequence_Fast_GET_SIZE(acts);
    if (na != n_robots || n_robots != A) {
        Py_DECREF(acts);
        PyErr_SetString(PyExc_ValueError, "The number of actions must match the number of robots.");
        return -1;
    }
    for (Py_ssize_t i = 0; i < na; i++) {
        PyObject* pr = PySequence_Fast(PySequence_Fast_GET_ITEM(acts, i), "each action must be a (move, op) pair");
        if (!pr) {
            Py_DECREF(acts);
            return -1;
        }
        if (PySequence_Fast_GET_SIZE(pr) != 2) {
            Py_DECREF(pr);
            Py_DECREF(acts);
            PyErr_SetString(PyExc_ValueError, "each action must be a (move, op) pair");
            return -1;
        }
        row[i] = (uint8_t)(move_code(PySequence_Fast_GET_ITEM(pr, 0)) | (op_code(PySequence_Fast_GET_ITEM(pr, 1)) << 3));
        Py_DECREF(pr);
    }
    Py_DECREF(acts);
    return 0;
}

static int encode_row(const MailCtx* c, int w, PyObject* actions, int n_robots) {
    return encode_into(c->codes + (size_t)w * c->A, c->A, actions, n_robots);
}

/* encode(actions, n_robots) -> bytes: the mailbox's codes of one env's actions (host only; the
 * tests hold it against compat.encode_actions) */
static PyObject* encode(PyObject* self, PyObject* args) {
    PyObject* actions;
    int n_robots;
    (void)self;
    if (!PyArg_ParseTuple(args, "Oi", &actions, &n_robots)) return NULL;
    if (n_robots < 0 || n_robots > 64) {
        PyErr_SetString(PyExc_ValueError, "0..64 robots");
        return NULL;
    }
    uint8_t row[64];
    if (encode_into(row, n_robots, actions, n_robots)) return NULL;
    return PyBytes_FromStringAndSize((const char*)row, n_robots);
}

/* row w's results: (state dict, r_env float, rterms int, done bool, t int, total float, robot rows bytes,
 * package rows bytes) */
static PyObject* row_result(const MailCtx* c, int w, PyObject* grid) {
    PyObject* st = state_dict(c, w, grid);
    if (!st) return NULL;
    return Py_BuildValue("(NdiOidy#y#)", st, c->r_env[w], (int)c->rterms[w], c->done[w] ? Py_True : Py_False,
                         (int)c->t[w], c->total[w], (const char*)(c->robots + (size_t)w * c->A * 3),
                         (Py_ssize_t)(12 * c->A), (const char*)(c->pkgs + (size_t)w * c->P * 8),
                         (Py_ssize_t)(32 * c->P));
}

/* env_step(ctx, stream, actions, n_robots, idx (-1: the engine's only env), grid) -> row_result
 * compat.Environment.step's engine part: the actions' codes into the mailbox, mdl_mail_step, then
 * the new state dict and the env's rows from the mailbox. */
static PyObject* env_step(PyObject* self, PyObject* args) {
    PyObject *cap, *actions, *grid;
    unsigned long long stream;
    int n_robots, idx;
    (void)self;
    if (!PyArg_ParseTuple(args, "OKOiiO", &cap, &stream, &actions, &n_robots, &idx, &grid)) return NULL;
    MailCtx* c = (MailCtx*)PyCapsule_GetPointer(cap, "mdl.mailctx");
    if (!c) return NULL;
    if (encode_row(c, 0, actions, n_robots)) return NULL;
    if (idx >= 0) c->ids[0] = idx;
    int rc;
    rc = c->step(c->eng, 1, idx >= 0 ? 1 : 0, 0, (void*)(uintptr_t)stream);
    if (rc) return lib_error("mdl_mail_step");
    return row_result(c, 0, grid);
}

/* vec_step(ctx, stream, actions_per_row, n_robots, ids (None: rows are envs 0..n-1), grid)
 *   -> [row_result, ...]: one mdl_mail_step over n distinct envs (compat.VectorizedEnv.step's rounds) */
static PyObject* vec_step(PyObject* self, PyObject* args) {
    PyObject *cap, *rows, *ids, *grid;
    unsigned long long stream;
    int n_robots;
    (void)self;
    if (!PyArg_ParseTuple(args, "OKOiOO", &cap, &stream, &rows, &n_robots, &ids, &grid)) return NULL;
    MailCtx* c = (MailCtx*)PyCapsule_GetPointer(cap, "mdl.mailctx");
    if (!c) return NULL;
    PyObject* rs = PySequence_Fast(rows, "actions must be a sequence");
    if (!rs) return NULL;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(rs);
    PyObject* out = NULL;
    for (Py_ssize_t w = 0; w < n; w++)
        if (encode_row(c, (int)w, PySequence_Fast_GET_ITEM(rs, w), n_robots)) goto done;
    const int use_ids = ids != Py_None;
    if (use_ids) {
        PyObject* is = PySequence_Fast(ids, "ids must be a sequence");
        if (!is) goto done;
        if (PySequence_Fast_GET_SIZE(is) != n) {
            Py_DECREF(is);
            PyErr_SetString(PyExc_ValueError, "one id per action row");
            goto done;
        }
        for (Py_ssize_t w = 0; w < n; w++) {
            const long e = PyLong_AsLong(PySequence_Fast_GET_ITEM(is, w));
            if (e == -1 && PyErr_Occurred()) {
                Py_DECREF(is);
                goto done;
            }
            c->ids[w] = (int32_t)e;
        }
        Py_DECREF(is);
    }
    int rc;
    rc = c->step(c->eng, (int32_t)n, use_ids, 0, (void*)(uintptr_t)stream);
    if (rc) {
        lib_error("mdl_mail_step");
        goto done;
    }
    out = PyList_New(n);
    if (!out) goto done;
    for (Py_ssize_t w = 0; w < n; w++) {
        PyObject* r = row_result(c, (int)w, grid);
        if (!r) {
            Py_CLEAR(out);
            goto done;
        }
        PyList_SET_ITEM(out, w, r);
    }
done:
    Py_DECREF(rs);
    return out;
}

static PyMethodDef methods[] = {
    {"pack_view", pack_view, METH_VARARGS, "Pack a state view record into host memory; returns words written."},
    {"pack_robots", pack_robots, METH_VARARGS, "Pack a [t, A, robots] record into host memory."},
    {"bind", bind, METH_VARARGS, "Bind the engine's self-publishing helper entry points."},
    {"features", features, METH_VARARGS, "One helper featurizer call: pack, launch, wait, numpy outputs."},
    {"shaped", shaped, METH_VARARGS, "One compute_shaped_rewards call: pack, launch, wait, numpy.float32."},
    {"mail_ctx", mail_ctx, METH_VARARGS, "The mailbox addresses of an engine, for env_step."},
    {"env_step", env_step, METH_VARARGS, "Environment.step's engine part in one call."},
    {"vec_step", vec_step, METH_VARARGS, "One VectorizedEnv.step round's engine part in one call."},
    {"encode", encode, METH_VARARGS, "The action codes of one env's actions (host only)."},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_mdl_pack", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__mdl_pack(void) {
    import_array();
    s_in_transit = PyUnicode_InternFromString("in_transit");
    k_id = PyUnicode_InternFromString("id");
    k_status = PyUnicode_InternFromString("status");
    k_start_pos = PyUnicode_InternFromString("start_pos");
    k_target_pos = PyUnicode_InternFromString("target_pos");
    k_start_time = PyUnicode_InternFromString("start_time");
    k_deadline = PyUnicode_InternFromString("deadline");
    if (!s_in_transit || !k_id || !k_status || !k_start_pos || !k_target_pos || !k_start_time || !k_deadline)
        return NULL;
    return PyModule_Create(&module);
}
