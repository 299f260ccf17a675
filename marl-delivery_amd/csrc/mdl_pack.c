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
 * Host plumbing only (no GPU code, no reference semantics beyond the record layout).  The tracker
 * dict is read in insertion order (PyDict_Next), the order the reference iterates
 * persistent_packages.values() in (MAPPO/trainer.py:95-130); 'status' == 'in_transit' -> 2, else 1.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

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

/* pack_view(addr, cap_words, t, robots, tracker, H, W, map_index) -> words written.
 * robots: sequence of (row, col, carrying) 1-indexed; tracker: dict id -> entry dict in insertion order
 * (MAPPO/trainer.py:95-130 layout), or a sequence of rows (id, status, sr, sc, tr, tc, st, dl). */
static PyObject* pack_view(PyObject* self, PyObject* args) {
    unsigned long long addr;
    Py_ssize_t cap;
    long t, H, W, map_index;
    PyObject *robots, *tracker;
    (void)self;
    if (!PyArg_ParseTuple(args, "KnlOOlll", &addr, &cap, &t, &robots, &tracker, &H, &W, &map_index)) return NULL;
    int32_t* w = (int32_t*)(uintptr_t)addr;
    PyObject* rs = PySequence_Fast(robots, "robots must be a sequence");
    if (!rs) return NULL;
    const Py_ssize_t A = PySequence_Fast_GET_SIZE(rs);
    const int is_dict = PyDict_Check(tracker);
    PyObject* ts = NULL;
    Py_ssize_t n;
    if (is_dict) {
        n = PyDict_Size(tracker);
    } else {
        ts = PySequence_Fast(tracker, "tracker must be a dict or a sequence of rows");
        if (!ts) {
            Py_DECREF(rs);
            return NULL;
        }
        n = PySequence_Fast_GET_SIZE(ts);
    }
    PyObject* ret = NULL;
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
    ret = PyLong_FromSsize_t(4 + 3 * A + 8 * n);
done:
    Py_DECREF(rs);
    Py_XDECREF(ts);
    return ret;
}

/* pack_robots(addr, cap_words, t, robots) -> words: [t, A] + A x (row, col, carrying) 0-indexed
 * (the "current state" record of mdl_views_shaped_reward). */
static PyObject* pack_robots(PyObject* self, PyObject* args) {
    unsigned long long addr;
    Py_ssize_t cap;
    long t;
    PyObject* robots;
    (void)self;
    if (!PyArg_ParseTuple(args, "KnlO", &addr, &cap, &t, &robots)) return NULL;
    PyObject* rs = PySequence_Fast(robots, "robots must be a sequence");
    if (!rs) return NULL;
    const Py_ssize_t A = PySequence_Fast_GET_SIZE(rs);
    if (2 + 3 * A > cap) {
        Py_DECREF(rs);
        PyErr_SetString(PyExc_ValueError, "record larger than the arena");
        return NULL;
    }
    int32_t* w = (int32_t*)(uintptr_t)addr;
    w[0] = (int32_t)t;
    w[1] = (int32_t)A;
    for (Py_ssize_t i = 0; i < A; i++) {
        long r, c, cy;
        PyObject* rb = PySequence_Fast_GET_ITEM(rs, i);
        if (seq_int(rb, 0, &r) || seq_int(rb, 1, &c) || seq_int(rb, 2, &cy)) {
            Py_DECREF(rs);
            return NULL;
        }
        w[2 + 3 * i] = (int32_t)(r - 1);
        w[3 + 3 * i] = (int32_t)(c - 1);
        w[4 + 3 * i] = (int32_t)cy;
    }
    Py_DECREF(rs);
    return PyLong_FromSsize_t(2 + 3 * A);
}

static PyMethodDef methods[] = {
    {"pack_view", pack_view, METH_VARARGS, "Pack a state view record into host memory; returns words written."},
    {"pack_robots", pack_robots, METH_VARARGS, "Pack a [t, A, robots] record into host memory."},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_mdl_pack", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__mdl_pack(void) {
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
