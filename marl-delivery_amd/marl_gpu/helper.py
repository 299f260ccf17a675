"""Helper-compatible featurizers / shaping on state dicts, run on the GPU.

Same signatures and outputs as MAPPO/helper.py (and QMIX/helper.py, which
differs only in the shaping constants and the missing defaults of
generate_vector_features):

  convert_observation(state, tracker, idx)                         -> f32[6,H,W]   MAPPO/helper.py:6-66
  generate_vector_features(state, tracker, idx, T, MO=100, MP=100) -> f32[D]       MAPPO/helper.py:68-165
  convert_global_state(state, tracker, T, MR=100, MPs=100)         -> (f32[4,H,W], f32[Dg])  :167-255
  compute_shaped_rewards(g, prev, cur, actions, tracker_prev, A)   -> np.float32   :257-369

Each call is one C call (_mdl_pack.features / .shaped): it packs the dict(s)
into the engine's view record format straight into the engine's host-mapped
arena, launches the same device code the batched engine uses
(mdl_host_views_features / mdl_host_views_shaped_reward: mdl_views_* reading
their inputs from and writing their outputs to that host memory, whose last
wave publishes a completion word), spins on that word and returns the numpy
result: one kernel launch, no copies, no stream synchronisation, no ctypes.
The launches go to a helper stream of the engine's own (nothing on the device
depends on them), so they never queue behind the caller's GPU work.
They exist for drop-in use and for the known-answer tests; batched training
should use BatchedEnv.build_obs instead.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _mdl_pack
from ._lib import check, lib, pack
from .engine import MAPPO_SHAPING, QMIX_SHAPING, BatchedEnv
from .compat import MOVE_CODES, OP_CODES, _code  # noqa: F401  (MOVE_CODES / OP_CODES re-exported)

_engines: dict = {}
_CONSTS: dict = {}   # shaping-constant tuples -> their C double[9]


_last_grid: list = [None, None]   # [grid object, _Arena] of the previous call


def _arena_for(grid) -> "_Arena":
    """The helper engine of a map, as its arena.  The reference's state dicts carry the env's own
    grid object (``state['map']`` aliases ``env.grid``, env.py:140), so the same object is
    recognised by identity first; any other grid is keyed by its contents."""
    if grid is _last_grid[0]:
        return _last_grid[1]
    g = np.asarray(grid, dtype=np.uint8)
    key = (g.shape, g.tobytes())
    eng = _engines.get(key)
    if eng is None:
        eng = BatchedEnv(g, 1, 1, 1, 2, tracker="fresh")
        _engines[key] = eng
    ar = _arena(eng)
    _last_grid[0], _last_grid[1] = grid, ar
    return ar


def _engine_for(grid) -> BatchedEnv:
    return _arena_for(grid).eng


class _Arena:
    """The engine's host-mapped arena (mdl_host_arena) as one numpy byte view; grows on demand
    (every call has finished with it on return: the helper calls are synchronous).  ``h`` /
    ``stream``: the engine handle and its helper stream, as integers for the C calls."""

    def __init__(self, eng):
        import torch
        pack()
        self.eng = eng
        self.cap = 0
        self.addr = 0
        self.u8 = None
        L = lib()
        self._views, self._wait = L.mdl_host_views_features, L.mdl_host_wait
        self._dev = eng.device.index
        self._stream_obj = torch.cuda.Stream(device=eng.device)
        self.stream = int(self._stream_obj.cuda_stream)
        self.h = int(eng._h.value if isinstance(eng._h, C.c_void_p) else eng._h)
        self.hw = tuple(int(x) for x in eng.grids[0].shape)
        self.get(1)

    def get(self, nbytes):
        if nbytes > self.cap:
            p = C.c_void_p()
            check(lib().mdl_host_arena(self.eng._h, int(nbytes), C.byref(p)), "mdl_host_arena")
            cap = 64 * 1024
            while cap < nbytes:
                cap *= 2
            self.cap, self.addr = cap, p.value
            self.u8 = np.ctypeslib.as_array((C.c_uint8 * cap).from_address(p.value))
        return self.u8

    def wait(self):
        rc = self._wait(self.eng._h, self.stream)
        if rc:
            check(rc, "mdl_host_wait")


def _arena(eng) -> _Arena:
    a = eng.__dict__.get("_arena")
    if a is None:
        a = eng._arena = _Arena(eng)
    return a


def _tracker_rows(tracker: dict) -> np.ndarray:
    rows = np.zeros((len(tracker), 8), np.int32)
    for k, v in enumerate(tracker.values()):
        rows[k] = (v["id"], 2 if v["status"] == "in_transit" else 1, v["start_pos"][0], v["start_pos"][1],
                   v["target_pos"][0], v["target_pos"][1], v["start_time"], v["deadline"])
    return rows


def pack_view(t, robots1, tracker_rows, H, W, map_index=0) -> np.ndarray:
    """[t, A, n, map] + A*(r, c, carry) (0-indexed) + n*(id, status, sr, sc, tr, tc, st, dl)."""
    rows = tracker_rows if isinstance(tracker_rows, dict) else np.asarray(tracker_rows, np.int64).reshape(-1, 8).tolist()
    n = 4 + 3 * len(robots1) + 8 * len(rows)
    out = np.zeros(n, np.int32)
    _mdl_pack.pack_view(out.ctypes.data, n, int(t), robots1, rows, H, W, map_index)
    return out


def _align(x, a=16):
    return (x + a - 1) // a * a


_OUT_NAMES = ("obs", "vec", "gmap", "gvec")
_layouts: dict = {}


def _features_layout(H, W, A, ns, n, MO, MP, MR, MPs, want):
    """Byte offsets in the arena of one features call: view record, int64 offsets, agent
    indices, then each wanted output (cached per shape)."""
    key = (H, W, A, ns, n, MO, MP, MR, MPs, want)
    lay = _layouts.get(key)
    if lay is None:
        sizes = {"obs": 6 * H * W, "vec": 6 + 5 * MO + 5 * MP + 1, "gmap": 4 * H * W, "gvec": 6 * MR + 7 * MPs + 1}
        shapes = {"obs": (n, 6, H, W), "vec": (n, sizes["vec"]), "gmap": (n, 4, H, W), "gvec": (n, sizes["gvec"])}
        vw = 4 + 3 * A + 8 * ns
        o_off = _align(4 * vw)                      # int64 offsets (all 0: one shared record)
        o_idx = _align(o_off + 8 * n)
        pos = _align(o_idx + 4 * n)
        outs = {}
        for k in _OUT_NAMES:
            if k in want:
                outs[k] = (pos, 4 * n * sizes[k], shapes[k])
                pos = _align(pos + 4 * n * sizes[k])
        lay = _layouts[key] = (vw, o_off, o_idx, pos, outs,
                               tuple(outs[k][0] if k in outs else None for k in _OUT_NAMES))
    return lay


def _one(state, tracker, idx, T, MO, MP, MR, MPs, want):
    """One view (one C call): the outputs named by the bits of ``want`` (1 obs, 2 vec, 4 gmap, 8 gvec)."""
    grid = state["map"]
    ar = _last_grid[1] if grid is _last_grid[0] else _arena_for(grid)
    H, W = ar.hw
    T = int(T)
    r = _mdl_pack.features(ar.h, ar.stream, ar.addr, ar.cap, state["time_step"], state["robots"], tracker, H, W, idx,
                           T, MO, MP, MR, MPs, want)
    if r.__class__ is int:   # the arena is too small for this call: grow it, once
        ar.get(r)
        r = _mdl_pack.features(ar.h, ar.stream, ar.addr, ar.cap, state["time_step"], state["robots"], tracker, H, W,
                               idx, T, MO, MP, MR, MPs, want)
    return r


def features(state, tracker, agent_indices, T, MO, MP, MR, MPs, want=("obs", "vec", "gmap", "gvec")):
    """Batched helper entry: one view per agent index (same state / tracker: one record that
    every view's offset points at).  ``tracker``: the reference's tracker dict (insertion order)
    or rows (id, status 1|2, sr, sc, tr, tc, start_time, deadline)."""
    grid = state["map"]
    ar = _arena_for(grid)
    eng = ar.eng
    H, W = ar.hw
    if not isinstance(tracker, dict):
        tracker = np.asarray(tracker, np.int64).reshape(-1, 8).tolist()
    robots = state["robots"]
    ns = len(tracker)
    n = len(agent_indices)
    vw, o_off, o_idx, nbytes, outs, o_ptr = _features_layout(H, W, len(robots), ns, n, MO, MP, MR, MPs, tuple(want))
    u8 = ar.get(nbytes)
    base = ar.addr
    _mdl_pack.pack_view(base, vw, int(state["time_step"]), robots, tracker, H, W, 0)
    u8[o_off:o_off + 8 * n] = 0
    u8[o_idx:o_idx + 4 * n].view(np.int32)[:] = agent_indices
    rc = ar._views(eng._h, base, base + o_off, n, ns, base + o_idx, int(T), MO, MP, MR, MPs,
                   None if o_ptr[0] is None else base + o_ptr[0], None if o_ptr[1] is None else base + o_ptr[1],
                   None if o_ptr[2] is None else base + o_ptr[2], None if o_ptr[3] is None else base + o_ptr[3],
                   ar.stream)
    if rc:
        check(rc, "mdl_host_views_features")
    return {k: u8[o:o + nb].view(np.float32).reshape(shape).copy() for k, (o, nb, shape) in outs.items()}


def convert_observation(env_state_dict, persistent_packages_for_env, current_robot_idx):
    return _one(env_state_dict, persistent_packages_for_env, current_robot_idx, 0, 0, 0, 0, 0, 1)[0]


def generate_vector_features(env_state_dict, persistent_packages_for_env, current_robot_idx, max_time_steps,
                             max_other_robots_to_observe=100, max_packages_to_observe=100):
    return _one(env_state_dict, persistent_packages_for_env, current_robot_idx, max_time_steps,
                max_other_robots_to_observe, max_packages_to_observe, 0, 0, 2)[0]


def convert_global_state(env_state_dict, persistent_packages_for_env, max_time_steps, max_robots_in_state=100,
                         max_packages_in_state=100):
    return _one(env_state_dict, persistent_packages_for_env, 0, max_time_steps, 0, 0, max_robots_in_state,
                max_packages_in_state, 12)


_last_consts: list = [None, 0]   # [constants tuple, address of its C double[9]] of the previous call


def _consts_addr(consts):
    """Address of a C double[9] holding ``consts`` (0: the engine's own); cached per tuple."""
    if consts is None:
        return 0
    if consts is _last_consts[0]:
        return _last_consts[1]
    ck = tuple(consts)
    cs = _CONSTS.get(ck)
    if cs is None:
        cs = _CONSTS[ck] = (C.c_double * 9)(*[float(v) for v in ck])
    a = C.addressof(cs)
    if isinstance(consts, tuple):   # immutable: safe to recognise by identity next time
        _last_consts[0], _last_consts[1] = consts, a
    return a


def _shaped(ar, g, prev_t, prev_robots1, cur_t, cur_robots1, actions, num_agents, tracker, consts):
    """One transition (one C call).  ``actions``: (move, op) pairs, or MDL_ACTION_CODES bytes."""
    H, W = ar.hw
    ca = _consts_addr(consts)
    r = _mdl_pack.shaped(ar.h, ar.stream, ar.addr, ar.cap, g, prev_t, prev_robots1, cur_t, cur_robots1, actions,
                         num_agents, tracker, H, W, ca)
    if r.__class__ is int:   # the arena is too small for this call: grow it, once
        ar.get(r)
        r = _mdl_pack.shaped(ar.h, ar.stream, ar.addr, ar.cap, g, prev_t, prev_robots1, cur_t, cur_robots1, actions,
                             num_agents, tracker, H, W, ca)
    return r


def shaped_rewards_views(g, prev_t, prev_robots1, cur_t, cur_robots1, action_codes, tracker, grid,
                         consts=MAPPO_SHAPING):
    """Raw entry for compute_shaped_rewards: one transition; ``action_codes``: MDL_ACTION_CODES
    bytes (move | op << 3); ``tracker``: the tracker dict of the previous state (insertion order)
    or its rows."""
    return _shaped(_arena_for(grid), float(g), int(prev_t), prev_robots1, int(cur_t), cur_robots1,
                   bytes(action_codes), len(prev_robots1), tracker, consts)


def compute_shaped_rewards(global_reward, prev_env_state_dict, current_env_state_dict, actions_taken_for_all_agents,
                           persistent_packages_at_prev_state, num_agents, consts=MAPPO_SHAPING, grid=None):
    """MAPPO/helper.py:257-369 (pass consts=QMIX_SHAPING for QMIX/helper.py:257-368).

    The state dicts need no 'map' key (the notebook KAT omits it); ``grid``
    defaults to a map large enough for the coordinates used."""
    if grid is None:
        grid = prev_env_state_dict.get("map")
    if grid is None:
        trk = persistent_packages_at_prev_state
        prev_r = list(prev_env_state_dict["robots"])[:num_agents]
        cur_r = list(current_env_state_dict["robots"])[:num_agents]
        rows = _tracker_rows(trk) if isinstance(trk, dict) else np.asarray(trk).reshape(-1, 8)
        coords = [x for r in prev_r + cur_r for x in r[:2]]
        coords += [int(v) + 1 for row in rows for v in row[2:6]]
        n = max(coords + [2])
        grid = [[0] * n for _ in range(n)]
    ar = _last_grid[1] if grid is _last_grid[0] else _arena_for(grid)
    return _shaped(ar, global_reward, prev_env_state_dict["time_step"], prev_env_state_dict["robots"],
                   current_env_state_dict["time_step"], current_env_state_dict["robots"],
                   actions_taken_for_all_agents, num_agents, persistent_packages_at_prev_state, consts)


__all__ = ["convert_observation", "generate_vector_features", "convert_global_state", "compute_shaped_rewards",
           "MAPPO_SHAPING", "QMIX_SHAPING", "features", "pack_view"]
