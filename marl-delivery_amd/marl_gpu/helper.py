"""Helper-compatible featurizers / shaping on state dicts, run on the GPU.

Same signatures and outputs as MAPPO/helper.py (and QMIX/helper.py, which
differs only in the shaping constants and the missing defaults of
generate_vector_features):

  convert_observation(state, tracker, idx)                         -> f32[6,H,W]   MAPPO/helper.py:6-66
  generate_vector_features(state, tracker, idx, T, MO=100, MP=100) -> f32[D]       MAPPO/helper.py:68-165
  convert_global_state(state, tracker, T, MR=100, MPs=100)         -> (f32[4,H,W], f32[Dg])  :167-255
  compute_shaped_rewards(g, prev, cur, actions, tracker_prev, A)   -> np.float32   :257-369

Each call packs the dict(s) into the engine's view record format, uploads it,
and runs the same device code the batched engine uses (mdl_views_features /
mdl_views_shaped_reward).  They exist for drop-in use and for the known-answer
tests; batched training should use BatchedEnv.build_obs instead.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from ._lib import check, lib, stream_handle
from .engine import MAPPO_SHAPING, QMIX_SHAPING, BatchedEnv
from .compat import MOVE_CODES, OP_CODES

_engines: dict = {}


def _engine_for(grid) -> BatchedEnv:
    g = np.asarray(grid, dtype=np.uint8)
    key = (g.shape, g.tobytes())
    eng = _engines.get(key)
    if eng is None:
        eng = BatchedEnv(g, 1, 1, 1, 2, tracker="fresh")
        _engines[key] = eng
    return eng


def _tracker_rows(tracker: dict) -> np.ndarray:
    rows = np.zeros((len(tracker), 8), np.int32)
    for k, v in enumerate(tracker.values()):
        rows[k] = (v["id"], 2 if v["status"] == "in_transit" else 1, v["start_pos"][0], v["start_pos"][1],
                   v["target_pos"][0], v["target_pos"][1], v["start_time"], v["deadline"])
    return rows


def pack_view(t, robots1, tracker_rows, H, W, map_index=0) -> np.ndarray:
    """[t, A, n, map] + A*(r, c, carry) (0-indexed) + n*(id, status, sr, sc, tr, tc, st, dl)."""
    rb = np.asarray(robots1, dtype=np.int64).reshape(-1, 3).copy()
    rb[:, :2] -= 1
    rows = np.asarray(tracker_rows, dtype=np.int64).reshape(-1, 8)
    if rb.shape[0] > 64:
        raise ValueError("at most 64 robots per view")
    if ((rb[:, 0] < 0) | (rb[:, 0] >= H) | (rb[:, 1] < 0) | (rb[:, 1] >= W)).any():
        raise ValueError("robot positions must lie inside the map")
    if rows.size and ((rows[:, 2] < 0) | (rows[:, 2] >= H) | (rows[:, 4] < 0) | (rows[:, 4] >= H) |
                      (rows[:, 3] < 0) | (rows[:, 3] >= W) | (rows[:, 5] < 0) | (rows[:, 5] >= W)).any():
        raise ValueError("package cells must lie inside the map")
    if rows.size and ((rows[:, 6] < 0) | (rows[:, 6] > 65535) | (rows[:, 7] < 0) | (rows[:, 7] > 65535)).any():
        raise ValueError("start_time / deadline must fit 16 bits")
    head = np.array([t, rb.shape[0], rows.shape[0], map_index], np.int64)
    return np.concatenate([head, rb.reshape(-1), rows.reshape(-1)]).astype(np.int32)


class _Xfer:
    """Pinned staging of one helper call: the packed inputs go up in ONE host-to-device copy
    and every output comes back in ONE device-to-host copy, with one synchronisation (the
    buffers grow on demand and are reused: each call has retired its transfers on return)."""

    def __init__(self, device):
        self.device = device
        self.h_in = self.d_in = self.d_out = self.h_out = None

    @staticmethod
    def _grow(n):
        return 1 << max(10, (int(n) - 1).bit_length())

    def up(self, words: np.ndarray) -> torch.Tensor:
        n = words.size
        if self.h_in is None or self.h_in.numel() < n:
            m = self._grow(n)
            self.h_in = torch.empty(m, dtype=torch.int32, pin_memory=True)
            self.d_in = torch.empty(m, dtype=torch.int32, device=self.device)
        self.h_in.numpy()[:n] = words
        self.d_in[:n].copy_(self.h_in[:n], non_blocking=True)
        return self.d_in

    def out(self, n: int) -> torch.Tensor:
        if self.d_out is None or self.d_out.numel() < n:
            m = self._grow(n)
            self.d_out = torch.empty(m, dtype=torch.float32, device=self.device)
            self.h_out = torch.empty(m, dtype=torch.float32, pin_memory=True)
        return self.d_out

    def down(self, n: int) -> np.ndarray:
        self.h_out[:n].copy_(self.d_out[:n], non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return self.h_out.numpy()[:n].copy()


def _xfer(eng) -> _Xfer:
    x = eng.__dict__.get("_helper_xfer")
    if x is None:
        x = eng._helper_xfer = _Xfer(eng.device)
    return x


def _layout(parts):
    """Word offsets of consecutive parts, each starting at a multiple of its alignment (words)."""
    offs, pos = [], 0
    for size, align in parts:
        pos = (pos + align - 1) // align * align
        offs.append(pos)
        pos += size
    return offs, pos


def features(state, tracker_rows, agent_indices, T, MO, MP, MR, MPs, want=("obs", "vec", "gmap", "gvec")):
    """Batched helper entry: one view per agent index (same state / tracker)."""
    grid = state["map"]
    eng = _engine_for(grid)
    H, W = len(grid), len(grid[0])
    view = pack_view(state["time_step"], state["robots"], tracker_rows, H, W)
    n = len(agent_indices)
    x = _xfer(eng)
    # inputs: n copies of the view, their int64 offsets, the agent indices -- one upload
    (o_v, o_o, o_i), nin = _layout([(view.size * n, 1), (2 * n, 2), (n, 1)])
    words = np.zeros(nin, np.int32)
    words[o_v:o_v + view.size * n] = np.tile(view, n)
    words[o_o:o_o + 2 * n] = (np.arange(n, dtype=np.int64) * view.size).view(np.int32)
    words[o_i:o_i + n] = np.asarray(agent_indices, np.int32)
    din = x.up(words)
    base_in = din.data_ptr()
    # outputs: one float buffer, each output 16-B aligned -- one download
    sizes = {"obs": 6 * H * W, "vec": 6 + 5 * MO + 5 * MP + 1, "gmap": 4 * H * W, "gvec": 6 * MR + 7 * MPs + 1}
    names = [k for k in ("obs", "vec", "gmap", "gvec") if k in want]
    offs, nout = _layout([(n * sizes[k], 4) for k in names])
    dout = x.out(nout)
    ptrs = {k: dout.data_ptr() + 4 * o for k, o in zip(names, offs)}
    ns = int(np.asarray(tracker_rows).reshape(-1, 8).shape[0])
    check(lib().mdl_views_features(eng._h, base_in + 4 * o_v, base_in + 4 * o_o, n, ns, base_in + 4 * o_i, int(T),
                                   MO, MP, MR, MPs, ptrs.get("obs"), ptrs.get("vec"), ptrs.get("gmap"),
                                   ptrs.get("gvec"), C.c_void_p(stream_handle())), "mdl_views_features")
    host = x.down(nout)
    shapes = {"obs": (n, 6, H, W), "vec": (n, sizes["vec"]), "gmap": (n, 4, H, W), "gvec": (n, sizes["gvec"])}
    return {k: host[o:o + n * sizes[k]].reshape(shapes[k]) for k, o in zip(names, offs)}


def convert_observation(env_state_dict, persistent_packages_for_env, current_robot_idx):
    rows = _tracker_rows(persistent_packages_for_env)
    return features(env_state_dict, rows, [current_robot_idx], 0, 0, 0, 0, 0, want=("obs",))["obs"][0]


def generate_vector_features(env_state_dict, persistent_packages_for_env, current_robot_idx, max_time_steps,
                             max_other_robots_to_observe=100, max_packages_to_observe=100):
    rows = _tracker_rows(persistent_packages_for_env)
    return features(env_state_dict, rows, [current_robot_idx], max_time_steps, max_other_robots_to_observe,
                    max_packages_to_observe, 0, 0, want=("vec",))["vec"][0]


def convert_global_state(env_state_dict, persistent_packages_for_env, max_time_steps, max_robots_in_state=100,
                         max_packages_in_state=100):
    rows = _tracker_rows(persistent_packages_for_env)
    o = features(env_state_dict, rows, [0], max_time_steps, 0, 0, max_robots_in_state, max_packages_in_state,
                 want=("gmap", "gvec"))
    return o["gmap"][0], o["gvec"][0]


def shaped_rewards_views(g, prev_t, prev_robots1, cur_t, cur_robots1, action_codes, tracker_rows, grid,
                         consts=MAPPO_SHAPING):
    """Raw entry for compute_shaped_rewards: packed inputs, one or many transitions."""
    eng = _engine_for(grid)
    H, W = len(grid), len(grid[0])
    prev = pack_view(prev_t, prev_robots1, tracker_rows, H, W)
    cr = np.asarray(cur_robots1, np.int64).reshape(-1, 3).copy()
    cr[:, :2] -= 1
    cur = np.concatenate([[cur_t, cr.shape[0]], cr.reshape(-1)]).astype(np.int32)
    codes = np.asarray(action_codes, np.uint8).reshape(-1)
    cw = (codes.size + 3) // 4
    x = _xfer(eng)
    # one upload: prev view, cur view, action bytes, three int64 offsets (all 0), g (fp64)
    (o_p, o_c, o_a, o_off, o_g), nin = _layout([(prev.size, 1), (cur.size, 1), (cw, 1), (6, 2), (2, 2)])
    words = np.zeros(nin, np.int32)
    words[o_p:o_p + prev.size] = prev
    words[o_c:o_c + cur.size] = cur
    ab = np.zeros(4 * cw, np.uint8)
    ab[:codes.size] = codes
    words[o_a:o_a + cw] = ab.view(np.int32)
    words[o_g:o_g + 2] = np.array([float(g)], np.float64).view(np.int32)
    b = x.up(words).data_ptr()
    out = x.out(1)
    cs = (C.c_double * 9)(*[float(v) for v in consts])
    ns = int(np.asarray(tracker_rows).reshape(-1, 8).shape[0])
    check(lib().mdl_views_shaped_reward(eng._h, b + 4 * o_p, b + 4 * o_off, ns, b + 4 * o_c, b + 4 * o_off,
                                        b + 4 * o_a, b + 4 * o_off, b + 4 * o_g, 1, cs, out.data_ptr(),
                                        C.c_void_p(stream_handle())), "mdl_views_shaped_reward")
    return np.float32(x.down(1)[0])


def compute_shaped_rewards(global_reward, prev_env_state_dict, current_env_state_dict, actions_taken_for_all_agents,
                           persistent_packages_at_prev_state, num_agents, consts=MAPPO_SHAPING, grid=None):
    """MAPPO/helper.py:257-369 (pass consts=QMIX_SHAPING for QMIX/helper.py:257-368).

    The state dicts need no 'map' key (the notebook KAT omits it); ``grid``
    defaults to a map large enough for the coordinates used."""
    prev_r = list(prev_env_state_dict["robots"])[:num_agents]
    cur_r = list(current_env_state_dict["robots"])[:num_agents]
    codes = np.array([MOVE_CODES.get(m, 5) | (OP_CODES.get(o, 3) << 3)
                      for m, o in list(actions_taken_for_all_agents)[:num_agents]], np.uint8)
    rows = _tracker_rows(persistent_packages_at_prev_state)
    if grid is None:
        grid = prev_env_state_dict.get("map")
    if grid is None:
        coords = [x for r in prev_r + cur_r for x in r[:2]]
        coords += [int(v) + 1 for row in rows for v in row[2:6]]
        n = max(coords + [2])
        grid = [[0] * n for _ in range(n)]
    return shaped_rewards_views(global_reward, prev_env_state_dict["time_step"], prev_r,
                                current_env_state_dict["time_step"], cur_r, codes, rows, grid, consts)


__all__ = ["convert_observation", "generate_vector_features", "convert_global_state", "compute_shaped_rewards",
           "MAPPO_SHAPING", "QMIX_SHAPING", "features", "pack_view"]
