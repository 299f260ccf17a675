"""IDQ / qmix featurizers and IDQ reward shaping on the device.

Drop-ins for ``IDQ/networks.py`` / ``qmix/networks.py``:
  convert_state(state, persistent_packages, current_robot_idx)            IDQ/networks.py:112-217
                                                                          (== qmix/networks.py:243-348)
  convert_global_state_to_tensor(state_dict, persistent_packages, shape)  qmix/networks.py:350-468
  reward_shaping(prev_state, cur_state, actions, packages_before, n)      IDQ/networks.py:228-349
All three run as gfx950 kernels (``mdl_views_alt_features`` / ``mdl_views_idq_reward``);
the batched form over an engine's envs is ``BatchedEnv.build_obs_alt``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib, stream_handle
from .helper import _engine_for, _layout, _tracker_rows, _xfer, pack_view

OP_NO_MATCH = 255   # a string op: the reference compares it with the ints 1 / 2 and never matches


def _alt(state, persistent_packages, agent_indices, shape, want):
    """One upload (views, offsets, agent indices), the kernel, one download -> numpy."""
    grid = state["map"]
    eng = _engine_for(grid)
    H, W = len(grid), len(grid[0])
    rows = _tracker_rows(persistent_packages)
    view = pack_view(state["time_step"], state["robots"], rows, H, W)
    n = len(agent_indices)
    x = _xfer(eng)
    (o_v, o_o, o_i), nin = _layout([(view.size * n, 1), (2 * n, 2), (n, 1)])
    words = np.zeros(nin, np.int32)
    words[o_v:o_v + view.size * n] = np.tile(view, n)
    words[o_o:o_o + 2 * n] = (np.arange(n, dtype=np.int64) * view.size).view(np.int32)
    words[o_i:o_i + n] = np.asarray(agent_indices, np.int32)
    b = x.up(words).data_ptr()
    oh, ow = (shape[1], shape[2]) if shape is not None else (H, W)
    names = [k for k in ("idq", "qmix") if k in want]
    sizes = {"idq": 6 * H * W, "qmix": 7 * oh * ow}
    offs, nout = _layout([(n * sizes[k], 4) for k in names])
    dout = x.out(nout)
    ptrs = {k: dout.data_ptr() + 4 * o for k, o in zip(names, offs)}
    check(lib().mdl_views_alt_features(eng._h, b + 4 * o_v, b + 4 * o_o, n, int(rows.shape[0]), b + 4 * o_i,
                                       ptrs.get("idq"), ptrs.get("qmix"), int(oh), int(ow),
                                       C.c_void_p(stream_handle())), "mdl_views_alt_features")
    host = x.down(nout)
    shapes = {"idq": (n, 6, H, W), "qmix": (n, 7, oh, ow)}
    res = {k: host[o:o + n * sizes[k]].reshape(shapes[k]) for k, o in zip(names, offs)}
    return res.get("idq"), res.get("qmix")


def convert_state(state, persistent_packages, current_robot_idx):
    """IDQ/networks.py:112-217 (qmix/networks.py:243-348): float32 [6, H, W]."""
    idq, _ = _alt(state, persistent_packages, [int(current_robot_idx)], None, ("idq",))
    return idq[0]


def convert_global_state_to_tensor(state_dict, persistent_packages, state_tensor_shape):
    """qmix/networks.py:350-468: float32 state_tensor_shape (channels beyond the 7 defined stay zero)."""
    nc, oh, ow = (int(x) for x in state_tensor_shape)
    _, qst = _alt(state_dict, persistent_packages, [0], (7, oh, ow), ("qmix",))
    q = qst[0]
    out = np.zeros((nc, oh, ow), np.float32)
    out[:min(nc, 7)] = q[:min(nc, 7)]
    return out


def reward_shaping(prev_env_state, current_env_state, actions_taken, persistent_packages_before_action, num_agents):
    """IDQ/networks.py:228-349 -> list of per-agent rewards.  String package ops (what
    IDQ/trainer.py passes) never equal the ints 1 / 2, exactly as in the reference."""
    prev_r = list(prev_env_state["robots"])[:num_agents]
    cur_r = list(current_env_state["robots"])[:num_agents]
    t_cur = int(current_env_state["time_step"])
    t_prev = int(prev_env_state.get("time_step", t_cur - 1))
    H = max([r[0] for r in prev_r + cur_r] + [1])
    W = max([r[1] for r in prev_r + cur_r] + [1])
    rows = _tracker_rows(persistent_packages_before_action)
    if rows.size:
        H = max(H, int(rows[:, [2, 4]].max()) + 1)
        W = max(W, int(rows[:, [3, 5]].max()) + 1)
    grid = prev_env_state.get("map")
    if grid is None:
        grid = np.zeros((H, W), np.uint8)
    eng = _engine_for(grid)
    Hm, Wm = len(grid), len(grid[0])
    prev = pack_view(t_prev, prev_r, rows, Hm, Wm)
    cr = np.asarray(cur_r, np.int64).reshape(-1, 3).copy()
    cr[:, :2] -= 1
    cur = np.concatenate([[t_cur, cr.shape[0]], cr.reshape(-1)]).astype(np.int32)
    ops = np.array([int(a[1]) if isinstance(a[1], (int, np.integer)) and not isinstance(a[1], bool)
                    and 0 <= int(a[1]) < 255 else OP_NO_MATCH for a in actions_taken[:num_agents]], np.uint8)
    x = _xfer(eng)
    ow_ = (ops.size + 3) // 4
    (o_p, o_c, o_a, o_off), nin = _layout([(prev.size, 1), (cur.size, 1), (ow_, 1), (6, 2)])
    words = np.zeros(nin, np.int32)
    words[o_p:o_p + prev.size] = prev
    words[o_c:o_c + cur.size] = cur
    ab = np.zeros(4 * ow_, np.uint8)
    ab[:ops.size] = ops
    words[o_a:o_a + ow_] = ab.view(np.int32)
    b = x.up(words).data_ptr()
    out = x.out(2 * num_agents + 2)
    o64 = (out.data_ptr() + 7) // 8 * 8   # f64 outputs, 8-B aligned in the float buffer
    check(lib().mdl_views_idq_reward(eng._h, b + 4 * o_p, b + 4 * o_off, int(rows.shape[0]), b + 4 * o_c,
                                     b + 4 * o_off, b + 4 * o_a, b + 4 * o_off, 1, 1, o64,
                                     C.c_void_p(stream_handle())), "mdl_views_idq_reward")
    host = x.down(2 * num_agents + 2)
    sh = (o64 - out.data_ptr()) // 4
    return [float(v) for v in host[sh:sh + 2 * num_agents].view(np.float64)]
