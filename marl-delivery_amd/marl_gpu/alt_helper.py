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

import numpy as np

from . import _mdl_pack
from ._lib import check, lib
from .helper import _align, _arena, _engine_for, _tracker_rows

OP_NO_MATCH = 255   # a string op: the reference compares it with the ints 1 / 2 and never matches


def _alt(state, persistent_packages, agent_indices, shape, want):
    """The view record packed into the engine's host-mapped arena, the kernel reading it there
    and writing its outputs there, one completion wait -> numpy (as marl_gpu.helper.features)."""
    grid = state["map"]
    eng = _engine_for(grid)
    H, W = len(grid), len(grid[0])
    robots = state["robots"]
    ns = len(persistent_packages)
    n = len(agent_indices)
    vw = 4 + 3 * len(robots) + 8 * ns
    oh, ow = (shape[1], shape[2]) if shape is not None else (H, W)
    names = [k for k in ("idq", "qmix") if k in want]
    sizes = {"idq": 6 * H * W, "qmix": 7 * oh * ow}
    o_off = _align(4 * vw)
    o_idx = _align(o_off + 8 * n)
    pos = _align(o_idx + 4 * n)
    o_out = {}
    for k in names:
        o_out[k] = pos
        pos = _align(pos + 4 * n * sizes[k])
    ar = _arena(eng)
    u8 = ar.get(pos)
    b = ar.addr
    _mdl_pack.pack_view(b, vw, int(state["time_step"]), robots, persistent_packages, H, W, 0)
    u8[o_off:o_off + 8 * n] = 0
    u8[o_idx:o_idx + 4 * n].view(np.int32)[:] = agent_indices
    check(lib().mdl_views_alt_features(eng._h, b, b + o_off, n, ns, b + o_idx,
                                       b + o_out["idq"] if "idq" in o_out else None,
                                       b + o_out["qmix"] if "qmix" in o_out else None, int(oh), int(ow),
                                       ar.stream), "mdl_views_alt_features")
    ar.wait()
    shapes = {"idq": (n, 6, H, W), "qmix": (n, 7, oh, ow)}
    res = {k: u8[o_out[k]:o_out[k] + 4 * n * sizes[k]].view(np.float32).reshape(shapes[k]).copy() for k in names}
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
    grid = prev_env_state.get("map")
    if grid is None:   # a map large enough for every coordinate used
        H = max([r[0] for r in prev_r + cur_r] + [1])
        W = max([r[1] for r in prev_r + cur_r] + [1])
        rows = _tracker_rows(persistent_packages_before_action)
        if rows.size:
            H = max(H, int(rows[:, [2, 4]].max()) + 1)
            W = max(W, int(rows[:, [3, 5]].max()) + 1)
        grid = np.zeros((H, W), np.uint8)
    eng = _engine_for(grid)
    Hm, Wm = len(grid), len(grid[0])
    ops = bytes(int(a[1]) if isinstance(a[1], (int, np.integer)) and not isinstance(a[1], bool)
                and 0 <= int(a[1]) < 255 else OP_NO_MATCH for a in actions_taken[:num_agents])
    ns = len(persistent_packages_before_action)
    vw = 4 + 3 * len(prev_r) + 8 * ns
    cw = 2 + 3 * len(cur_r)
    # arena: prev view | cur record | op bytes | three int64 offsets (0) | out (f64 per agent)
    o_c = _align(4 * vw)
    o_a = _align(o_c + 4 * cw)
    o_off = _align(o_a + len(ops))
    o_out = o_off + 32
    ar = _arena(eng)
    u8 = ar.get(o_out + 8 * max(1, num_agents) + 16)
    b = ar.addr
    _mdl_pack.pack_view(b, vw, t_prev, prev_r, persistent_packages_before_action, Hm, Wm, 0)
    _mdl_pack.pack_robots(b + o_c, cw, t_cur, cur_r)
    u8[o_a:o_a + len(ops)] = np.frombuffer(ops, np.uint8)
    u8[o_off:o_off + 32] = 0
    check(lib().mdl_views_idq_reward(eng._h, b, b + o_off, ns, b + o_c, b + o_off, b + o_a, b + o_off, 1, 1,
                                     b + o_out, ar.stream), "mdl_views_idq_reward")
    ar.wait()
    return [float(v) for v in u8[o_out:o_out + 8 * num_agents].view(np.float64)]
