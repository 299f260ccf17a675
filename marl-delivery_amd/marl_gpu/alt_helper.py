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
import torch

from ._lib import check, lib, ptr, stream_handle
from .helper import _engine_for, _tracker_rows, _upload, pack_view

OP_NO_MATCH = 255   # a string op: the reference compares it with the ints 1 / 2 and never matches


def _alt(state, persistent_packages, agent_indices, shape, want):
    grid = state["map"]
    eng = _engine_for(grid)
    H, W = len(grid), len(grid[0])
    rows = _tracker_rows(persistent_packages)
    view = pack_view(state["time_step"], state["robots"], rows, H, W)
    n = len(agent_indices)
    views, offs = _upload([view] * n)
    idx = torch.as_tensor(np.asarray(agent_indices, np.int32)).cuda()
    oh, ow = (shape[1], shape[2]) if shape is not None else (H, W)
    idq = torch.empty((n, 6, H, W), dtype=torch.float32, device=views.device) if "idq" in want else None
    qst = torch.empty((n, 7, oh, ow), dtype=torch.float32, device=views.device) if "qmix" in want else None
    check(lib().mdl_views_alt_features(eng._h, ptr(views), ptr(offs), n, int(rows.shape[0]), ptr(idx), ptr(idq),
                                       ptr(qst), int(oh), int(ow), C.c_void_p(stream_handle())),
          "mdl_views_alt_features")
    return idq, qst


def convert_state(state, persistent_packages, current_robot_idx):
    """IDQ/networks.py:112-217 (qmix/networks.py:243-348): float32 [6, H, W]."""
    idq, _ = _alt(state, persistent_packages, [int(current_robot_idx)], None, ("idq",))
    return idq[0].cpu().numpy()


def convert_global_state_to_tensor(state_dict, persistent_packages, state_tensor_shape):
    """qmix/networks.py:350-468: float32 state_tensor_shape (channels beyond the 7 defined stay zero)."""
    nc, oh, ow = (int(x) for x in state_tensor_shape)
    _, qst = _alt(state_dict, persistent_packages, [0], (7, oh, ow), ("qmix",))
    q = qst[0].cpu().numpy()
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
    pv, po = _upload([prev])
    cv, co = _upload([cur])
    opt = torch.from_numpy(ops).cuda()
    oo = torch.zeros(1, dtype=torch.int64, device=opt.device)
    out = torch.empty(num_agents, dtype=torch.float64, device=opt.device)
    check(lib().mdl_views_idq_reward(eng._h, ptr(pv), ptr(po), int(rows.shape[0]), ptr(cv), ptr(co), ptr(opt),
                                     ptr(oo), 1, 1, ptr(out), C.c_void_p(stream_handle())), "mdl_views_idq_reward")
    return [float(x) for x in out.cpu().numpy()]
