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

from ._lib import check, lib, ptr, stream_handle
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


def _upload(blobs):
    offs = np.zeros(len(blobs), np.int64)
    pos = 0
    for i, b in enumerate(blobs):
        offs[i] = pos
        pos += b.size
    flat = np.concatenate(blobs) if blobs else np.zeros(1, np.int32)
    return torch.from_numpy(flat).cuda(), torch.from_numpy(offs).cuda()


def features(state, tracker_rows, agent_indices, T, MO, MP, MR, MPs, want=("obs", "vec", "gmap", "gvec")):
    """Batched helper entry: one view per agent index (same state / tracker)."""
    grid = state["map"]
    eng = _engine_for(grid)
    H, W = len(grid), len(grid[0])
    view = pack_view(state["time_step"], state["robots"], tracker_rows, H, W)
    n = len(agent_indices)
    views, offs = _upload([view] * n)
    idx = torch.as_tensor(np.asarray(agent_indices, np.int32)).cuda()
    dev = views.device
    out = {}
    if "obs" in want:
        out["obs"] = torch.empty((n, 6, H, W), dtype=torch.float32, device=dev)
    if "vec" in want:
        out["vec"] = torch.empty((n, 6 + 5 * MO + 5 * MP + 1), dtype=torch.float32, device=dev)
    if "gmap" in want:
        out["gmap"] = torch.empty((n, 4, H, W), dtype=torch.float32, device=dev)
    if "gvec" in want:
        out["gvec"] = torch.empty((n, 6 * MR + 7 * MPs + 1), dtype=torch.float32, device=dev)
    ns = int(np.asarray(tracker_rows).reshape(-1, 8).shape[0])
    check(lib().mdl_views_features(eng._h, ptr(views), ptr(offs), n, ns, ptr(idx), int(T), MO, MP, MR, MPs,
                                   ptr(out.get("obs")), ptr(out.get("vec")), ptr(out.get("gmap")),
                                   ptr(out.get("gvec")), C.c_void_p(stream_handle())), "mdl_views_features")
    return {k: v.cpu().numpy() for k, v in out.items()}


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
    pv, po = _upload([prev])
    cv, co = _upload([cur])
    acts = torch.from_numpy(np.asarray(action_codes, np.uint8)).cuda()
    ao = torch.zeros(1, dtype=torch.int64, device=acts.device)
    gg = torch.tensor([float(g)], dtype=torch.float64, device=acts.device)
    out = torch.empty(1, dtype=torch.float32, device=acts.device)
    cs = (C.c_double * 9)(*[float(x) for x in consts])
    ns = int(np.asarray(tracker_rows).reshape(-1, 8).shape[0])
    check(lib().mdl_views_shaped_reward(eng._h, ptr(pv), ptr(po), ns, ptr(cv), ptr(co), ptr(acts), ptr(ao),
                                        ptr(gg), 1, cs, ptr(out), C.c_void_p(stream_handle())),
          "mdl_views_shaped_reward")
    return np.float32(out.cpu().numpy()[0])


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
