"""Tensor API of the MI355X batched step engine.

``BatchedEnv`` holds E independent marl-delivery environments resident in HBM
and steps them with one gfx950 kernel launch per step (one wavefront per env).
It is the batched counterpart of ``VectorizedEnv(Environment, E, ...)``
(MAPPO/env_vectorized.py:1-24, QMIX/env_vectorized.py:1-49) fused with the
MAPPO rollout glue that surrounds it (MAPPO/trainer.py:194-286): integer
action decode, ``compute_shaped_rewards`` with the pre-step tracker, the
persistent-package tracker update and reset-on-done all run on the device.

Inputs and outputs are torch tensors on the engine's device; every call is
asynchronous on torch's current stream.
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr, stream_handle
from .maps import grid_array, load_map, map_path

# shaping constants, order: pickup, on_time, late, closer, wasted_pick,
# wasted_drop, stuck, idle, away  (MAPPO/helper.py:271-279, QMIX/helper.py:270-278)
MAPPO_SHAPING = (5, 200, 20, 0.02, 0, 0, -0.05, -0.05, -0.01)
QMIX_SHAPING = (0.5, 2.0, 0.2, 0.02, -0.1, -0.1, -0.05, -0.02, -0.02)

TRACKER_MODES = {"fresh": _lib.MDL_TRACKER_FRESH, "mappo": _lib.MDL_TRACKER_MAPPO_STALE,
                 "mappo_stale": _lib.MDL_TRACKER_MAPPO_STALE}
ACTION_FORMATS = {"int": _lib.MDL_ACTION_TRAINER_INT, "codes": _lib.MDL_ACTION_CODES}
STATUS_NAMES = ("None", "waiting", "in_transit", "delivered")


def _as_grid(m):
    if isinstance(m, str):
        return grid_array(load_map(map_path(m)))
    return grid_array(m)


class BatchedEnv:
    """E environments on one GPU.

    maps:      one map (path / name / 2-D 0-1 array) or a list of up to 8 maps;
    env_map:   per-env map index when several maps are given (contiguous
               groups keep each observation tensor single-shaped);
    seeds:     per-env RandomState seeds; default ``seed + i`` like
               VectorizedEnv (MAPPO/env_vectorized.py:8-9);
    tracker:   "mappo" (never cleared on auto-reset, MAPPO/trainer.py:232-233)
               or "fresh" (== env truth, QMIX/evaluation semantics);
    shaping:   "mappo" | "qmix" | 9 constants;
    obs dims:  max_other_robots / max_packages_obs (generate_vector_features),
               max_robots_state / max_packages_state (convert_global_state);
               obs_max_time_steps defaults to max_time_steps.
    After construction every env holds the constructor's layout draw; call
    ``reset()`` for the first episode, as the reference trainers do.
    """

    def __init__(self, maps, n_envs: int, n_robots: int = 5, n_packages: int = 20, max_time_steps: int = 100,
                 move_cost: float = -0.01, delivery_reward: float = 10.0, delay_reward: float = 1.0,
                 seed: int = 2025, seeds: Sequence[int] | None = None, env_map: Sequence[int] | None = None,
                 tracker: str = "mappo", shaping="mappo", max_other_robots: int | None = None,
                 max_packages_obs: int = 5, max_robots_state: int = 100, max_packages_state: int = 100,
                 obs_max_time_steps: int | None = None, device=None):
        if not torch.cuda.is_available():
            raise RuntimeError("marl_gpu.BatchedEnv needs a ROCm GPU (no CPU fallback)")
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        if isinstance(maps, (str, np.ndarray)) or (isinstance(maps, list) and maps and isinstance(maps[0], list)
                                                  and maps[0] and isinstance(maps[0][0], (int, np.integer))):
            maps = [maps]
        self.grids = [_as_grid(m) for m in maps]
        self.E, self.A, self.P, self.T = int(n_envs), int(n_robots), int(n_packages), int(max_time_steps)
        if isinstance(shaping, str):
            shaping = {"mappo": MAPPO_SHAPING, "qmix": QMIX_SHAPING}[shaping]
        self.shaping = tuple(float(x) for x in shaping)
        self.tracker = tracker
        self.MO = self.A - 1 if max_other_robots is None else int(max_other_robots)
        self.MP, self.MR, self.MPs = int(max_packages_obs), int(max_robots_state), int(max_packages_state)
        self.obs_T = self.T if obs_max_time_steps is None else int(obs_max_time_steps)
        cfg = _lib.MdlConfig()
        cfg.n_envs, cfg.n_robots, cfg.n_packages, cfg.max_time_steps = self.E, self.A, self.P, self.T
        cfg.move_cost, cfg.delivery_reward, cfg.delay_reward = float(move_cost), float(delivery_reward), float(delay_reward)
        cfg.tracker_mode = TRACKER_MODES[tracker]
        for i, v in enumerate(self.shaping):
            cfg.shaping[i] = v
        cfg.obs_max_time_steps = self.obs_T
        cfg.max_other_robots, cfg.max_packages_obs = self.MO, self.MP
        cfg.max_robots_state, cfg.max_packages_state = self.MR, self.MPs
        self.cfg = cfg
        flat = np.ascontiguousarray(np.concatenate([g.reshape(-1) for g in self.grids]).astype(np.uint8))
        hw = np.array([[g.shape[0], g.shape[1]] for g in self.grids], np.int32).reshape(-1)
        if env_map is None:
            env_map = [0] * self.E if len(self.grids) == 1 else None
            if env_map is None:
                raise ValueError("env_map is required with several maps")
        self.env_map = np.ascontiguousarray(np.asarray(env_map, np.int32))
        if self.env_map.shape != (self.E,):
            raise ValueError("env_map must have one entry per env")
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().mdl_create(C.byref(cfg), flat.ctypes.data, hw.ctypes.data, len(self.grids),
                                   self.env_map.ctypes.data, self.device.index, C.byref(h)), "mdl_create")
        self._h = h
        av, cv = C.c_int32(), C.c_int32()
        check(lib().mdl_obs_dims(self._h, C.byref(av), C.byref(cv)))
        self.actor_vec_dim, self.critic_vec_dim = av.value, cv.value
        if seeds is None:
            seeds = [int(seed) + i for i in range(self.E)]
        self.seeds = np.ascontiguousarray(np.asarray(seeds, np.int64) & 0xFFFFFFFF).astype(np.uint32)
        if self.seeds.shape != (self.E,):
            raise ValueError("seeds must have one entry per env")
        with torch.cuda.device(self.device):
            check(lib().mdl_seed(self._h, self.seeds.ctypes.data, C.c_void_p(stream_handle(self.device))),
                  "mdl_seed")
        # reusable outputs
        self._r = torch.zeros(self.E, dtype=torch.float64, device=self.device)
        self._sh = torch.zeros(self.E, dtype=torch.float32, device=self.device)
        self._done = torch.zeros(self.E, dtype=torch.uint8, device=self.device)

    # ------------------------------------------------------------------ core
    def close(self):
        if getattr(self, "_h", None):
            lib().mdl_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return C.c_void_p(stream_handle(self.device))

    def _ids(self, env_ids):
        if env_ids is None:
            return None, self.E
        ids = torch.as_tensor(env_ids, dtype=torch.int32, device=self.device).contiguous()
        return ids, int(ids.numel())

    def reset(self, env_ids=None):
        """Environment.reset() for all envs or a subset (QMIX/env_vectorized.py:13-21)."""
        ids, n = self._ids(env_ids)
        check(lib().mdl_reset(self._h, ptr(ids), n, self._stream()), "mdl_reset")
        self._keep = ids

    def clear_tracker(self, env_ids=None):
        ids, n = self._ids(env_ids)
        check(lib().mdl_tracker_clear(self._h, ptr(ids), n, self._stream()), "mdl_tracker_clear")
        self._keep = ids

    def step(self, actions: torch.Tensor, env_ids=None, auto_reset: bool = True, action_format: str = "int",
             out=None):
        """One transition for all envs (or ``env_ids``).

        actions: uint8 tensor [n, A] on the device -- trainer ints 0..14
        (MAPPO/trainer.py:198-205) or packed codes (action_format="codes").
        Returns (r_env f64 [n], r_shaped f32 [n], done uint8 [n]) views of
        reusable buffers unless ``out`` is given.
        """
        ids, n = self._ids(env_ids)
        if actions.dtype != torch.uint8 or actions.device != self.device or not actions.is_contiguous():
            actions = actions.to(device=self.device, dtype=torch.uint8).contiguous()
        if actions.numel() != n * self.A:
            raise ValueError(f"actions must hold {n}x{self.A} entries")
        if out is None:
            r, sh, d = self._r[:n], self._sh[:n], self._done[:n]
        else:
            r, sh, d = out
        check(lib().mdl_step(self._h, ptr(actions), ACTION_FORMATS[action_format], ptr(ids), n, int(bool(auto_reset)),
                             ptr(r), ptr(sh), ptr(d), self._stream()), "mdl_step")
        self._keep = (ids, actions)
        return r, sh, d

    def step_fused(self, actions: torch.Tensor, env_ids=None, auto_reset: bool = True, action_format: str = "int",
                   out=None):
        """Bench mode: K consecutive steps in one launch.

        actions: uint8 [K, n, A]; returns (r_env f64 [K, n], r_shaped f32 [K, n],
        done uint8 [K, n]), identical to K ``step`` calls with actions[k].
        """
        ids, n = self._ids(env_ids)
        if actions.dtype != torch.uint8 or actions.device != self.device or not actions.is_contiguous():
            actions = actions.to(device=self.device, dtype=torch.uint8).contiguous()
        if actions.dim() != 3 or actions.shape[1] != n or actions.shape[2] != self.A:
            raise ValueError(f"actions must be [K, {n}, {self.A}]")
        K = actions.shape[0]
        if out is None:
            r = torch.empty((K, n), dtype=torch.float64, device=self.device)
            sh = torch.empty((K, n), dtype=torch.float32, device=self.device)
            d = torch.empty((K, n), dtype=torch.uint8, device=self.device)
        else:
            r, sh, d = out
        check(lib().mdl_step_fused(self._h, ptr(actions), ACTION_FORMATS[action_format], ptr(ids), n, K,
                                   int(bool(auto_reset)), ptr(r), ptr(sh), ptr(d), self._stream()), "mdl_step_fused")
        self._keep = (ids, actions)
        return r, sh, d

    def obs_buffers(self, n=None, H=None, W=None):
        n = self.E if n is None else n
        H = self.grids[0].shape[0] if H is None else H
        W = self.grids[0].shape[1] if W is None else W
        f = dict(dtype=torch.float32, device=self.device)
        return dict(actor_map=torch.empty((n, self.A, 6, H, W), **f),
                    actor_vec=torch.empty((n, self.A, self.actor_vec_dim), **f),
                    critic_map=torch.empty((n, 4, H, W), **f),
                    critic_vec=torch.empty((n, self.critic_vec_dim), **f))

    def build_obs(self, env_begin: int = 0, n: int | None = None, out: dict | None = None,
                  which=("actor_map", "actor_vec", "critic_map", "critic_vec")):
        """convert_observation / generate_vector_features / convert_global_state
        for every agent of envs [env_begin, env_begin+n) (one map shape)."""
        n = self.E - env_begin if n is None else n
        g = self.grids[int(self.env_map[env_begin])] if n else self.grids[0]
        if out is None:
            out = self.obs_buffers(n, g.shape[0], g.shape[1])
        p = {k: (out[k] if k in which else None) for k in ("actor_map", "actor_vec", "critic_map", "critic_vec")}
        check(lib().mdl_build_obs(self._h, env_begin, n, ptr(p["actor_map"]), ptr(p["actor_vec"]),
                                  ptr(p["critic_map"]), ptr(p["critic_vec"]), self._stream()), "mdl_build_obs")
        return out

    # ---- IDQ / qmix featurizers ----
    def build_obs_alt(self, env_begin: int = 0, n: int | None = None, out: dict | None = None,
                      state_shape=None, which=("idq_obs", "qmix_state")):
        """convert_state for every agent (IDQ/networks.py:112-217, == qmix/networks.py:243-348) and
        convert_global_state_to_tensor (qmix/networks.py:350-468) for envs [env_begin, env_begin+n).
        state_shape (7, h, w) defaults to the map's (7, H, W) as the qmix trainer uses; build the
        engine with tracker="fresh" for the IDQ / qmix trainers' per-episode trackers."""
        n = self.E - env_begin if n is None else n
        g = self.grids[int(self.env_map[env_begin])] if n else self.grids[0]
        H, W = g.shape
        oh, ow = (H, W) if state_shape is None else (int(state_shape[1]), int(state_shape[2]))
        if out is None:
            f = dict(dtype=torch.float32, device=self.device)
            out = {}
            if "idq_obs" in which:
                out["idq_obs"] = torch.empty((n, self.A, 6, H, W), **f)
            if "qmix_state" in which:
                out["qmix_state"] = torch.empty((n, 7, oh, ow), **f)
        check(lib().mdl_build_obs_alt(self._h, env_begin, n, ptr(out.get("idq_obs")), ptr(out.get("qmix_state")),
                                      oh, ow, self._stream()), "mdl_build_obs_alt")
        return out

    # ---- greedy baseline: greedyagent.py batched on the device ----
    def greedy_init(self, env_ids=None):
        """``GreedyAgents()`` + ``init_agents(state)`` for the listed envs (right after their reset)."""
        ids, n = self._ids(env_ids)
        check(lib().mdl_greedy_init(self._h, ptr(ids), n, self._stream()), "mdl_greedy_init")
        self._keep_g = ids

    def greedy_actions(self, env_ids=None, out=None) -> torch.Tensor:
        """One ``get_actions(state)`` per listed env: uint8 [n, A] in the "codes" action format."""
        ids, n = self._ids(env_ids)
        if out is None:
            out = torch.empty((n, self.A), dtype=torch.uint8, device=self.device)
        check(lib().mdl_greedy_actions(self._h, ptr(ids), n, ptr(out), self._stream()), "mdl_greedy_actions")
        self._keep_g = ids
        return out

    # ---- checkpoint: engine state incl. every env's MT19937 stream ----
    def save_state(self, path=None) -> np.ndarray:
        """Snapshot of the whole engine state as a uint8 array (written to ``path`` as .npy
        when given).  Loading it into an engine built with the same configuration resumes
        every env exactly (the reference cannot: its RandomState lives inside each env)."""
        n = C.c_int64()
        check(lib().mdl_state_bytes(self._h, C.byref(n)), "mdl_state_bytes")
        buf = np.zeros(n.value, np.uint8)
        check(lib().mdl_save_state(self._h, buf.ctypes.data, n.value, self._stream()), "mdl_save_state")
        if path is not None:
            np.save(path, buf, allow_pickle=False)
        return buf

    def load_state(self, src) -> None:
        """Restore a ``save_state`` snapshot (array or .npy path); raises on a mismatched engine."""
        buf = np.load(src, allow_pickle=False) if isinstance(src, (str, bytes)) or hasattr(src, "__fspath__") \
            else np.asarray(src)
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        check(lib().mdl_load_state(self._h, buf.ctypes.data, buf.nbytes, self._stream()), "mdl_load_state")

    def read_state(self):
        """int32/f64 device tensors: robots [E,A,3] (r,c,carry), pkgs [E,P,8]
        (sr,sc,tr,tc,start_time,deadline,id,status), t [E], total_reward [E],
        tracker [E,P,4] (present,in_transit,order,_), tracker_data [E,P,6]."""
        i = dict(dtype=torch.int32, device=self.device)
        s = dict(robots=torch.empty((self.E, self.A, 3), **i), pkgs=torch.empty((self.E, self.P, 8), **i),
                 t=torch.empty(self.E, **i), total_reward=torch.empty(self.E, dtype=torch.float64, device=self.device),
                 tracker=torch.empty((self.E, self.P, 4), **i), tracker_data=torch.empty((self.E, self.P, 6), **i))
        check(lib().mdl_read_state(self._h, ptr(s["robots"]), ptr(s["pkgs"]), ptr(s["t"]), ptr(s["total_reward"]),
                                   ptr(s["tracker"]), ptr(s["tracker_data"]), self._stream()), "mdl_read_state")
        return s

    def tracker_rows(self, state_cpu: dict, e: int) -> np.ndarray:
        """Tracker of env e as ordered dict rows (id, status, sr, sc, tr, tc, st, dl)."""
        trk = state_cpu["tracker"][e]
        data = state_cpu["tracker_data"][e]
        pres = np.nonzero(trk[:, 0])[0]
        order = pres[np.argsort(trk[pres, 2], kind="stable")]
        rows = np.zeros((len(order), 8), np.int32)
        rows[:, 0] = order + 1
        rows[:, 1] = np.where(trk[order, 1] != 0, 2, 1)
        rows[:, 2:8] = data[order]
        return rows
