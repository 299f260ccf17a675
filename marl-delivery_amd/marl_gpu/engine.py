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
from ._lib import raw_stream as _raw_stream
from .maps import grid_array, load_map, map_path

# shaping constants, order: pickup, on_time, late, closer, wasted_pick,
# wasted_drop, stuck, idle, away  (MAPPO/helper.py:271-279, QMIX/helper.py:270-278)
MAPPO_SHAPING = (5, 200, 20, 0.02, 0, 0, -0.05, -0.05, -0.01)
QMIX_SHAPING = (0.5, 2.0, 0.2, 0.02, -0.1, -0.1, -0.05, -0.02, -0.02)

TRACKER_MODES = {"fresh": _lib.MDL_TRACKER_FRESH, "mappo": _lib.MDL_TRACKER_MAPPO_STALE,
                 "mappo_stale": _lib.MDL_TRACKER_MAPPO_STALE}
ACTION_FORMATS = {"int": _lib.MDL_ACTION_TRAINER_INT, "codes": _lib.MDL_ACTION_CODES}
OBS_BUILDERS = {"auto": _lib.MDL_OBS_BUILDER_AUTO, "generic": _lib.MDL_OBS_BUILDER_GENERIC}
STEP_LAYOUTS = {"auto": _lib.MDL_STEP_LAYOUT_AUTO, "wave": _lib.MDL_STEP_LAYOUT_WAVE, "rows": _lib.MDL_STEP_LAYOUT_ROWS,
                "halves": _lib.MDL_STEP_LAYOUT_HALVES}
_LAYOUT_NAMES = {_lib.MDL_STEP_LAYOUT_WAVE: "wave", _lib.MDL_STEP_LAYOUT_ROWS: "rows", _lib.MDL_STEP_LAYOUT_HALVES: "halves"}
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
               obs_max_time_steps defaults to max_time_steps;
    obs_builder:   "auto" (the small builder where it applies, A <= 8 and P <= 64) or
               "generic" (always the general builder): the same observations either way.
    step_layout:   "auto" (four envs per wavefront for full-batch steps of >= 7,168 envs where A <= 8
               and P <= 64; two for >= 12,288 envs where A == 16 and P <= 128), "wave" (one env per
               wavefront), "rows" (four per wavefront) or "halves" (two per wavefront; both an error
               where they do not apply): the same results either way (MdlConfig.step_layout).
    After construction every env holds the constructor's layout draw; call
    ``reset()`` for the first episode, as the reference trainers do.
    """

    def __init__(self, maps, n_envs: int, n_robots: int = 5, n_packages: int = 20, max_time_steps: int = 100,
                 move_cost: float = -0.01, delivery_reward: float = 10.0, delay_reward: float = 1.0,
                 seed: int = 2025, seeds: Sequence[int] | None = None, env_map: Sequence[int] | None = None,
                 tracker: str = "mappo", shaping="mappo", max_other_robots: int | None = None,
                 max_packages_obs: int = 5, max_robots_state: int = 100, max_packages_state: int = 100,
                 obs_max_time_steps: int | None = None, obs_builder: str = "auto", step_layout: str = "auto",
                 device=None):
        if not torch.cuda.is_available():
            raise RuntimeError("marl_gpu.BatchedEnv needs a ROCm GPU (no CPU fallback)")
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        if self.device.type != "cuda":
            raise ValueError(f"marl_gpu.BatchedEnv runs on a GPU device, not {self.device}")
        if self.device.index is None:   # "cuda" -> the current device, explicitly
            self.device = torch.device("cuda", torch.cuda.current_device())
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
        cfg.obs_builder = OBS_BUILDERS[obs_builder]
        cfg.step_layout = STEP_LAYOUTS[step_layout]
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
        # whether a full-batch step runs four envs per wavefront: the engine's own decision
        self.step_rows = self.step_layout() == "rows"
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
        self._fn_step = lib().mdl_step
        self._out_ok = None
        self._dev = self.device.index
        self._full_out = (self._r, self._sh, self._done)
        # end (exclusive) of each env's run of consecutive envs with the same map shape:
        # an observation range must lie inside one run (its tensors have one H x W)
        hw_env = np.array([self.grids[m].shape for m in self.env_map], np.int64).reshape(self.E, 2)
        brk = np.nonzero(np.any(hw_env[1:] != hw_env[:-1], axis=1))[0] + 1
        ends = np.append(brk, self.E)
        self._shape_run_end = np.repeat(ends, np.diff(np.concatenate(([0], ends))))

    # ------------------------------------------------------------------ core
    def close(self):
        if getattr(self, "_h", None):
            # the mailbox context (compat's C step path) holds raw engine addresses: drop it first
            self.__dict__.pop("_mail_ctx", None)
            self.__dict__.pop("_mb", None)
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
        """Env-id subset -> (int32 device tensor or None, count).

        Host-side ids (list / numpy / CPU tensor) are checked like the reference's
        ``self.envs[i]`` indexing: negatives count from the end, anything outside
        [-E, E) raises IndexError.  Duplicates raise ValueError (one launch steps
        every listed env once, in parallel; ``compat.VectorizedEnv`` splits repeated
        ids into sequential launches as the reference's loop does).  Device tensors
        are taken as they are, without a host round trip: their ids must be unique
        and in [0, E) (the kernels skip ids outside that range, so a bad id cannot
        touch another env's memory, but it is not reported)."""
        if env_ids is None:
            return None, self.E
        if isinstance(env_ids, torch.Tensor) and env_ids.is_cuda:
            ids = env_ids
            if ids.dtype != torch.int32 or ids.get_device() != self.device.index or not ids.is_contiguous():
                ids = ids.to(device=self.device, dtype=torch.int32).contiguous()
            return ids.reshape(-1), int(ids.numel())
        a = np.asarray(env_ids.numpy() if isinstance(env_ids, torch.Tensor) else env_ids).reshape(-1)
        if a.size and a.dtype.kind not in "iu":
            raise TypeError(f"env ids must be integers, got {a.dtype}")
        a = a.astype(np.int64)
        if a.size and (a.min() < -self.E or a.max() >= self.E):
            raise IndexError(f"env id out of range for {self.E} envs")
        a = np.where(a < 0, a + self.E, a)
        if np.unique(a).size != a.size:
            raise ValueError("duplicate env ids in one call (each listed env is stepped once, in parallel)")
        return torch.from_numpy(a.astype(np.int32)).to(self.device), int(a.size)

    def reset(self, env_ids=None):
        """Environment.reset() for all envs or a subset (QMIX/env_vectorized.py:13-21)."""
        ids, n = self._ids(env_ids)
        if n == 0:
            return
        check(lib().mdl_reset(self._h, ptr(ids), n, self._stream()), "mdl_reset")
        self._keep = ids

    def clear_tracker(self, env_ids=None):
        ids, n = self._ids(env_ids)
        if n == 0:
            return
        check(lib().mdl_tracker_clear(self._h, ptr(ids), n, self._stream()), "mdl_tracker_clear")
        self._keep = ids

    def _check_out(self, out, shape):
        """The caller's (r_env f64, r_shaped f32, done uint8) buffers: dtype, device, size.
        The last checked buffers are remembered (objects, shape, addresses), so a step loop
        that reuses its buffers pays for the full check once."""
        if len(out) != 3:
            raise ValueError("out must be (r_env, r_shaped, done)")
        want = 1
        for s in shape:
            want *= s
        for t, dt, name in zip(out, (torch.float64, torch.float32, torch.uint8), ("r_env", "r_shaped", "done")):
            if not isinstance(t, torch.Tensor) or t.dtype != dt:
                raise TypeError(f"out {name} must be a {dt} tensor")
            if not t.is_cuda or t.get_device() != self.device.index or not t.is_contiguous():
                raise ValueError(f"out {name} must be contiguous on {self.device}")
            if t.numel() < want:
                raise ValueError(f"out {name} holds {t.numel()} entries, needs {want}")
        self._out_ok = (out[0], out[1], out[2], shape, (out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr()))

    def _out_ptrs(self, out, shape):
        """Addresses of checked output buffers (the full check only for new buffers)."""
        r, sh, d = out
        ptrs = (r.data_ptr(), sh.data_ptr(), d.data_ptr())
        m = self._out_ok
        if m is None or r is not m[0] or sh is not m[1] or d is not m[2] or m[3] != shape or m[4] != ptrs:
            self._check_out(out, shape)
        return ptrs

    def _step_args(self, actions, n, lead=()):
        if actions.dtype != torch.uint8 or not actions.is_cuda or actions.get_device() != self.device.index \
                or not actions.is_contiguous():
            actions = actions.to(device=self.device, dtype=torch.uint8).contiguous()
        if actions.numel() != n * self.A * (lead[0] if lead else 1) \
                or (lead and (actions.dim() != 3 or actions.shape[1] != n or actions.shape[2] != self.A)):
            raise ValueError(f"actions must be [{', '.join(str(x) for x in lead + (n, self.A))}]")
        return actions

    def step(self, actions: torch.Tensor, env_ids=None, auto_reset: bool = True, action_format: str = "int",
             out=None):
        """One transition for all envs (or ``env_ids``).

        actions: uint8 tensor [n, A] on the device -- trainer ints 0..14
        (MAPPO/trainer.py:198-205) or packed codes (action_format="codes").
        Returns (r_env f64 [n], r_shaped f32 [n], done uint8 [n]) views of
        reusable buffers unless ``out`` is given (then: float64 / float32 / uint8
        tensors of >= n entries on the engine's device).
        """
        if env_ids is None:
            ids, n = None, self.E
        else:
            ids, n = self._ids(env_ids)
        if actions.dtype is not torch.uint8 or not actions.is_cuda or not actions.is_contiguous() \
                or actions.get_device() != self._dev or actions.numel() != n * self.A:
            actions = self._step_args(actions, n)
        if out is None:
            out = self._full_out if n == self.E else (self._r[:n], self._sh[:n], self._done[:n])
            ptrs = (out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr())
        else:
            ptrs = self._out_ptrs(out, (n,))
        if n == 0:
            return out
        check(self._fn_step(self._h, actions.data_ptr(), ACTION_FORMATS[action_format],
                            None if ids is None else ids.data_ptr(), n, 1 if auto_reset else 0,
                            ptrs[0], ptrs[1], ptrs[2], _raw_stream(self._dev)), "mdl_step")
        self._keep = (ids, actions)
        return out[0], out[1], out[2]

    def step_obs(self, actions: torch.Tensor, auto_reset: bool = True, action_format: str = "int", out=None,
                 obs_out: dict | None = None, which=("actor_map", "actor_vec", "critic_map", "critic_vec")):
        """``step`` over all envs, then ``build_obs`` of the new state (the trainer's per-step
        sequence, MAPPO/trainer.py:229-286), as one launch when A <= 8 and P <= 64: the
        kernel builds the observations from the state the step leaves in registers.
        Bit-identical to ``step(...)`` followed by ``build_obs()``.  The envs must share one
        map shape.  Returns (r_env, r_shaped, done, obs dict); without ``obs_out`` the obs
        tensors are the engine's own buffers, overwritten by the next call."""
        n = self.E
        if actions.dtype is not torch.uint8 or not actions.is_cuda or not actions.is_contiguous() \
                or actions.get_device() != self._dev or actions.numel() != n * self.A:
            actions = self._step_args(actions, n)
        if out is None:
            out = self._full_out
            ptrs = (out[0].data_ptr(), out[1].data_ptr(), out[2].data_ptr())
        else:
            ptrs = self._out_ptrs(out, (n,))
        if self._shape_run_end[0] < n:
            raise ValueError("step_obs: the envs mix map shapes; use step() and build_obs() per same-shape group")
        H, W = self.grids[int(self.env_map[0])].shape
        if obs_out is None:
            obs_out = self._obs_cache if getattr(self, "_obs_cache", None) is not None else self.obs_buffers(n, H, W)
            self._obs_cache = obs_out
        shapes = dict(actor_map=(n, self.A, 6, H, W), actor_vec=(n, self.A, self.actor_vec_dim),
                      critic_map=(n, 4, H, W), critic_vec=(n, self.critic_vec_dim))
        op = {}
        for k in ("actor_map", "actor_vec", "critic_map", "critic_vec"):
            t = obs_out.get(k) if k in which else None
            if t is not None:
                self._check_obs_out(t, k, shapes[k])
            op[k] = None if t is None else t.data_ptr()
        check(lib().mdl_step_obs(self._h, actions.data_ptr(), ACTION_FORMATS[action_format], 1 if auto_reset else 0,
                                 ptrs[0], ptrs[1], ptrs[2], op["actor_map"], op["actor_vec"], op["critic_map"],
                                 op["critic_vec"], _raw_stream(self._dev)), "mdl_step_obs")
        self._keep = (None, actions)
        # only the outputs written by this call (a cached dict's other entries would be stale)
        return out[0], out[1], out[2], {k: (v if k in which else None) for k, v in obs_out.items()}

    def step_fused(self, actions: torch.Tensor, env_ids=None, auto_reset: bool = True, action_format: str = "int",
                   out=None):
        """Bench mode: K consecutive steps in one launch.

        actions: uint8 [K, n, A]; returns (r_env f64 [K, n], r_shaped f32 [K, n],
        done uint8 [K, n]), identical to K ``step`` calls with actions[k].
        """
        ids, n = self._ids(env_ids)
        if actions.dim() != 3:
            raise ValueError(f"actions must be [K, {n}, {self.A}]")
        K = actions.shape[0]
        actions = self._step_args(actions, n, (K,))
        if out is None:
            r = torch.empty((K, n), dtype=torch.float64, device=self.device)
            sh = torch.empty((K, n), dtype=torch.float32, device=self.device)
            d = torch.empty((K, n), dtype=torch.uint8, device=self.device)
        else:
            self._out_ptrs(out, (K, n))
            r, sh, d = out
        if n == 0 or K == 0:
            return r, sh, d
        check(lib().mdl_step_fused(self._h, ptr(actions), ACTION_FORMATS[action_format], ptr(ids), n, K,
                                   int(bool(auto_reset)), ptr(r), ptr(sh), ptr(d), self._stream()), "mdl_step_fused")
        self._keep = (ids, actions)
        return r, sh, d

    def step_layout(self, n: int | None = None) -> str:
        """The layout ``step`` launches ("wave": one env per wavefront, "rows": four, "halves": two) for the full
        batch (n None) or an ``env_ids`` subset of n envs -- asked of the engine (mdl_step_layout),
        which takes the same decision inside mdl_step."""
        lay = C.c_int32()
        check(lib().mdl_step_layout(self._h, self.E if n is None else int(n), 0 if n is None else 1,
                                    C.byref(lay)), "mdl_step_layout")
        return _LAYOUT_NAMES[lay.value]

    def step_kernel_name(self, layout: str | None = None, with_obs: bool = False) -> str:
        """The kernel symbol (as rocprof names it) ``step`` launches in ``layout`` (default: the
        full batch's), or ``step_obs``'s step launch with ``with_obs`` -- from the engine."""
        lay = ("wave" if with_obs else self.step_layout()) if layout is None else layout
        buf = C.create_string_buffer(128)
        check(lib().mdl_step_kernel_name(self._h, STEP_LAYOUTS[lay], 1 if with_obs else 0, buf, 128),
              "mdl_step_kernel_name")
        return buf.value.decode()

    def last_step_layout(self) -> str | None:
        """The layout of the last ``step`` launch (None before the first), as the engine recorded it."""
        lay = C.c_int32()
        check(lib().mdl_last_step_layout(self._h, C.byref(lay)), "mdl_last_step_layout")
        return None if lay.value == 0 else _LAYOUT_NAMES[lay.value]

    def step_floor(self, n: int | None = None):
        """Measurement aid: one launch of an empty kernel in ``step``'s launch shape over n envs
        (grid, workgroup, LDS, kernel arguments); touches no state.  bench.py's launch floor."""
        n = self.E if n is None else int(n)
        check(lib().mdl_step_floor(self._h, n, _raw_stream(self._dev)), "mdl_step_floor")

    def obs_buffers(self, n=None, H=None, W=None):
        n = self.E if n is None else n
        H = self.grids[0].shape[0] if H is None else H
        W = self.grids[0].shape[1] if W is None else W
        f = dict(dtype=torch.float32, device=self.device)
        return dict(actor_map=torch.empty((n, self.A, 6, H, W), **f),
                    actor_vec=torch.empty((n, self.A, self.actor_vec_dim), **f),
                    critic_map=torch.empty((n, 4, H, W), **f),
                    critic_vec=torch.empty((n, self.critic_vec_dim), **f))

    def _obs_range(self, env_begin, n):
        """Checked env range of one observation call -> (n, grid of its map shape)."""
        env_begin = int(env_begin)
        n = self.E - env_begin if n is None else int(n)
        if env_begin < 0 or n < 0 or env_begin + n > self.E:
            raise IndexError(f"env range [{env_begin}, {env_begin + n}) outside [0, {self.E})")
        if n == 0:
            return n, self.grids[0]
        if self._shape_run_end[env_begin] < env_begin + n:
            raise ValueError(f"envs [{env_begin}, {env_begin + n}) mix map shapes: build observations per "
                             f"same-shape group (this one ends at env {int(self._shape_run_end[env_begin])})")
        return n, self.grids[int(self.env_map[env_begin])]

    def _check_obs_out(self, t, name, shape):
        want = 1
        for s in shape:
            want *= s
        if not isinstance(t, torch.Tensor) or t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise TypeError(f"{name} must be a contiguous float32 device tensor")
        if t.get_device() != self.device.index:
            raise ValueError(f"{name} must be on {self.device}, not cuda:{t.get_device()}")
        if t.numel() < want:
            raise ValueError(f"{name} holds {t.numel()} floats, needs {want} {tuple(shape)}")

    def build_obs(self, env_begin: int = 0, n: int | None = None, out: dict | None = None,
                  which=("actor_map", "actor_vec", "critic_map", "critic_vec")):
        """convert_observation / generate_vector_features / convert_global_state
        for every agent of envs [env_begin, env_begin+n) (one map shape: raises
        on a range that mixes map shapes)."""
        n, g = self._obs_range(env_begin, n)
        H, W = g.shape
        if out is None:
            out = self.obs_buffers(n, H, W)
        p = {k: (out[k] if k in which else None) for k in ("actor_map", "actor_vec", "critic_map", "critic_vec")}
        shapes = dict(actor_map=(n, self.A, 6, H, W), actor_vec=(n, self.A, self.actor_vec_dim),
                      critic_map=(n, 4, H, W), critic_vec=(n, self.critic_vec_dim))
        for k, t in p.items():
            if t is not None:
                self._check_obs_out(t, k, shapes[k])
        if n == 0:
            return out
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
        n, g = self._obs_range(env_begin, n)
        H, W = g.shape
        oh, ow = (H, W) if state_shape is None else (int(state_shape[1]), int(state_shape[2]))
        if out is None:
            f = dict(dtype=torch.float32, device=self.device)
            out = {}
            if "idq_obs" in which:
                out["idq_obs"] = torch.empty((n, self.A, 6, H, W), **f)
            if "qmix_state" in which:
                out["qmix_state"] = torch.empty((n, 7, oh, ow), **f)
        if out.get("idq_obs") is not None:
            self._check_obs_out(out["idq_obs"], "idq_obs", (n, self.A, 6, H, W))
        if out.get("qmix_state") is not None:
            self._check_obs_out(out["qmix_state"], "qmix_state", (n, 7, oh, ow))
        if n == 0:
            return out
        check(lib().mdl_build_obs_alt(self._h, env_begin, n, ptr(out.get("idq_obs")), ptr(out.get("qmix_state")),
                                      oh, ow, self._stream()), "mdl_build_obs_alt")
        return out

    # ---- greedy baseline: greedyagent.py batched on the device ----
    def greedy_init(self, env_ids=None):
        """``GreedyAgents()`` + ``init_agents(state)`` for the listed envs (right after their reset)."""
        ids, n = self._ids(env_ids)
        if n == 0 and env_ids is not None:
            return
        check(lib().mdl_greedy_init(self._h, ptr(ids), n, self._stream()), "mdl_greedy_init")
        self._keep_g = ids

    def greedy_actions(self, env_ids=None, out=None) -> torch.Tensor:
        """One ``get_actions(state)`` per listed env: uint8 [n, A] in the "codes" action format."""
        ids, n = self._ids(env_ids)
        if out is None:
            out = torch.empty((n, self.A), dtype=torch.uint8, device=self.device)
        elif out.dtype != torch.uint8 or not out.is_cuda or not out.is_contiguous() or out.numel() < n * self.A \
                or out.get_device() != self.device.index:
            raise ValueError(f"out must be a contiguous uint8 tensor on {self.device} of >= {n}x{self.A} entries")
        if n == 0:
            return out
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

    # ---- dict-API mailbox (include/mdl_engine.h: mdl_mailbox / mdl_mail_*) ----
    def mailbox(self) -> dict:
        """numpy views of the engine's host-mapped mailbox (allocated on first use): inputs
        ``codes`` [E, A] (MDL_ACTION_CODES bytes) and ``ids`` [E]; outputs, row w = the w-th env
        of the last call: ``r_env``, ``r_shaped``, ``done``, ``robots`` [E, A, 3], ``pkgs``
        [E, P, 8], ``t``, ``total_reward``, ``rterms`` (the MDL_RTERM_* bits of the reward
        terms the step added).  The device reads the inputs and writes the outputs in place;
        every ``mail_*`` call returns once its rows are there (it spins on a completion word)."""
        mb = self.__dict__.get("_mb")
        if mb is None:
            m = _lib.MdlMailbox()
            check(lib().mdl_mailbox(self._h, C.byref(m)), "mdl_mailbox")
            E, A, P = self.E, self.A, self.P

            def arr(addr, ctype, shape):
                n = 1
                for d in shape:
                    n *= d
                return np.ctypeslib.as_array((ctype * n).from_address(addr)).reshape(shape)
            mb = dict(codes=arr(m.codes, C.c_uint8, (E, A)), ids=arr(m.ids, C.c_int32, (E,)),
                      r_env=arr(m.r_env, C.c_double, (E,)), r_shaped=arr(m.r_shaped, C.c_float, (E,)),
                      done=arr(m.done, C.c_uint8, (E,)), robots=arr(m.robots, C.c_int32, (E, A, 3)),
                      pkgs=arr(m.pkgs, C.c_int32, (E, P, 8)), t=arr(m.t, C.c_int32, (E,)),
                      total_reward=arr(m.total_reward, C.c_double, (E,)), rterms=arr(m.rterms, C.c_int32, (E,)))
            self._mb = mb
            self._mbox = m
            L = lib()
            self._mail_fns = (L.mdl_mail_step, L.mdl_mail_reset, L.mdl_mail_export)
        return mb

    def mail_ctx(self):
        """The mailbox as the C extension's context (compat.Environment.step in one C call)."""
        c = self.__dict__.get("_mail_ctx")
        if c is None:
            self.mailbox()
            m = self._mbox
            c = self._mail_ctx = _lib.pack().mail_ctx(
                C.cast(lib().mdl_mail_step, C.c_void_p).value, self._h.value, m.codes, m.ids, m.r_env, m.done,
                m.robots, m.pkgs, m.t, m.total_reward, m.rterms, self.A, self.P)
        return c

    def mail_step(self, n: int, use_ids: bool, auto_reset: bool = False) -> None:
        """Step the mailbox's envs (``ids[:n]`` when use_ids, else all E, with ``codes[:n]``) and
        bring their rows into the mailbox: one step launch + one export launch, then a spin."""
        rc = self._mail_fns[0](self._h, n, 1 if use_ids else 0, 1 if auto_reset else 0, _raw_stream(self._dev))
        if rc:
            check(rc, "mdl_mail_step")

    def mail_reset(self, n: int, use_ids: bool) -> None:
        rc = self._mail_fns[1](self._h, n, 1 if use_ids else 0, _raw_stream(self._dev))
        if rc:
            check(rc, "mdl_mail_reset")

    def mail_export(self, n: int, use_ids: bool) -> None:
        rc = self._mail_fns[2](self._h, n, 1 if use_ids else 0, _raw_stream(self._dev))
        if rc:
            check(rc, "mdl_mail_export")

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
