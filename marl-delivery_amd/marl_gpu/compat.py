"""Drop-in dict API over the GPU engine.

``Environment`` mirrors env.py:18-455 (constructor signature, attributes,
``reset()`` / ``step()`` / ``get_state()`` dicts, ``render()``) and
``VectorizedEnv`` mirrors MAPPO/env_vectorized.py:1-24 plus the ``indices=``
variant of QMIX/env_vectorized.py:1-49, so agents and trainer loops written
against the reference run unchanged.  Every transition executes on the GPU;
the dicts are materialised from a device snapshot after each call.

Differences (documented, not silent):
  * ``step`` returns the int ``0`` whenever the step reward is 0.0 (the
    reference returns the int 0 when no reward term fired, and a float that
    happens to equal 0.0 in the rare case the terms cancel);
  * ``render_pygame`` is a no-op (headless), ``render`` prints text as the
    reference's ``render``.
"""
from __future__ import annotations

import operator

import numpy as np
import torch

from .engine import STATUS_NAMES, BatchedEnv
from .maps import grid_array, load_map, map_path

MOVE_CODES = {"S": 0, "L": 1, "R": 2, "U": 3, "D": 4}   # anything else -> 5 (no move, != 'S')
OP_CODES = {"0": 0, "1": 1, "2": 2}                     # anything else -> 3 (no env effect)


def _codes_to_device(eng, codes):
    """Action codes -> the engine's device through a reused pinned staging buffer (no
    synchronous pageable copy; the previous call's snapshot synchronisation has retired
    the previous copy, so reuse is safe)."""
    key = codes.shape
    cache = eng.__dict__.setdefault("_compat_codes", {})
    bufs = cache.get(key)
    if bufs is None:
        bufs = cache[key] = (torch.empty(key, dtype=torch.uint8, pin_memory=True),
                             torch.empty(key, dtype=torch.uint8, device=eng.device))
    h, d = bufs
    h.numpy()[...] = codes
    d.copy_(h, non_blocking=True)
    return d


def encode_actions(actions, n_robots):
    """list[(move_str, op_str)] -> packed codes (move | op << 3), env.py:193-195 strings."""
    if len(actions) != n_robots:
        raise ValueError("The number of actions must match the number of robots.")
    out = np.empty(n_robots, np.uint8)
    for i, (mv, op) in enumerate(actions):
        m = MOVE_CODES.get(mv, 5)
        out[i] = m | (OP_CODES.get(op, 3) << 3)
    return out


class Robot:
    __slots__ = ("position", "carrying")

    def __init__(self, position, carrying=0):
        self.position = position
        self.carrying = carrying


class Package:
    __slots__ = ("start", "start_time", "target", "deadline", "package_id", "status")

    def __init__(self, start, start_time, target, deadline, package_id, status="None"):
        self.start = start
        self.start_time = start_time
        self.target = target
        self.deadline = deadline
        self.package_id = package_id
        self.status = status


class _Slot:
    """Host mirror of one env slot of a BatchedEnv, refreshed after each call.  The
    ``robots`` / ``packages`` object lists are built on first access after a refresh (the
    state dict is built from the snapshot arrays directly)."""

    def __init__(self, owner, idx):
        self._owner = owner
        self._idx = idx

    def _refresh(self, snap):
        e = self._idx
        self._rob = snap["robots"][e]
        self._pk = snap["pkgs"][e]
        self.t = int(snap["t"][e])
        self.total_reward = float(snap["total_reward"][e])
        self._robots = None
        self._packages = None

    @property
    def robots(self):
        if self._robots is None:
            self._robots = [Robot((r[0], r[1]), r[2]) for r in self._rob.tolist()]
        return self._robots

    @robots.setter
    def robots(self, v):
        self._robots = v

    @property
    def packages(self):
        if self._packages is None:
            self._packages = [Package((p[0], p[1]), p[4], (p[2], p[3]), p[5], p[6], STATUS_NAMES[p[7]])
                              for p in self._pk.tolist()]
        return self._packages

    @packages.setter
    def packages(self, v):
        self._packages = v

    def _state_dict(self):
        t = self.t
        pk = self._pk
        new = pk[pk[:, 4] == t].tolist()   # get_state lists the packages spawned at this t (env.py:133-146)
        return {
            "time_step": t,
            "map": self.grid,
            "robots": [(r[0] + 1, r[1] + 1, r[2]) for r in self._rob.tolist()],
            "packages": [(p[6], p[0] + 1, p[1] + 1, p[2] + 1, p[3] + 1, p[4], p[5]) for p in new],
        }


class Environment(_Slot):
    """env.py:18-455 on the GPU engine (one env)."""

    def __init__(self, map_file, max_time_steps=100, n_robots=5, n_packages=20, move_cost=-0.01,
                 delivery_reward=10., delay_reward=1., seed=2025, _engine=None, _idx=0):
        self.map_file = map_file
        self.grid = load_map(map_path(map_file)) if _engine is None else _engine._grid_list
        self.n_rows = len(self.grid)
        self.n_cols = len(self.grid[0]) if self.grid else 0
        self.move_cost = move_cost
        self.delivery_reward = delivery_reward
        self.delay_reward = delay_reward
        self.n_robots = n_robots
        self.max_time_steps = max_time_steps
        self.n_packages = n_packages
        if _engine is None:
            _engine = BatchedEnv(grid_array(self.grid), 1, n_robots, n_packages, max_time_steps, move_cost,
                                 delivery_reward, delay_reward, seeds=[seed], tracker="fresh")
            _engine._grid_list = self.grid
            self._vec = None
        super().__init__(_engine, _idx)
        self.engine = _engine
        self.done = False
        self.state = None
        if getattr(_engine, "_snap", None) is None:
            _engine._snap = _snapshot(_engine)
        self._refresh(_engine._snap)

    # env.py:81-125
    def reset(self):
        ids = None if self.engine.E == 1 else [self._idx]
        self.engine.reset(ids)
        snap = self.engine.host_snapshot()
        self.engine._snap = snap
        self._refresh(snap)
        self.done = False
        self.state = None
        return self._state_dict()

    def get_state(self):
        return self._state_dict()

    # env.py:173-306
    def step(self, actions):
        codes = encode_actions(actions, self.n_robots)
        eng = self.engine
        a = _codes_to_device(eng, codes.reshape(1, -1))
        ids = None if eng.E == 1 else [self._idx]
        eng.step(a, env_ids=ids, auto_reset=False, action_format="codes", out=eng.snapshot_step_out(1))
        snap = eng.host_snapshot()
        r_h = float(snap["r_env"][0])
        done = bool(snap["done"][0])
        eng._snap = snap
        self._refresh(snap)
        infos = {}
        if done:
            infos["total_reward"] = self.total_reward
            infos["total_time_steps"] = self.t
        return self._state_dict(), (0 if r_h == 0.0 else r_h), done, infos

    def check_terminate(self):
        if self.t == self.max_time_steps:
            return True
        return all(p.status == "delivered" for p in self.packages)

    def is_free_cell(self, position):
        r, c = position
        if r < 0 or r >= self.n_rows or c < 0 or c >= self.n_cols:
            return False
        return self.grid[r][c] == 0

    def valid_position(self, pos):
        r, c = pos
        if r < 0 or r >= self.n_rows or c < 0 or c >= self.n_cols:
            return False
        return self.grid[r][c] != 1

    def compute_new_position(self, position, move):
        r, c = position
        return {"S": (r, c), "L": (r, c - 1), "R": (r, c + 1), "U": (r - 1, c), "D": (r + 1, c)}.get(move, (r, c))

    def render(self):
        grid_copy = [row[:] for row in self.grid]
        for i, robot in enumerate(self.robots):
            r, c = robot.position
            grid_copy[r][c] = "R%i" % i
        for row in grid_copy:
            print("\t".join(str(cell) for cell in row))

    def render_pygame(self, cell_size=40):  # headless engine
        return None


def _snapshot(engine: BatchedEnv):
    return engine.host_snapshot()


class VectorizedEnv:
    """MAPPO/env_vectorized.py:1-24 + QMIX ``indices=`` (QMIX/env_vectorized.py:13-37).

    One BatchedEnv holds all envs; env i is seeded ``seed + i``.
    """

    def __init__(self, env_cls=None, num_envs=1, **env_kwargs):
        map_file = env_kwargs.get("map_file")
        grid = load_map(map_path(map_file))
        base_seed = env_kwargs.get("seed", None)
        # MAPPO/env_vectorized.py:4-10: seed + idx, or the Environment default
        seeds = [base_seed + i for i in range(num_envs)] if base_seed is not None else [2025] * num_envs
        n_robots = env_kwargs.get("n_robots", 5)
        n_packages = env_kwargs.get("n_packages", 20)
        T = env_kwargs.get("max_time_steps", 100)
        self.engine = BatchedEnv(grid_array(grid), num_envs, n_robots, n_packages, T,
                                 env_kwargs.get("move_cost", -0.01), env_kwargs.get("delivery_reward", 10.),
                                 env_kwargs.get("delay_reward", 1.), seeds=seeds, tracker="fresh")
        self.engine._grid_list = grid
        self.engine._snap = None
        self.envs = [Environment(map_file, T, n_robots, n_packages, env_kwargs.get("move_cost", -0.01),
                                 env_kwargs.get("delivery_reward", 10.), env_kwargs.get("delay_reward", 1.),
                                 seeds[i], _engine=self.engine, _idx=i) for i in range(num_envs)]
        self.num_envs = num_envs

    def _refresh_all(self, snap=None):
        snap = _snapshot(self.engine) if snap is None else snap
        self.engine._snap = snap
        for env in self.envs:
            env._refresh(snap)

    def _index(self, indices):
        """``self.envs[i]`` semantics of the reference's loops: negatives count from the
        end, anything else out of range raises IndexError."""
        n = self.num_envs
        out = []
        for i in indices:
            i = operator.index(i)
            if i < -n or i >= n:
                raise IndexError("list index out of range")
            out.append(i % n)
        return out

    @staticmethod
    def _rounds(idx):
        """Split positions into launches with distinct envs: the k-th occurrence of an env
        goes to launch k, so repeated envs step (or reset) in list order, as the
        reference's serial loop does (QMIX/env_vectorized.py:13-37)."""
        seen, rounds = {}, []
        for pos, e in enumerate(idx):
            k = seen.get(e, 0)
            seen[e] = k + 1
            if k == len(rounds):
                rounds.append([])
            rounds[k].append(pos)
        return rounds

    def reset(self, indices=None):
        if indices is None:
            self.engine.reset(None)
            self._refresh_all()
            return [env._state_dict() for env in self.envs]
        idx = self._index(indices)
        out = [None] * len(idx)
        for rnd in self._rounds(idx):
            self.engine.reset([idx[p] for p in rnd])
            self._refresh_all()
            for p in rnd:
                out[p] = self.envs[idx[p]]._state_dict()
        return out

    def step(self, actions, indices=None):
        # zip() semantics of the reference (QMIX/env_vectorized.py:32-35): the shorter of
        # the env list and the action list decides how many envs step
        actions = list(actions)
        if indices is None:
            idx = list(range(min(self.num_envs, len(actions))))
            rounds = [list(range(len(idx)))]
            full = len(idx) == self.num_envs
        else:
            idx = self._index(indices)[:len(actions)]
            rounds = self._rounds(idx)
            full = False
        eng = self.engine
        res = [None] * len(idx)
        for rnd in rounds:
            ids = [idx[p] for p in rnd]
            codes = np.stack([encode_actions(actions[p], self.envs[e].n_robots) for p, e in zip(rnd, ids)])
            a = _codes_to_device(eng, codes)
            eng.step(a, env_ids=None if full else ids, auto_reset=False, action_format="codes",
                     out=eng.snapshot_step_out(len(ids)))
            snap = eng.host_snapshot()
            r_h, d_h = snap["r_env"], snap["done"].astype(bool)
            self._refresh_all(snap)
            for k, (p, e) in enumerate(zip(rnd, ids)):
                env = self.envs[e]
                info = {}
                if d_h[k]:
                    info = {"total_reward": env.total_reward, "total_time_steps": env.t}
                res[p] = (env._state_dict(), 0 if r_h[k] == 0.0 else float(r_h[k]), bool(d_h[k]), info)
        if not res:
            raise ValueError("not enough values to unpack (expected 4, got 0)")   # zip(*[]) in the reference
        states, rewards, dones, infos = (list(x) for x in zip(*res))
        return states, rewards, dones, infos

    def render(self, indices=None):
        return None
