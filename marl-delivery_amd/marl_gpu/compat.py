"""Drop-in dict API over the GPU engine.

``Environment`` mirrors env.py:18-455 (constructor signature, attributes,
``reset()`` / ``step()`` / ``get_state()`` dicts, ``render()``) and
``VectorizedEnv`` mirrors MAPPO/env_vectorized.py:1-24 plus the ``indices=``
variant of QMIX/env_vectorized.py:1-49, so agents and trainer loops written
against the reference run unchanged.  Every transition executes on the GPU.
A call goes through the engine's host-mapped mailbox (``BatchedEnv.mailbox``):
the action codes are written into it, the step kernel reads them there, an
export kernel writes the touched envs' rows back into it and the call returns
when they have arrived -- no device staging buffers, copies or stream syncs.

``step`` returns the reward with the reference's type: env.py:181 starts from
the int ``0`` and adds the move costs / delivery rewards (env.py:256,288,291),
so the result is the int 0 when no term fired, a float once a float constant
was added (also when the terms cancel to 0.0), and an int when only int
constants were added.  ``total_reward`` (and ``infos['total_reward']``) likewise: the
int 0 after a reset (env.py:34,89), an int while every step's reward was an int, a float once
one was a float (``self.total_reward += r``, env.py:297,303).  ``render_pygame`` is a no-op
(headless); ``render`` prints text as the reference's ``render`` does.

Not thread-safe per engine: the envs of one ``VectorizedEnv`` share its mailbox.
"""
from __future__ import annotations

import numbers
import operator

import numpy as np

from ._lib import MDL_RTERM_LATE, MDL_RTERM_MOVE, MDL_RTERM_ONTIME
from ._lib import pack as _pack
from ._lib import raw_stream as _raw_stream
from .engine import STATUS_NAMES, BatchedEnv
from .maps import grid_array, load_map, map_path

MOVE_CODES = {"S": 0, "L": 1, "R": 2, "U": 3, "D": 4}   # anything else -> 5 (no move, != 'S')
OP_CODES = {"0": 0, "1": 1, "2": 2}                     # anything else -> 3 (no env effect)
# the code byte of every (move, op) string pair: move | op << 3
_PAIR_CODES = {(m, o): mc | (oc << 3) for m, mc in list(MOVE_CODES.items()) for o, oc in list(OP_CODES.items())}


def _code(mv, op):
    c = _PAIR_CODES.get((mv, op)) if isinstance(mv, str) and isinstance(op, str) else None
    if c is None:
        c = (MOVE_CODES.get(mv, 5) if isinstance(mv, str) else 5) | \
            ((OP_CODES.get(op, 3) if isinstance(op, str) else 3) << 3)
    return c


def _encode(actions, n_robots):
    if len(actions) != n_robots:   # env.py:182-183
        raise ValueError("The number of actions must match the number of robots.")
    return [_code(mv, op) for mv, op in actions]


def encode_actions(actions, n_robots):
    """list[(move_str, op_str)] -> packed codes (move | op << 3), env.py:193-195 strings."""
    return np.array(_encode(actions, n_robots), np.uint8)


def _is_int(c):
    return isinstance(c, numbers.Integral)


def typed_reward(r, rterms, move_cost, delivery_reward, delay_reward):
    """The value env.step returns, with the reference's type (env.py:181,256,288,291): the int 0
    when no term fired, an int when every fired term's constant is integral, a float otherwise
    (any non-integral constant: Python floats, numpy floating scalars, ...; the value is the
    engine's fp64 sum)."""
    if not rterms:
        return 0
    if (rterms & MDL_RTERM_MOVE and not _is_int(move_cost)) or \
            (rterms & MDL_RTERM_ONTIME and not _is_int(delivery_reward)) or \
            (rterms & MDL_RTERM_LATE and not _is_int(delay_reward)):
        return float(r)
    return int(r)


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
    """Host mirror of one env slot of a BatchedEnv, refreshed from the mailbox rows after each
    call that touched it.  The ``robots`` / ``packages`` object lists are built on first access
    after a refresh (the state dict is built from the row arrays directly)."""

    _tot_float = False   # a float reward was added since the last reset (env.py:89,297)

    def __init__(self, owner, idx):
        self._owner = owner
        self._idx = idx

    def _set_rows(self, rob, pk, t, total):
        """rob [A, 3] / pk [P, 8] int32 rows, as arrays or as their bytes (viewed on first use).
        ``total`` is the engine's fp64 running total; its Python type follows ``_tot_float``."""
        self._rob_v = rob
        self._pk_v = pk
        self.t = int(t)
        self.total_reward = float(total) if self._tot_float else int(total)
        self._robots = None
        self._packages = None

    @property
    def _rob(self):
        v = self._rob_v
        if v.__class__ is bytes:
            v = self._rob_v = np.frombuffer(v, np.int32).reshape(-1, 3)
        return v

    @property
    def _pk(self):
        v = self._pk_v
        if v.__class__ is bytes:
            v = self._pk_v = np.frombuffer(v, np.int32).reshape(-1, 8)
        return v

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


def _rows(mb, n):
    """Copies of the first n rows of the mailbox's state outputs (the next call overwrites them)."""
    return mb["robots"][:n].copy(), mb["pkgs"][:n].copy(), mb["t"][:n].tolist(), mb["total_reward"][:n].tolist()


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
            mb = _engine.mailbox()
            _engine.mail_export(1, False)       # the constructor's layout (env.py:41)
            rob, pk, t, tot = _rows(mb, 1)
            self._set_rows(rob[0], pk[0], t[0], tot[0])
        super().__init__(_engine, _idx)
        self.engine = _engine
        self._mb = _engine.mailbox()
        self._single = _engine.E == 1
        self._ctx = _engine.mail_ctx()
        self._dev = _engine.device.index
        self.done = False
        self.state = None

    def _live_mailbox(self):
        """The engine's mailbox views, refused once the engine is closed (its host allocation
        is freed by mdl_destroy, so the views must not be written)."""
        if self.engine._h is None:
            raise RuntimeError("the environment's engine was closed")
        return self._mb

    def _call_one(self, fn):
        """One mailbox call on this env alone; refreshes this env's rows."""
        mb = self._live_mailbox()
        if not self._single:
            mb["ids"][0] = self._idx
        fn(1, not self._single)
        self._set_rows(mb["robots"][0].copy(), mb["pkgs"][0].copy(), mb["t"][0], mb["total_reward"][0])

    # env.py:81-125
    def reset(self):
        self._tot_float = False                 # env.py:89: total_reward = 0
        self._call_one(self.engine.mail_reset)
        self.done = False
        self.state = None
        return self._state_dict()

    def get_state(self):
        return self._state_dict()

    # env.py:173-306
    def step(self, actions):
        # one C call (_mdl_pack.env_step): the action codes into the mailbox, mdl_mail_step, the
        # new state dict and this env's rows out of it
        if actions.__class__ is not list and actions.__class__ is not tuple:
            actions = list(actions)
        if self.engine._h is None:
            raise RuntimeError("the environment's engine was closed")
        st, r_env, rterms, done, t, total, rob, pk = _pack().env_step(
            self._ctx, _raw_stream(self._dev), actions, self.n_robots, -1 if self._single else self._idx, self.grid)
        r = typed_reward(r_env, rterms, self.move_cost, self.delivery_reward, self.delay_reward)
        if r.__class__ is float:
            self._tot_float = True              # env.py:297: total_reward += r
        self._set_rows(rob, pk, t, total)
        infos = {}
        if done:
            infos["total_reward"] = self.total_reward
            infos["total_time_steps"] = self.t
        return st, r, done, infos

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

    def render_pygame(self, cell_size=40, window_pos=(100, 100), **kwargs):
        """Headless engine: accepts MAPPO/marl_delivery/env.py:362's signature and draws nothing."""
        return None


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
        consts = (env_kwargs.get("move_cost", -0.01), env_kwargs.get("delivery_reward", 10.),
                  env_kwargs.get("delay_reward", 1.))
        self.engine = BatchedEnv(grid_array(grid), num_envs, n_robots, n_packages, T, *consts, seeds=seeds,
                                 tracker="fresh")
        self.engine._grid_list = grid
        self.envs = [Environment(map_file, T, n_robots, n_packages, *consts, seeds[i], _engine=self.engine, _idx=i)
                     for i in range(num_envs)]
        self.num_envs = num_envs
        self._mb = self.engine.mailbox()
        self.engine.mail_export(num_envs, False)   # every env's constructor layout (env.py:41)
        self._take_rows(list(range(num_envs)))

    def _live_mailbox(self):
        if self.engine._h is None:
            raise RuntimeError("the environments' engine was closed")
        return self._mb

    def _take_rows(self, ids):
        """Refresh the envs of the last mailbox call, a reset (row k = env ids[k])."""
        rob, pk, t, tot = _rows(self._live_mailbox(), len(ids))
        for k, e in enumerate(ids):
            env = self.envs[e]
            env._tot_float = False              # env.py:89: total_reward = 0
            env._set_rows(rob[k], pk[k], t[k], tot[k])

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
        eng = self.engine
        mb = self._live_mailbox()
        if indices is None:
            eng.mail_reset(self.num_envs, False)
            self._take_rows(list(range(self.num_envs)))
            return [env._state_dict() for env in self.envs]
        idx = self._index(indices)
        out = [None] * len(idx)
        for rnd in self._rounds(idx):
            ids = [idx[p] for p in rnd]
            mb["ids"][:len(ids)] = ids
            eng.mail_reset(len(ids), True)
            self._take_rows(ids)
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
            # zip(indices, actions): ids past the end of the action list are never looked up
            idx = self._index(list(indices)[:len(actions)])
            rounds = self._rounds(idx)
            full = False
        if not idx:
            raise ValueError("not enough values to unpack (expected 4, got 0)")   # zip(*[]) in the reference
        if self.engine._h is None:
            raise RuntimeError("the environments' engine was closed")
        res = [None] * len(idx)
        env0 = self.envs[0]
        ctx, stream, grid = env0._ctx, _raw_stream(env0._dev), env0.grid
        mc, dr, lr = env0.move_cost, env0.delivery_reward, env0.delay_reward
        envs = self.envs
        for rnd in rounds:
            ids = [idx[p] for p in rnd]
            # one C call per round: codes in, mdl_mail_step, each row's state dict and rows out
            rows = _pack().vec_step(ctx, stream, [actions[p] for p in rnd], env0.n_robots, None if full else ids,
                                    grid)
            for p, e, (st, r_env, rterms, done, t, total, rob, pk) in zip(rnd, ids, rows):
                env = envs[e]
                r = typed_reward(r_env, rterms, mc, dr, lr)
                if r.__class__ is float:
                    env._tot_float = True
                env._set_rows(rob, pk, t, total)
                info = {"total_reward": env.total_reward, "total_time_steps": env.t} if done else {}
                res[p] = (st, r, done, info)
        states, rewards, dones, infos = (list(x) for x in zip(*res))
        return states, rewards, dones, infos

    def render(self, indices=None):
        return None
