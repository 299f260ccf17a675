"""Host-side logic that needs no GPU: the dict API's index semantics
(QMIX/env_vectorized.py:13-37 loops over ``self.envs[i]``), the helper layer's packing
and transfer layout, and the bench's strong / weak sharding arithmetic."""
import numpy as np
import pytest

from marl_gpu import compat
from marl_gpu import helper as H
from marl_gpu import dist as D


def _venv(n):
    v = object.__new__(compat.VectorizedEnv)
    v.num_envs = n
    return v


def test_index_follows_list_indexing():
    v = _venv(4)
    assert v._index([0, 3, -1, -4]) == [0, 3, 3, 0]
    with pytest.raises(IndexError):
        v._index([4])
    with pytest.raises(IndexError):
        v._index([-5])
    with pytest.raises(TypeError):
        v._index([1.0])
    assert v._index(np.array([2, -2])) == [2, 2]


def test_rounds_keep_list_order_of_repeated_envs():
    # the k-th occurrence of an env goes to launch k; launches hold distinct envs
    idx = [2, 2, 1, 2, 0, 1]
    rounds = compat.VectorizedEnv._rounds(idx)
    assert rounds == [[0, 2, 4], [1, 5], [3]]
    for r in rounds:
        envs = [idx[p] for p in r]
        assert len(envs) == len(set(envs))
    # every position exactly once, and each env's positions in increasing launch order
    flat = sorted(p for r in rounds for p in r)
    assert flat == list(range(len(idx)))
    assert compat.VectorizedEnv._rounds([]) == []
    assert compat.VectorizedEnv._rounds([0, 1, 2]) == [[0, 1, 2]]


def test_encode_actions_codes_and_length_check():
    codes = compat.encode_actions([("S", "0"), ("L", "1"), ("R", "2"), ("U", "x"), ("D", "0"), ("?", "1")], 6)
    assert codes.tolist() == [0, 1 | 8, 2 | 16, 3 | 24, 4, 5 | 8]
    with pytest.raises(ValueError):
        compat.encode_actions([("S", "0")], 2)


def test_c_action_encoder_matches_compat():
    """The C encoder the dict-API step uses (_mdl_pack.encode / env_step / vec_step) maps every
    (move, op) the way compat._code does: the five move letters and '0'/'1'/'2', anything else
    (other strings, ints, None, str subclasses) to the no-op codes 5 / 3."""
    from marl_gpu import _mdl_pack

    class S(str):
        pass
    vals = ["S", "L", "R", "U", "D", "0", "1", "2", "3", "", "SS", "s", 1, 0, None, 2.0, S("L"), S("1")]
    rs = np.random.RandomState(3)
    for _ in range(200):
        n = int(rs.randint(0, 9))
        acts = [(vals[rs.randint(len(vals))], vals[rs.randint(len(vals))]) for _ in range(n)]
        assert _mdl_pack.encode(acts, n) == bytes(compat.encode_actions(acts, n).tolist()), acts
    with pytest.raises(ValueError):
        _mdl_pack.encode([("S", "0")], 2)
    with pytest.raises(ValueError):
        _mdl_pack.encode([("S", "0", "x")], 1)


def test_align_and_c_packer_matches_numpy_layout():
    """The helper functions' dict packer (CPython extension _mdl_pack) writes the view record
    mdl_views_features reads: [t, A, n, map] + robots 0-indexed + tracker rows in dict order."""
    assert [H._align(x) for x in (0, 1, 16, 17)] == [0, 16, 16, 32]
    rs = np.random.RandomState(2)
    for trial in range(20):
        A, n, Hh, Ww = rs.randint(1, 9), rs.randint(0, 30), rs.randint(2, 30), rs.randint(2, 30)
        robots = [(int(rs.randint(1, Hh + 1)), int(rs.randint(1, Ww + 1)), int(rs.randint(0, 5))) for _ in range(A)]
        trk = {}
        for j in rs.permutation(100)[:n]:
            trk[int(j) + 1] = dict(id=int(j) + 1, status=("in_transit", "waiting")[rs.randint(2)],
                                   start_pos=(int(rs.randint(Hh)), int(rs.randint(Ww))),
                                   target_pos=(int(rs.randint(Hh)), int(rs.randint(Ww))),
                                   start_time=int(rs.randint(50)), deadline=int(rs.randint(50, 500)))
        rows = H._tracker_rows(trk)
        want = np.concatenate([[7, A, n, 0], (np.array(robots) - [1, 1, 0]).reshape(-1),
                               rows.reshape(-1)]).astype(np.int32)
        assert np.array_equal(H.pack_view(7, robots, trk, Hh, Ww), want)        # dict, insertion order
        assert np.array_equal(H.pack_view(7, robots, rows, Hh, Ww), want)       # rows
    with pytest.raises(ValueError):
        H.pack_view(0, [(0, 1, 0)], {}, 5, 5)                                    # 1-indexed cells
    with pytest.raises(KeyError):
        H.pack_view(0, [(1, 1, 0)], {1: dict(id=1, status="waiting")}, 5, 5)     # incomplete entry


def test_pack_view_layout_and_checks():
    v = H.pack_view(7, [(1, 1, 0), (2, 3, 5)], np.array([[5, 1, 0, 0, 1, 1, 0, 9]]), 4, 4)
    assert v.dtype == np.int32
    assert v[:4].tolist() == [7, 2, 1, 0]
    assert v[4:10].tolist() == [0, 0, 0, 1, 2, 5]          # robots 0-indexed
    assert v[10:].tolist() == [5, 1, 0, 0, 1, 1, 0, 9]
    with pytest.raises(ValueError):
        H.pack_view(0, [(5, 1, 0)], np.zeros((0, 8)), 4, 4)  # robot outside the map
    with pytest.raises(ValueError):
        H.pack_view(0, [(1, 1, 0)], np.array([[1, 1, 0, 0, 7, 1, 0, 9]]), 4, 4)  # package cell outside


def test_shards_cover_every_env_once():
    for total, world in ((4096, 8), (1000, 3), (7, 8)):
        seen = []
        for r in range(world):
            ids, seeds = D.shard_strong(total, r, world, 42)
            seen += list(ids)
            assert list(seeds) == [42 + i for i in ids]
        assert sorted(seen) == list(range(total))
    ids, seeds = D.shard(4096, 3, 42)
    assert ids[0] == 3 * 4096 and len(ids) == 4096 and seeds[0] == 42 + 3 * 4096


def test_typed_reward_follows_constant_types():
    """env.py:181 ``r = 0`` plus the fired terms' constants: the int 0 when none fired, an int
    when every fired constant is integral (numpy integers included), a float otherwise --
    numpy floating constants too (np.float32 must not truncate through int())."""
    M, ON, LATE = compat.MDL_RTERM_MOVE, compat.MDL_RTERM_ONTIME, compat.MDL_RTERM_LATE
    tr = compat.typed_reward
    assert tr(0.0, 0, -0.01, 10.0, 1.0) == 0 and type(tr(0.0, 0, -0.01, 10.0, 1.0)) is int
    r = tr(-0.03, M, np.float32(-0.01), 10, 1)
    assert type(r) is float and r == -0.03
    assert type(tr(-3.0, M, np.int32(-1), 10, 1)) is int
    assert type(tr(10.0, ON, -0.01, 10, 1)) is int          # only the int constant fired
    assert type(tr(9.99, ON | M, -0.01, 10, 1)) is float
    assert type(tr(1.0, LATE, 0, 10, np.float64(1.0))) is float
    assert type(tr(1.0, LATE, 0, 10, True)) is int
