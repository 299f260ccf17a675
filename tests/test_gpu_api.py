"""Argument checking at the tensor API and the dict API:
env-id subsets, caller-owned output buffers, observation ranges over mixed map
shapes, and the reference's list semantics for repeated / negative indices in
``VectorizedEnv`` (QMIX/env_vectorized.py:13-37)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from golden_io import grid  # noqa: E402


def _mg():
    import marl_gpu
    return marl_gpu


def snap(env):
    s = env.read_state()
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in s.items()}


def test_host_env_ids_checked_like_list_indexing():
    mg = _mg()
    E, A = 8, 5
    env = mg.BatchedEnv(grid("map1.txt"), E, A, 20, 50, seed=3)
    env.reset()
    acts = torch.randint(0, 15, (2, A), dtype=torch.uint8, device="cuda")
    with pytest.raises(IndexError):
        env.step(acts, env_ids=[0, 8])
    with pytest.raises(IndexError):
        env.step(acts, env_ids=[-9, 1])
    with pytest.raises(ValueError, match="duplicate"):
        env.step(acts, env_ids=[3, 3])
    with pytest.raises(IndexError):
        env.reset([E])
    with pytest.raises(TypeError):
        env.reset([0.5])
    # negative ids count from the end: [-1, 2] == [7, 2]
    twin = mg.BatchedEnv(grid("map1.txt"), E, A, 20, 50, seed=3)
    twin.reset()
    r1, _, _ = env.step(acts, env_ids=[-1, 2])
    r1 = r1.clone()
    r2, _, _ = twin.step(acts, env_ids=np.array([7, 2]))
    assert torch.equal(r1, r2)
    s1, s2 = snap(env), snap(twin)
    for k in s1:
        assert np.array_equal(s1[k], s2[k]), k
    # an empty subset is a no-op (an empty id tensor must not read as "all envs")
    before = snap(env)
    r, sh, d = env.step(torch.empty((0, A), dtype=torch.uint8, device="cuda"), env_ids=[])
    assert r.numel() == 0
    env.reset([])
    after = snap(env)
    for k in before:
        assert np.array_equal(before[k], after[k]), k


def test_device_env_ids_out_of_range_are_skipped():
    """Device-side ids are not read back on the host; an id outside [0, E) is skipped by
    the kernels instead of writing another env's (or another allocation's) memory."""
    mg = _mg()
    E, A = 8, 5
    env = mg.BatchedEnv(grid("map1.txt"), E, A, 20, 50, seed=5)
    env.reset()
    before = snap(env)
    ids = torch.tensor([E, 1 << 20, -3], dtype=torch.int32, device="cuda")
    env.step(torch.randint(0, 15, (3, A), dtype=torch.uint8, device="cuda"), env_ids=ids)
    env.reset(ids)
    env.clear_tracker(ids)
    after = snap(env)
    for k in before:
        assert np.array_equal(before[k], after[k]), k


def test_out_buffers_checked():
    mg = _mg()
    E, A = 16, 5
    env = mg.BatchedEnv(grid("map1.txt"), E, A, 20, 50, seed=1)
    env.reset()
    acts = torch.randint(0, 15, (E, A), dtype=torch.uint8, device="cuda")
    f64 = torch.zeros(E, dtype=torch.float64, device="cuda")
    f32 = torch.zeros(E, dtype=torch.float32, device="cuda")
    u8 = torch.zeros(E, dtype=torch.uint8, device="cuda")
    env.step(acts, out=(f64, f32, u8))
    with pytest.raises(TypeError):
        env.step(acts, out=(f32, f32, u8))
    with pytest.raises(ValueError, match="needs 16"):
        env.step(acts, out=(f64[:8], f32, u8))
    with pytest.raises(ValueError):
        env.step(acts, out=(f64.cpu(), f32, u8))
    with pytest.raises(ValueError):
        env.step(acts[:3])
    with pytest.raises(ValueError):
        env.step_fused(acts.view(1, E, A), out=(f64, f32, u8[:4]))


def test_obs_range_must_not_mix_map_shapes():
    mg = _mg()
    maps = [grid("map1.txt"), grid("map2.txt"), grid("map3.txt")]
    env_map = [0] * 4 + [1] * 3 + [2] * 3       # 10x10, then 20x20 (map2, map3 share a shape)
    env = mg.BatchedEnv(maps, 10, 5, 20, 50, seed=1, env_map=env_map)
    env.reset()
    with pytest.raises(ValueError, match="mix map shapes"):
        env.build_obs()                           # whole batch: 10x10 and 20x20
    with pytest.raises(ValueError, match="mix map shapes"):
        env.build_obs(2, 4)
    with pytest.raises(ValueError, match="mix map shapes"):
        env.build_obs_alt()
    a = env.build_obs(0, 4)
    assert a["actor_map"].shape == (4, 5, 6, 10, 10)
    b = env.build_obs(4, 6)                       # map2 + map3: one 20x20 run
    assert b["critic_map"].shape == (6, 4, 20, 20)
    with pytest.raises(ValueError, match="needs"):
        env.build_obs(4, 6, out=a)                # 10x10 buffers for 20x20 envs
    with pytest.raises(IndexError):
        env.build_obs(8, 5)
    # the C ABI refuses a mixed range on its own (not only the Python layer)
    lib = mg.lib()
    import ctypes as C
    rc = lib.mdl_build_obs(env._h, 0, 10, None, None, None, None, C.c_void_p(0))
    assert rc != 0 and b"mix map shapes" in lib.mdl_last_error()


def test_vectorized_env_repeated_and_negative_indices():
    """The reference steps ``self.envs[i]`` in list order: an env listed twice steps
    twice (the second result sees the first), a negative index counts from the end."""
    from marl_gpu.compat import VectorizedEnv
    kw = dict(map_file="map1.txt", n_robots=3, n_packages=10, max_time_steps=30, seed=11)
    v1 = VectorizedEnv(None, 4, **kw)
    v2 = VectorizedEnv(None, 4, **kw)
    v1.reset()
    v2.reset()
    rs = np.random.RandomState(0)
    moves, ops = ["S", "L", "R", "U", "D"], ["0", "1", "2"]
    for _ in range(10):
        acts = [[(moves[rs.randint(5)], ops[rs.randint(3)]) for _ in range(3)] for _ in range(3)]
        s1, r1, d1, i1 = v1.step(acts, indices=[2, -2, 2])
        # the same as three single-env calls in order
        want = [v2.step([acts[0]], indices=[2]), v2.step([acts[1]], indices=[2]), v2.step([acts[2]], indices=[2])]
        for k in range(3):
            assert s1[k] == want[k][0][0]
            assert r1[k] == want[k][1][0]
            assert d1[k] == want[k][2][0]
            assert i1[k] == want[k][3][0]
    with pytest.raises(IndexError):
        v1.step([[("S", "0")] * 3], indices=[4])
    # zip semantics: more indices than actions steps only as many envs as there are actions
    s, r, d, i = v1.step([[("S", "0")] * 3], indices=[0, 1])
    assert len(s) == 1
    # ... and an index past the end of the action list is never looked up (zip), even out of range
    s, r, d, i = v1.step([[("S", "0")] * 3], indices=[0, 99])
    assert len(s) == 1
    st = v1.reset(indices=[1, 1])
    assert len(st) == 2
