"""The two-envs-per-wavefront step (k_step_halves, MdlConfig.step_layout "halves": one env per
32-lane half, A == 16, P <= 128) against the one-env-per-wavefront step (k_step, "wave") and the
oracle: same seeds, same actions, every output and the whole engine state (save_state: robots,
packages, statuses, tracker, per-env scalars and reward-term bits, RNG words, episode records) bit
for bit after every step -- across auto-resets, in both tracker modes, both action formats, P from 1
to 128 (all four 32-lane package chunks), odd env counts (the last wave's second half empty), mixed
maps, steps without auto-reset, a done env stepped past t = 0xffff (the sentinel slots' start time),
and BASELINE config 5's shape (64x64 map, 16 robots, 100 packages) against the oracle directly
(env.py:173-316, MAPPO/helper.py:257-369, MAPPO/trainer.py:95-130,211-259)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from golden_io import grid  # noqa: E402
from test_gpu_step_rows import _run, _set_clock  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    O.build()


def _pair(maps, E, A, P, T, **kw):
    import marl_gpu as mg
    a = mg.BatchedEnv(maps, E, A, P, T, step_layout="wave", **kw)
    b = mg.BatchedEnv(maps, E, A, P, T, step_layout="halves", **kw)
    a.reset()
    b.reset()
    assert b.step_layout() == "halves" and b.step_kernel_name().startswith("mdl::k_step_halves<")
    return a, b


@pytest.mark.parametrize("tracker", ["mappo", "fresh"])
def test_halves_equals_wave_config5_shape(tracker):
    """The 64x64 synthetic map with 16 robots and 100 packages, three auto-resets of every env."""
    a, b = _pair(grid("synthetic64.txt"), 515, 16, 100, 30, seed=7, tracker=tracker)
    assert _run(a, b, 100, seed=3, check_every=10) > 0
    assert b.last_step_layout() == "halves"


@pytest.mark.parametrize("P,E,T", [(1, 31, 12), (17, 64, 20), (32, 33, 18), (33, 96, 25), (64, 129, 22),
                                   (100, 250, 35), (128, 61, 30)])
def test_halves_equals_wave_shapes(P, E, T):
    a, b = _pair(grid("map3.txt"), E, 16, P, T, seed=5 + P, tracker="mappo")
    _run(a, b, 2 * T + 7, seed=P)


def test_halves_equals_wave_codes_fresh():
    a, b = _pair(grid("map2.txt"), 200, 16, 50, 22, seed=9, tracker="fresh")
    _run(a, b, 50, seed=4, fmt="codes")


def test_halves_equals_wave_mixed_maps():
    maps = [grid("synthetic64.txt")] + [grid(f"map{i}.txt") for i in (2, 3, 4)]
    E = 301
    env_map = np.repeat(np.arange(4), [75, 76, 75, 75])
    a, b = _pair(maps, E, 16, 100, 30, seed=21, tracker="mappo", env_map=env_map)
    _run(a, b, 70, seed=8, check_every=7)


def test_halves_no_auto_reset_and_subset():
    """auto_reset off (done envs keep stepping) and a subset step in between (one wave per env)."""
    a, b = _pair(grid("synthetic64.txt"), 130, 16, 100, 9, seed=2, tracker="mappo")
    gen = torch.Generator(device="cuda").manual_seed(6)
    ids = torch.arange(1, 130, 3, dtype=torch.int32, device="cuda")
    for k in range(30):
        acts = torch.randint(0, 15, (130, 16), dtype=torch.uint8, device="cuda", generator=gen)
        if k % 4 == 3:
            sub = acts[: ids.numel()].contiguous()
            a.step(sub, env_ids=ids)
            b.step(sub, env_ids=ids)
            assert b.last_step_layout() == "wave"
        else:
            r1, s1, d1 = a.step(acts, auto_reset=k < 20)
            r2, s2, d2 = b.step(acts, auto_reset=k < 20)
            assert torch.equal(r1, r2) and torch.equal(s1.view(torch.int32), s2.view(torch.int32))
            assert torch.equal(d1, d2)
        torch.cuda.synchronize()
        assert np.array_equal(a.save_state(), b.save_state()), k


@pytest.mark.parametrize("tracker", ["mappo", "fresh"])
def test_halves_sentinel_slots_past_t_65535(tracker):
    """Slots j >= P carry the sentinel start time 0xffff: stepping a done env on without reset
    across t = 0xffff must not store them (their offsets name the next env's slots)."""
    a, b = _pair(grid("synthetic64.txt"), 7, 16, 40, 4, seed=17, tracker=tracker)
    _run(a, b, 3, seed=2)
    for e in (a, b):
        _set_clock(e, 65530)
    gen = torch.Generator(device="cuda").manual_seed(9)
    for k in range(12):
        acts = torch.randint(0, 15, (7, 16), dtype=torch.uint8, device="cuda", generator=gen)
        r1, s1, d1 = a.step(acts, auto_reset=False)
        r2, s2, d2 = b.step(acts, auto_reset=False)
        torch.cuda.synchronize()
        assert torch.equal(r1, r2) and torch.equal(s1.view(torch.int32), s2.view(torch.int32)) and torch.equal(d1, d2)
        assert np.array_equal(a.save_state(), b.save_state()), f"state differs after step {k}"


def test_halves_layout_refused_where_it_does_not_apply():
    import marl_gpu as mg
    for A, P in ((15, 50), (8, 50), (16, 129)):
        with pytest.raises(RuntimeError):
            mg.BatchedEnv(grid("map2.txt"), 8, A, P, 10, step_layout="halves")


@pytest.mark.parametrize("tracker", ["mappo", "fresh"])
def test_halves_vs_oracle_config5(tracker):
    """BASELINE config 5's env (64x64, 16 robots, 100 packages) on the halves layout against the
    oracle's literal restatement: 24 envs, 140 steps across two auto-resets (T = 60)."""
    import marl_gpu as mg
    g = grid("synthetic64.txt")
    E, A, P, T = 24, 16, 100, 60
    env = mg.BatchedEnv(g, E, A, P, T, seed=7, tracker=tracker, step_layout="halves")
    env.reset()
    ob = O.OracleBatch(E, g, A, P, T, seed_base=7, clear_on_reset=(tracker == "fresh"))
    gen = np.random.RandomState(19)
    for k in range(140):
        ints = gen.randint(0, 15, size=(E, A)).astype(np.uint8)
        r, sh, d = env.step(torch.from_numpy(ints).cuda())
        r0, s0, d0 = ob.step(ints, auto_reset=True, consts=O.MAPPO_CONSTS)
        np.testing.assert_array_equal(r.cpu().numpy(), r0, err_msg=f"r_env step {k}")
        np.testing.assert_array_equal(sh.cpu().numpy(), s0, err_msg=f"shaped step {k}")
        np.testing.assert_array_equal(d.cpu().numpy().astype(bool), d0, err_msg=f"done step {k}")
        if k % 35 == 34:
            s = env.read_state()
            torch.cuda.synchronize()
            s = {kk: v.cpu().numpy() for kk, v in s.items()}
            for e in range(E):
                os_ = ob.env(e).state()
                np.testing.assert_array_equal(s["robots"][e], os_["robots"], err_msg=f"robots env {e} step {k}")
                np.testing.assert_array_equal(s["pkgs"][e], os_["pkgs"], err_msg=f"pkgs env {e} step {k}")
                assert s["t"][e] == os_["t"] and s["total_reward"][e] == os_["total_reward"]
                np.testing.assert_array_equal(env.tracker_rows(s, e), ob.tracker(e).rows(), err_msg=f"tracker env {e}")
    env.close()


def test_halves_auto_threshold():
    """auto: one wave per env below 12,288 envs, two per wave from there on (A == 16, P <= 128) -- the
    engine's own decision (mdl_step_layout) and what its launches record; same results."""
    import marl_gpu as mg
    g = grid("synthetic64.txt")
    small = mg.BatchedEnv(g, 12287, 16, 100, 20, seed=1)
    big = mg.BatchedEnv(g, 12288, 16, 100, 20, seed=1)
    assert small.step_layout() == "wave" and big.step_layout() == "halves"
    assert mg.BatchedEnv(g, 20000, 16, 129, 20, seed=1).step_layout() == "wave"   # P > 128
    ref = mg.BatchedEnv(g, 12288, 16, 100, 20, seed=1, step_layout="wave")
    for e in (big, ref):
        e.reset()
    gen = torch.Generator(device="cuda").manual_seed(13)
    for k in range(25):
        acts = torch.randint(0, 15, (12288, 16), dtype=torch.uint8, device="cuda", generator=gen)
        r1, s1, d1 = big.step(acts)
        assert big.last_step_layout() == "halves"
        r2, s2, d2 = ref.step(acts)
        assert torch.equal(r1, r2) and torch.equal(s1.view(torch.int32), s2.view(torch.int32)) and torch.equal(d1, d2)
    torch.cuda.synchronize()
    assert np.array_equal(big.save_state(), ref.save_state())
