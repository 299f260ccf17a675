"""The four-envs-per-wavefront step (k_step_rows, MdlConfig.step_layout "rows") against the
one-env-per-wavefront step (k_step, "wave"): same seeds, same actions, every output and the whole
engine state (save_state: robots, packages, statuses, tracker, per-env scalars and reward-term bits,
RNG words, episode records) bit for bit after every step -- across auto-resets, in both tracker
modes, both action formats, A < 5 / A = 5 / A = 8 (numpy's 8-partial sum), P from 1 to 64 (the four package chunks per lane of the
only instantiated form, k_step_rows<.., .., 4, ..>), env counts that leave the last wave's rows empty, mixed
maps, and a done env stepped on without reset past t = 0xffff (the sentinel slots' start time).
The oracle and golden-fixture tests run this kernel too (test_gpu_parity.py: test_vs_oracle_rows_layout,
the "rows" cases of test_vs_oracle_map1 and test_mappo_rollout_golden); the default layout ("auto")
picks it for full-batch steps of >= 7,168 envs (test_rows_auto_threshold)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from golden_io import grid  # noqa: E402


def _mg():
    import marl_gpu
    return marl_gpu


def _pair(maps, E, A, P, T, **kw):
    mg = _mg()
    a = mg.BatchedEnv(maps, E, A, P, T, step_layout="wave", **kw)
    b = mg.BatchedEnv(maps, E, A, P, T, step_layout="rows", **kw)
    a.reset()
    b.reset()
    return a, b


def _run(a, b, steps, seed, fmt="int", check_every=1):
    E, A = a.E, a.A
    gen = torch.Generator(device="cuda").manual_seed(seed)
    hi = 15 if fmt == "int" else 64
    n_done = 0
    for k in range(steps):
        acts = torch.randint(0, hi, (E, A), dtype=torch.uint8, device="cuda", generator=gen)
        r1, s1, d1 = a.step(acts, action_format=fmt)
        r2, s2, d2 = b.step(acts, action_format=fmt)
        torch.cuda.synchronize()
        assert torch.equal(r1, r2), f"r_env differs at step {k}"
        assert torch.equal(s1.view(torch.int32), s2.view(torch.int32)), f"r_shaped differs at step {k}"
        assert torch.equal(d1, d2), f"done differs at step {k}"
        n_done += int(d1.sum())
        if (k + 1) % check_every == 0 or k == steps - 1:
            sa, sb = a.save_state(), b.save_state()
            if not np.array_equal(sa, sb):
                bad = np.nonzero(sa != sb)[0]
                raise AssertionError(f"state differs after step {k}: {bad.size} bytes from offset {bad[0]}")
    return n_done


@pytest.mark.parametrize("tracker", ["mappo", "fresh"])
def test_rows_equals_wave_config2(tracker):
    a, b = _pair(grid("map1.txt"), 1024, 5, 50, 40, seed=11, tracker=tracker)
    assert _run(a, b, 130, seed=1, check_every=10) > 0   # three auto-resets of every env


@pytest.mark.parametrize("A,P,E,T", [(5, 64, 257, 25), (5, 1, 130, 12), (8, 40, 301, 30), (3, 17, 66, 20),
                                     (1, 33, 99, 15), (7, 48, 203, 35), (8, 64, 128, 18), (2, 16, 5, 10)])
def test_rows_equals_wave_shapes(A, P, E, T):
    a, b = _pair(grid("map2.txt"), E, A, P, T, seed=3 + A + P, tracker="mappo")
    _run(a, b, 2 * T + 7, seed=A * 100 + P)


@pytest.mark.parametrize("mapname,A,P,E,T", [("synthetic64.txt", 5, 64, 66, 40), ("synthetic64.txt", 8, 50, 50, 30)])
def test_rows_equals_wave_large_map(mapname, A, P, E, T):
    """The 64x64 map (cells up to 63 | 63 << 8, distances up to 126)."""
    a, b = _pair(grid(mapname), E, A, P, T, seed=40 + A + P, tracker="mappo")
    _run(a, b, 2 * T + 5, seed=A * 7 + P, check_every=5)


def test_rows_equals_wave_codes_fresh():
    a, b = _pair(grid("map3.txt"), 200, 5, 30, 22, seed=5, tracker="fresh")
    _run(a, b, 50, seed=4, fmt="codes")


def test_rows_equals_wave_mixed_maps():
    maps = [grid(f"map{i}.txt") for i in range(1, 6)]
    E = 403
    env_map = np.repeat(np.arange(5), [81, 80, 81, 80, 81])
    a, b = _pair(maps, E, 5, 50, 30, seed=21, tracker="mappo", env_map=env_map)
    _run(a, b, 70, seed=8, check_every=7)


def test_rows_no_auto_reset_and_subset():
    """auto_reset off (done envs keep stepping) and a subset step in between (one wave per env)."""
    a, b = _pair(grid("map1.txt"), 300, 5, 50, 9, seed=2, tracker="mappo")
    gen = torch.Generator(device="cuda").manual_seed(6)
    ids = torch.arange(1, 300, 3, dtype=torch.int32, device="cuda")
    for k in range(30):
        acts = torch.randint(0, 15, (300, 5), dtype=torch.uint8, device="cuda", generator=gen)
        if k % 4 == 3:
            sub = acts[: ids.numel()].contiguous()
            a.step(sub, env_ids=ids)
            b.step(sub, env_ids=ids)
        else:
            r1, s1, d1 = a.step(acts, auto_reset=k < 20)
            r2, s2, d2 = b.step(acts, auto_reset=k < 20)
            assert torch.equal(r1, r2) and torch.equal(s1.view(torch.int32), s2.view(torch.int32))
            assert torch.equal(d1, d2)
        torch.cuda.synchronize()
        assert np.array_equal(a.save_state(), b.save_state()), k


def test_rows_layout_refused_where_it_does_not_apply():
    mg = _mg()
    with pytest.raises(RuntimeError):
        mg.BatchedEnv(grid("map1.txt"), 8, 9, 20, 10, step_layout="rows")
    with pytest.raises(RuntimeError):
        mg.BatchedEnv(grid("map1.txt"), 8, 5, 65, 10, step_layout="rows")
    with pytest.raises(RuntimeError):
        mg.BatchedEnv(grid("map2.txt"), 8, 16, 50, 10, step_layout="rows")
    env = mg.BatchedEnv(grid("map1.txt"), 8, 9, 20, 10)   # auto: one wave per env there
    env.reset()
    env.step(torch.zeros((8, 9), dtype=torch.uint8, device="cuda"))


def test_rows_auto_threshold():
    """auto: one wave per env below 7,168 envs, four per wave from there on; same results."""
    mg = _mg()
    small = mg.BatchedEnv(grid("map1.txt"), 7167, 5, 50, 30, seed=1)
    big = mg.BatchedEnv(grid("map1.txt"), 7168, 5, 50, 30, seed=1)
    # the engine's own decision (mdl_step_layout), and what its launches recorded (mdl_last_step_layout)
    assert small.step_layout() == "wave" and big.step_layout() == "rows"
    assert big.step_layout(n=7168) == "wave"   # an env_ids subset: always one wave per env
    assert big.last_step_layout() is None
    assert big.step_kernel_name() == "mdl::k_step_rows<true, 5, 4, 3>"
    assert small.step_kernel_name() == "mdl::k_step<true, 1, false, 5>"
    ref = mg.BatchedEnv(grid("map1.txt"), 7168, 5, 50, 30, seed=1, step_layout="wave")
    for e in (big, ref, small):
        e.reset()
    small.step(torch.zeros((7167, 5), dtype=torch.uint8, device="cuda"))
    assert small.last_step_layout() == "wave"
    gen = torch.Generator(device="cuda").manual_seed(12)
    for k in range(40):
        acts = torch.randint(0, 15, (7168, 5), dtype=torch.uint8, device="cuda", generator=gen)
        r1, s1, d1 = big.step(acts)
        assert big.last_step_layout() == "rows"
        r2, s2, d2 = ref.step(acts)
        assert ref.last_step_layout() == "wave"
        assert torch.equal(r1, r2) and torch.equal(s1.view(torch.int32), s2.view(torch.int32)) and torch.equal(d1, d2)
    big.step(torch.zeros((3, 5), dtype=torch.uint8, device="cuda"), env_ids=[0, 5, 9])
    assert big.last_step_layout() == "wave"
    ref.step(torch.zeros((3, 5), dtype=torch.uint8, device="cuda"), env_ids=[0, 5, 9])
    torch.cuda.synchronize()
    assert np.array_equal(big.save_state(), ref.save_state())


def _set_clock(env, t):
    """Every env's clock = t, through the checkpoint blob (header, then the state sections in
    mdl_save_state's order: robots, packages, state words, env records {t, rterms, total})."""
    E, A, P = env.E, env.A, env.P
    blob = env.save_state()
    pay = E * A * 4 + E * P * 8 + E * P * 2 + E * 16 + E * 624 * 4 + E * 4 + (E * P * 8 if env.tracker != "fresh"
                                                                                  else 0) + E * 8 + E * 4
    off = blob.nbytes - pay + E * A * 4 + E * P * 8 + E * P * 2
    es = blob[off:off + E * 16].view(np.uint32).reshape(E, 4)
    es[:, 0] = t
    env.load_state(blob)


@pytest.mark.parametrize("tracker", ["mappo", "fresh"])
def test_rows_sentinel_slots_past_t_65535(tracker):
    """slots without a package (j >= P) carry the sentinel start time 0xffff, so
    a done env stepped on without reset reaches t1 == 0xffff and "spawns" them.  Their state-word
    and tracker stores must stay off: the offsets of those slots name the next env's packages (or
    lie past the allocation for the last env).  Both layouts from the same state near the wrap, 12
    steps without reset: every output and the whole saved state equal, bit for bit."""
    a, b = _pair(grid("map1.txt"), 8, 5, 20, 4, seed=17, tracker=tracker)
    _run(a, b, 3, seed=2)
    for e in (a, b):
        _set_clock(e, 65530)
    assert np.array_equal(a.save_state(), b.save_state())
    gen = torch.Generator(device="cuda").manual_seed(9)
    for k in range(12):
        acts = torch.randint(0, 15, (8, 5), dtype=torch.uint8, device="cuda", generator=gen)
        r1, s1, d1 = a.step(acts, auto_reset=False)
        r2, s2, d2 = b.step(acts, auto_reset=False)
        assert b.last_step_layout() == "rows"
        torch.cuda.synchronize()
        assert torch.equal(r1, r2) and torch.equal(s1.view(torch.int32), s2.view(torch.int32)) and torch.equal(d1, d2)
        assert np.array_equal(a.save_state(), b.save_state()), f"state differs after step {k} (t = {65531 + k})"
    st = b.read_state()
    torch.cuda.synchronize()
    assert (st["t"].cpu().numpy() == 65542).all()
