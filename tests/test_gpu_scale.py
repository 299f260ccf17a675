"""GPU parity at BASELINE.json sizes and configurations (configs 2-5), mixed-map
batches, edge cases and graph capture.  Full-size runs are checked through
size-independent invariants plus exact oracle comparison of sampled envs
(envs are independent, so any subset can be replayed on the CPU)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from golden_io import grid  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    O.build()


def _mg():
    import marl_gpu
    return marl_gpu


def snap(env):
    s = env.read_state()
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in s.items()}


def check_invariants(s, g, P):
    H, W = g.shape
    rob = s["robots"]
    pk = s["pkgs"]
    E, A, _ = rob.shape
    cells = rob[:, :, 0] * W + rob[:, :, 1]
    # robots on free cells, pairwise distinct
    assert (g.reshape(-1)[cells] == 0).all()
    srt = np.sort(cells, axis=1)
    assert (np.diff(srt, axis=1) != 0).all()
    # carried ids <-> in_transit statuses
    st = pk[:, :, 7]
    for e in range(0, E, max(1, E // 256)):
        car = rob[e, :, 2]
        ids = car[car != 0]
        assert len(ids) == len(set(ids.tolist()))
        assert (st[e, ids - 1] == 2).all()
        assert set(np.nonzero(st[e] == 2)[0] + 1) == set(ids.tolist())
    # packages sorted by start time, ids 1..P, deadlines after start
    assert (np.diff(pk[:, :, 4], axis=1) >= 0).all()
    assert (pk[:, :, 6] == np.arange(1, P + 1)).all()
    assert (pk[:, :, 5] > pk[:, :, 4]).all()
    # spawn rule: waiting/in_transit/delivered only once start_time <= t
    t = s["t"][:, None]
    assert ((st == 0) == (pk[:, :, 4] > t)).all()


def test_config2_full_size_invariants_and_sampled_parity():
    """4096 envs map1 A=5 P=50 T=500, 520 steps (crosses the synchronized reset)."""
    mg = _mg()
    g = grid("map1.txt")
    E, A, P, T = 4096, 5, 50, 500
    env = mg.BatchedEnv(g, E, A, P, T, seed=42, tracker="mappo", max_packages_obs=5)
    env.reset()
    sample = np.arange(0, E, 256)
    obs = [O.OracleBatch(1, g, A, P, T, seed_base=42 + int(e), clear_on_reset=False) for e in sample]
    gen = np.random.RandomState(11)
    totals = np.zeros(E)
    for k in range(520):
        ints = gen.randint(0, 15, size=(E, A)).astype(np.uint8)
        r, sh, d = env.step(torch.from_numpy(ints).cuda())
        rh, shh, dh = r.cpu().numpy(), sh.cpu().numpy(), d.cpu().numpy().astype(bool)
        for i, e in enumerate(sample):
            r0, s0, d0 = obs[i].step(ints[e:e + 1], auto_reset=True, consts=O.MAPPO_CONSTS)
            assert rh[e] == r0[0] and shh[e] == s0[0] and dh[e] == d0[0], (k, e)
        totals = np.where(dh, 0.0, totals + rh)
        if k % 65 == 0 or k == 519:
            s = snap(env)
            check_invariants(s, g, P)
            np.testing.assert_array_equal(s["total_reward"], totals)
    assert k >= T   # the episode boundary was crossed
    env.close()


def test_config3_full_size_obs_sampled():
    """16384 envs: observation tensors of sampled envs equal the oracle's."""
    mg = _mg()
    g = grid("map1.txt")
    E, A, P, T = 16384, 5, 50, 500
    env = mg.BatchedEnv(g, E, A, P, T, seed=42, tracker="mappo", max_other_robots=4, max_packages_obs=5)
    env.reset()
    sample = np.arange(0, E, 1024)
    obs = [O.OracleBatch(1, g, A, P, T, seed_base=42 + int(e), clear_on_reset=False) for e in sample]
    gen = np.random.RandomState(5)
    bufs = env.obs_buffers()
    for k in range(40):
        ints = gen.randint(0, 15, size=(E, A)).astype(np.uint8)
        env.step(torch.from_numpy(ints).cuda())
        for i, e in enumerate(sample):
            obs[i].step(ints[e:e + 1], auto_reset=True, consts=O.MAPPO_CONSTS)
        if k % 13 == 0:
            env.build_obs(out=bufs)
            o = {kk: v.cpu().numpy() for kk, v in bufs.items()}
            for i, e in enumerate(sample):
                oe, ot = obs[i].env(0), obs[i].tracker(0)
                st, rb1, rows = oe.state(), oe.robots1(), ot.rows()
                av = np.stack([O.generate_vector_features(10, 10, st["t"], rb1, rows, a, T, 4, 5) for a in range(A)])
                am = np.stack([O.convert_observation(g, st["t"], rb1, rows, a) for a in range(A)])
                gm, gv = O.convert_global_state(g, st["t"], rb1, rows, T, 100, 100)
                np.testing.assert_array_equal(o["actor_vec"][e], av)
                np.testing.assert_array_equal(o["actor_map"][e], am)
                np.testing.assert_array_equal(o["critic_map"][e], gm)
                np.testing.assert_array_equal(o["critic_vec"][e], gv)
    env.close()


def test_config4_mixed_maps():
    """map1..map5 in one batch, contiguous groups; obs per group."""
    mg = _mg()
    names = ["map1.txt", "map2.txt", "map3.txt", "map4.txt", "map5.txt"]
    grids = [grid(n) for n in names]
    per = 6
    E, A, P, T = per * 5, 5, 30, 50
    env_map = np.repeat(np.arange(5), per)
    env = mg.BatchedEnv(grids, E, A, P, T, seed=42, env_map=env_map, tracker="mappo", max_other_robots=4,
                        max_packages_obs=5, max_robots_state=10, max_packages_state=20)
    env.reset()
    batches = [O.OracleBatch(per, grids[m], A, P, T, seed_base=42 + m * per, clear_on_reset=False) for m in range(5)]
    gen = np.random.RandomState(2)
    for k in range(110):
        ints = gen.randint(0, 15, size=(E, A)).astype(np.uint8)
        r, sh, d = env.step(torch.from_numpy(ints).cuda())
        for m in range(5):
            r0, s0, d0 = batches[m].step(ints[m * per:(m + 1) * per], auto_reset=True, consts=O.MAPPO_CONSTS)
            np.testing.assert_array_equal(r.cpu().numpy()[m * per:(m + 1) * per], r0)
            np.testing.assert_array_equal(sh.cpu().numpy()[m * per:(m + 1) * per], s0)
        if k % 27 == 0:
            for m in range(5):
                o = env.build_obs(env_begin=m * per, n=per)
                av = o["actor_vec"].cpu().numpy()
                cv = o["critic_vec"].cpu().numpy()
                cm = o["critic_map"].cpu().numpy()
                H, W = grids[m].shape
                for e in range(per):
                    oe, ot = batches[m].env(e), batches[m].tracker(e)
                    st, rb1, rows = oe.state(), oe.robots1(), ot.rows()
                    want = np.stack([O.generate_vector_features(H, W, st["t"], rb1, rows, a, T, 4, 5)
                                     for a in range(A)])
                    np.testing.assert_array_equal(av[e], want)
                    gm, gv = O.convert_global_state(grids[m], st["t"], rb1, rows, T, 10, 20)
                    np.testing.assert_array_equal(cv[e], gv)
                    np.testing.assert_array_equal(cm[e], gm)
    env.close()


def test_config5_synthetic_sampled():
    """64x64 map, A=16, P=100: 2048 envs, sampled oracle replay + invariants."""
    mg = _mg()
    g = grid("synthetic64.txt")
    E, A, P, T = 2048, 16, 100, 60
    env = mg.BatchedEnv(g, E, A, P, T, seed=7, tracker="mappo", max_other_robots=15, max_packages_obs=20,
                        max_robots_state=16, max_packages_state=100)
    env.reset()
    sample = np.arange(0, E, 512)
    obs = [O.OracleBatch(1, g, A, P, T, seed_base=7 + int(e), clear_on_reset=False) for e in sample]
    gen = np.random.RandomState(9)
    for k in range(70):
        ints = gen.randint(0, 15, size=(E, A)).astype(np.uint8)
        r, sh, d = env.step(torch.from_numpy(ints).cuda())
        rh, shh = r.cpu().numpy(), sh.cpu().numpy()
        for i, e in enumerate(sample):
            r0, s0, d0 = obs[i].step(ints[e:e + 1], auto_reset=True, consts=O.MAPPO_CONSTS)
            assert rh[e] == r0[0] and shh[e] == s0[0], (k, e)
    check_invariants(snap(env), g, P)
    o = env.build_obs(env_begin=0, n=4)
    av = o["actor_vec"].cpu().numpy()
    st, rb1, rows = obs[0].env(0).state(), obs[0].env(0).robots1(), obs[0].tracker(0).rows()
    want = np.stack([O.generate_vector_features(64, 64, st["t"], rb1, rows, a, T, 15, 20) for a in range(A)])
    np.testing.assert_array_equal(av[0], want)
    env.close()


def test_edge_cases_vs_oracle():
    mg = _mg()
    cases = [("map1.txt", 1, 1, 5), ("map.txt", 2, 3, 2), ("map1.txt", 5, 6, 3), ("map2.txt", 20, 80, 7)]
    for m, A, P, T in cases:
        g = grid(m)
        E = 8
        env = mg.BatchedEnv(g, E, A, P, T, seed=3, tracker="mappo")
        env.reset()
        ob = O.OracleBatch(E, g, A, P, T, seed_base=3, clear_on_reset=False)
        gen = np.random.RandomState(1)
        for k in range(3 * T + 5):
            ints = gen.randint(0, 256, size=(E, A)).astype(np.uint8)   # >= 15: op clamp to 0
            r, sh, d = env.step(torch.from_numpy(ints).cuda())
            r0, s0, d0 = ob.step(ints, auto_reset=True, consts=O.MAPPO_CONSTS)
            np.testing.assert_array_equal(r.cpu().numpy(), r0)
            np.testing.assert_array_equal(sh.cpu().numpy(), s0)
            np.testing.assert_array_equal(d.cpu().numpy().astype(bool), d0)
        env.close()


def test_step_past_done_without_reset():
    """t keeps rising after done; done is recomputed (IDQ relies on it)."""
    mg = _mg()
    g = grid("map1.txt")
    env = mg.BatchedEnv(g, 4, 5, 10, 6, seed=1, tracker="fresh")
    env.reset()
    envs = [O.OracleEnv(g, 5, 10, 6, seed=1 + i) for i in range(4)]
    for e in envs:
        e.reset()
    gen = np.random.RandomState(4)
    mv_codes = np.array([4, 1, 2, 0, 3], np.uint8)
    for k in range(15):
        ints = gen.randint(0, 15, size=(4, 5)).astype(np.uint8)
        r, sh, d = env.step(torch.from_numpy(ints).cuda(), auto_reset=False)
        for i, oe in enumerate(envs):
            r0, _, d0 = oe.step(mv_codes[ints[i] % 5], np.where(ints[i] // 5 >= 3, 0, ints[i] // 5).astype(np.uint8))
            assert float(r.cpu()[i]) == r0 and bool(d.cpu()[i]) == d0
    s = snap(env)
    assert (s["t"] == 15).all()


def test_graph_capture_matches_eager():
    mg = _mg()
    g = grid("map1.txt")
    E, A = 256, 5
    a = mg.BatchedEnv(g, E, A, 50, 40, seed=9, tracker="mappo")
    b = mg.BatchedEnv(g, E, A, 50, 40, seed=9, tracker="mappo")
    a.reset()
    b.reset()
    acts = torch.randint(0, 15, (30, E, A), device="cuda", dtype=torch.int32).to(torch.uint8)
    ra = torch.zeros(30, E, dtype=torch.float64, device="cuda")
    sa = torch.zeros(30, E, dtype=torch.float32, device="cuda")
    da = torch.zeros(30, E, dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        with torch.cuda.graph(graph, stream=st):
            for k in range(30):
                a.step(acts[k], out=(ra[k], sa[k], da[k]))
    torch.cuda.synchronize()
    for rep in range(3):
        graph.replay()
        torch.cuda.synchronize()
        for k in range(30):
            r, s, d = b.step(acts[k])
            assert torch.equal(r, ra[k]) and torch.equal(s, sa[k]) and torch.equal(d, da[k]), (rep, k)
    sa_, sb_ = snap(a), snap(b)
    for key in sa_:
        np.testing.assert_array_equal(sa_[key], sb_[key])


def test_compat_vectorized_indices():
    """QMIX/env_vectorized.py indices= semantics through the compat layer."""
    from marl_gpu.compat import VectorizedEnv
    ve = VectorizedEnv(None, 3, map_file="map1.txt", n_robots=5, n_packages=10, max_time_steps=20, seed=7)
    states = ve.reset()
    envs = [O.OracleEnv(grid("map1.txt"), 5, 10, 20, seed=7 + i) for i in range(3)]
    for e in envs:
        e.reset()
    for s, e in zip(states, envs):
        assert [r[:2] for r in s["robots"]] == [tuple(x) for x in (e.state()["robots"][:, :2] + 1).tolist()]
    gen = np.random.RandomState(0)
    for k in range(25):
        idx = [0, 2] if k % 2 else [1]
        acts = [[("SLRUD"[gen.randint(5)], "012"[gen.randint(3)]) for _ in range(5)] for _ in idx]
        st, rw, dn, inf = ve.step(acts, idx)
        for j, i in enumerate(idx):
            mv = np.array([{"S": 0, "L": 1, "R": 2, "U": 3, "D": 4}[m] for m, _ in acts[j]], np.uint8)
            op = np.array([int(o) for _, o in acts[j]], np.uint8)
            r0, _, d0 = envs[i].step(mv, op)
            assert rw[j] == r0 and dn[j] == d0
            assert [r[:2] for r in st[j]["robots"]] == [tuple(x) for x in (envs[i].state()["robots"][:, :2] + 1).tolist()]


@pytest.mark.parametrize("mapname,A,P,MO,MP", [("map4.txt", 5, 300, 4, 20), ("map2.txt", 8, 1024, 100, 100)])
def test_obs_large_package_tables(mapname, A, P, MO, MP):
    """The general observation builder (P > 64) up to MDL_MAX_PACKAGES vs the oracle."""
    mg = _mg()
    g = grid(mapname)
    H, W = g.shape
    E, T = 8, 60
    env = mg.BatchedEnv(g, E, A, P, T, seed=21, tracker="mappo", max_other_robots=MO, max_packages_obs=MP)
    env.reset()
    ob = O.OracleBatch(E, g, A, P, T, seed_base=21, clear_on_reset=False)
    gen = np.random.RandomState(8)
    bufs = env.obs_buffers()
    for k in range(25):
        ints = gen.randint(0, 15, size=(E, A)).astype(np.uint8)
        env.step(torch.from_numpy(ints).cuda())
        ob.step(ints, auto_reset=True, consts=O.MAPPO_CONSTS)
        if k % 12 == 0:
            env.build_obs(out=bufs)
            o = {kk: v.cpu().numpy() for kk, v in bufs.items()}
            for e in range(E):
                oe, ot = ob.env(e), ob.tracker(e)
                st, rb1, rows = oe.state(), oe.robots1(), ot.rows()
                av = np.stack([O.generate_vector_features(H, W, st["t"], rb1, rows, a, T, MO, MP) for a in range(A)])
                am = np.stack([O.convert_observation(g, st["t"], rb1, rows, a) for a in range(A)])
                gm, gv = O.convert_global_state(g, st["t"], rb1, rows, T, 100, 100)
                np.testing.assert_array_equal(o["actor_vec"][e], av, f"avec env {e} step {k}")
                np.testing.assert_array_equal(o["actor_map"][e], am, f"amap env {e} step {k}")
                np.testing.assert_array_equal(o["critic_map"][e], gm, f"cmap env {e} step {k}")
                np.testing.assert_array_equal(o["critic_vec"][e], gv, f"cvec env {e} step {k}")
    env.close()


@pytest.mark.parametrize("tracker", ["mappo", "fresh"])
def test_config5_obs_chunk_4096_vs_oracle(tracker):
    """The config-5 observation builder (general k_obs: 64x64 bit rows, staged actor vectors) at the
    4,096-env chunk size it is benchmarked at, where several waves share each workgroup's LDS, after
    one auto-reset (T = 60, 70 steps): all four tensors of 16 envs spread over workgroups and XCD
    slots, bit for bit against convert_observation / generate_vector_features /
    convert_global_state (MAPPO/helper.py:6-255) on the oracle's state and tracker (VERDICT r04
    item 6).  The fresh tracker equals env truth; the MAPPO one keeps an episode's leftovers."""
    mg = _mg()
    g = grid("synthetic64.txt")
    E, A, P, T = 4096, 16, 100, 60
    MO, MP, MR, MPs = 15, 20, 16, 100
    env = mg.BatchedEnv(g, E, A, P, T, seed=7, tracker=tracker, max_other_robots=MO, max_packages_obs=MP,
                        max_robots_state=MR, max_packages_state=MPs)
    env.reset()
    sample = np.array([0, 1, 2, 3, 257, 511, 1023, 1024, 1501, 2047, 2048, 2731, 3071, 3584, 4094, 4095])
    obs = [O.OracleBatch(1, g, A, P, T, seed_base=7 + int(e), clear_on_reset=(tracker == "fresh")) for e in sample]
    gen = np.random.RandomState(21)
    dones = 0
    for k in range(70):
        ints = gen.randint(0, 15, size=(E, A)).astype(np.uint8)
        r, sh, d = env.step(torch.from_numpy(ints).cuda())
        dones += int(d.sum().item())
        for i, e in enumerate(sample):
            obs[i].step(ints[e:e + 1], auto_reset=True, consts=O.MAPPO_CONSTS)
    assert dones == E   # every env crossed its reset at t = T
    o = env.build_obs(0, E)
    idx = torch.from_numpy(sample).cuda()
    am, av, cm, cv = (o[k].index_select(0, idx).cpu().numpy()
                      for k in ("actor_map", "actor_vec", "critic_map", "critic_vec"))
    del o
    for i, e in enumerate(sample):
        oe, ot = obs[i].env(0), obs[i].tracker(0)
        st, rb1, rows = oe.state(), oe.robots1(), ot.rows()
        for a in range(A):
            np.testing.assert_array_equal(am[i, a], O.convert_observation(g, st["t"], rb1, rows, a),
                                          err_msg=f"actor map env {e} agent {a}")
            np.testing.assert_array_equal(av[i, a], O.generate_vector_features(64, 64, st["t"], rb1, rows, a, T, MO, MP),
                                          err_msg=f"actor vec env {e} agent {a}")
        gm, gv = O.convert_global_state(g, st["t"], rb1, rows, T, MR, MPs)
        np.testing.assert_array_equal(cm[i], gm, err_msg=f"critic map env {e}")
        np.testing.assert_array_equal(cv[i], gv, err_msg=f"critic vec env {e}")
    env.close()
