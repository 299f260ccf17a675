"""GPU parity: the HIP engine (through the C ABI) against the reference's
golden fixtures and the CPU oracle.  Bit-exact for every integer/index value
and every reward (fp64 env reward, float32 shaped reward); observation
features are exact float32 values (0/1 and single int/int divisions)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from golden_io import decode_trainer, grid, load_json, meta, npz  # noqa: E402


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


# ------------------------------------------------------------------ reset
def test_reset_layouts_golden():
    mg = _mg()
    d = npz("reset.npz")
    cases = meta(d)
    groups = {}
    for i, c in enumerate(cases):
        groups.setdefault((c["map"], c["A"], c["P"], c["T"]), []).append(i)
    for (m, A, P, T), idxs in groups.items():
        seeds = [cases[i]["seed"] for i in idxs]
        env = mg.BatchedEnv(grid(m), len(seeds), A, P, T, seeds=seeds, tracker="fresh")
        for k in range(3):
            if k:
                env.reset()
            s = snap(env)
            for e, i in enumerate(idxs):
                np.testing.assert_array_equal(s["robots"][e, :, :2], d[f"robots_{i}"][k], err_msg=f"{cases[i]} draw {k}")
                np.testing.assert_array_equal(s["pkgs"][e, :, :6], d[f"pkgs_{i}"][k], err_msg=f"{cases[i]} draw {k}")
                assert (s["t"] == 0).all()
        env.close()


# ------------------------------------------------------------------ steps
def test_step_traces_golden():
    mg = _mg()
    d = npz("steps.npz")
    for ci, c in enumerate(meta(d)):
        env = mg.BatchedEnv(grid(c["map"]), 1, c["A"], c["P"], c["T"], seeds=[c["seed"]], tracker="fresh")
        env.reset()
        s = snap(env)
        np.testing.assert_array_equal(s["robots"][0, :, :2], d[f"pos0_{ci}"])
        acts = d[f"acts_{ci}"]
        codes = torch.from_numpy((acts[:, :, 0] | (acts[:, :, 1] << 3)).astype(np.uint8)).cuda()
        for k in range(c["n"]):
            r, sh, dn = env.step(codes[k:k + 1], auto_reset=c["auto_reset"], action_format="codes")
            s = snap(env)
            assert float(r.cpu()[0]) == d[f"r_{ci}"][k], (c, k)
            assert bool(dn.cpu()[0]) == d[f"done_{ci}"][k], (c, k)
            if not (d[f"done_{ci}"][k] and c["auto_reset"]):
                assert s["t"][0] == d[f"t_{ci}"][k] and s["total_reward"][0] == d[f"total_{ci}"][k], (c, k)
            np.testing.assert_array_equal(s["robots"][0, :, :2], d[f"pos_{ci}"][k], err_msg=f"{c} step {k}")
            np.testing.assert_array_equal(s["robots"][0, :, 2], d[f"carry_{ci}"][k], err_msg=f"{c} step {k}")
            np.testing.assert_array_equal(s["pkgs"][0, :, 7], d[f"status_{ci}"][k], err_msg=f"{c} step {k}")
            np.testing.assert_array_equal(s["pkgs"][0, :, :6], d[f"pkgs_{ci}"][k], err_msg=f"{c} step {k}")
        env.close()


# ---------------------------------------------------------- MAPPO rollout
def _check_obs(o, d, k, map_steps, pre="", big=None):
    np.testing.assert_array_equal(o["actor_vec"], d["avec"][k], err_msg=f"{pre} avec step {k}")
    np.testing.assert_array_equal(o["critic_vec"], d["cvec"][k], err_msg=f"{pre} cvec step {k}")
    if k in map_steps:
        j = map_steps.index(k)
        np.testing.assert_array_equal(o["actor_map"], d["amap"][j], err_msg=f"{pre} amap step {k}")
        np.testing.assert_array_equal(o["critic_map"], d["cmap"][j], err_msg=f"{pre} cmap step {k}")


@pytest.mark.parametrize("layout", ["wave", "rows"])
@pytest.mark.parametrize("tag", ["mappo", "mappo_map2", "mappo_syn64"])
def test_mappo_rollout_golden(tag, layout):
    """The reference's MAPPO rollout, through both step layouts (rows: four envs per wavefront,
    where A <= 8 and P <= 64)."""
    mg = _mg()
    d = npz(f"rollout_{tag}.npz")
    m = meta(d)
    E, A, P, T = m["E"], m["A"], m["P"], m["T"]
    if layout == "rows" and (A > 8 or P > 64):
        pytest.skip("the rows layout needs A <= 8 and P <= 64")
    kw = dict(seed=m["seed"], tracker="mappo", shaping="mappo", step_layout=layout)
    env = mg.BatchedEnv(grid(m["map"]), E, A, P, T, max_other_robots=m["MO"], max_packages_obs=m["MP"],
                        max_robots_state=m["MR"], max_packages_state=m["MPs"], **kw)
    envq = mg.BatchedEnv(grid(m["map"]), E, A, P, T, max_other_robots=m["MO"], max_packages_obs=m["MP"],
                         max_robots_state=10, max_packages_state=20, **kw)
    envb = mg.BatchedEnv(grid(m["map"]), E, A, P, T, max_other_robots=100, max_packages_obs=100,
                         max_robots_state=1, max_packages_state=1, **kw)
    for x in (env, envq, envb):
        x.reset()
    map_steps = list(d["map_steps"])
    big_steps = list(d["big_steps"])

    def check(k):
        o = {kk: v.cpu().numpy() for kk, v in env.build_obs().items()}
        _check_obs(o, d, k, map_steps, tag)
        oq = envq.build_obs(which=("critic_vec",))["critic_vec"].cpu().numpy()
        np.testing.assert_array_equal(oq, d["cvec_qmix"][k], err_msg=f"cvec_qmix step {k}")
        if k in big_steps:
            ob = envb.build_obs(which=("actor_vec",))["actor_vec"].cpu().numpy()
            np.testing.assert_array_equal(ob, d["avec_big"][big_steps.index(k)], err_msg=f"avec_big step {k}")

    check(0)
    for k in range(d["acts"].shape[0]):
        a = torch.from_numpy(d["acts"][k].astype(np.uint8)).cuda()
        r, sh, dn = env.step(a, auto_reset=True)
        envq.step(a, auto_reset=True)
        envb.step(a, auto_reset=True)
        np.testing.assert_array_equal(r.cpu().numpy(), d["r_env"][k], err_msg=f"r_env step {k}")
        np.testing.assert_array_equal(sh.cpu().numpy(), d["r_shaped"][k], err_msg=f"r_shaped step {k}")
        np.testing.assert_array_equal(dn.cpu().numpy().astype(bool), d["done"][k], err_msg=f"done step {k}")
        check(k + 1)
    for x in (env, envq, envb):
        x.close()


# ----------------------------------------------------------- QMIX rollout
def test_qmix_rollout_golden():
    mg = _mg()
    d = npz("rollout_qmix.npz")
    m = meta(d)
    E, A, P, T = m["E"], m["A"], m["P"], m["T"]
    env = mg.BatchedEnv(grid(m["map"]), E, A, P, T, seed=m["seed"], tracker="fresh", shaping="qmix",
                        max_other_robots=m["MO"], max_packages_obs=m["MP"], max_robots_state=m["MR"],
                        max_packages_state=m["MPs"])
    env.reset()
    for k in range(d["active"].shape[0]):
        active = d["active"][k]
        if not active.any():
            env.reset()
        else:
            idx = np.nonzero(active)[0]
            a = torch.from_numpy(d["acts"][k][idx].astype(np.uint8)).cuda()
            r, sh, dn = env.step(a, env_ids=idx.tolist(), auto_reset=False)
            np.testing.assert_array_equal(r.cpu().numpy(), d["r"][k][idx])
            np.testing.assert_array_equal(dn.cpu().numpy().astype(bool), d["done"][k][idx])
            np.testing.assert_array_equal(sh.cpu().numpy(), d["sh"][k][idx], err_msg=f"shaped row {k}")
        o = {kk: v.cpu().numpy() for kk, v in env.build_obs().items()}
        np.testing.assert_array_equal(o["actor_vec"], d["avec"][k], err_msg=f"avec row {k}")
        np.testing.assert_array_equal(o["critic_vec"], d["cvec"][k], err_msg=f"cvec row {k}")
        np.testing.assert_array_equal(o["actor_map"], d["amap"][k], err_msg=f"amap row {k}")
    env.close()


# ------------------------------------------------------ helper dict inputs
def test_helper_dict_cases_golden():
    from marl_gpu import helper as Hm
    d = npz("helpers.npz")
    for i, c in enumerate(meta(d)):
        g = grid(c["map"]).tolist()
        rows = d[f"trk_{i}"]
        state = {"time_step": c["t"], "map": g, "robots": [tuple(x) for x in d[f"robots_{i}"]], "packages": []}
        out = Hm.features(state, rows, [c["idx"]], c["T"], c["MO"], c["MP"], c["MR"], c["MPs"])
        np.testing.assert_array_equal(out["obs"][0], d[f"obs_{i}"], err_msg=str(c))
        np.testing.assert_array_equal(out["vec"][0], d[f"vec_{i}"], err_msg=str(c))
        np.testing.assert_array_equal(out["gmap"][0], d[f"gmap_{i}"], err_msg=str(c))
        np.testing.assert_array_equal(out["gvec"][0], d[f"gvec_{i}"], err_msg=str(c))
        acts = d[f"acts_{i}"]
        codes = (acts[:, 0] | (acts[:, 1] << 3)).astype(np.uint8)
        g0 = 0 if c["g_int"] else c["g"]
        for j, consts in enumerate((Hm.MAPPO_SHAPING, Hm.QMIX_SHAPING)):
            sh = Hm.shaped_rewards_views(g0, c["t"], d[f"robots_{i}"], c["t"] + 1, d[f"cur_robots_{i}"], codes, rows,
                                         g, consts)
            assert sh.tobytes() == d[f"sh_{i}"][j].tobytes(), (i, c, j)


def test_helper_public_functions_golden():
    """The reference-signature helpers (one C call each: pack, launch, wait), with the tracker as the
    reference's dict and the actions as (move, op) string pairs, against the same fixtures."""
    from marl_gpu import helper as Hm
    d = npz("helpers.npz")
    mv_s, op_s = ["S", "L", "R", "U", "D", "X"], ["0", "1", "2", "9"]
    for i, c in enumerate(meta(d)):
        g = grid(c["map"]).tolist()
        rows = d[f"trk_{i}"].tolist()
        trk = {r[0]: {"id": r[0], "status": "in_transit" if r[1] == 2 else "waiting", "start_pos": (r[2], r[3]),
                      "target_pos": (r[4], r[5]), "start_time": r[6], "deadline": r[7]} for r in rows}
        robots = [tuple(x) for x in d[f"robots_{i}"].tolist()]
        state = {"time_step": c["t"], "map": g, "robots": robots, "packages": []}
        for tk in (trk, rows):
            o = Hm.convert_observation(state, tk, c["idx"])
            assert o.shape == d[f"obs_{i}"].shape
            np.testing.assert_array_equal(o, d[f"obs_{i}"], err_msg=str(c))
            v = Hm.generate_vector_features(state, tk, c["idx"], c["T"], c["MO"], c["MP"])
            np.testing.assert_array_equal(v, d[f"vec_{i}"], err_msg=str(c))
            gm, gv = Hm.convert_global_state(state, tk, c["T"], c["MR"], c["MPs"])
            np.testing.assert_array_equal(gm, d[f"gmap_{i}"], err_msg=str(c))
            np.testing.assert_array_equal(gv, d[f"gvec_{i}"], err_msg=str(c))
        acts = [(mv_s[a], op_s[b]) for a, b in d[f"acts_{i}"].tolist()]
        cur = {"time_step": c["t"] + 1, "map": g, "robots": [tuple(x) for x in d[f"cur_robots_{i}"].tolist()]}
        g0 = 0 if c["g_int"] else c["g"]
        for j, consts in enumerate((Hm.MAPPO_SHAPING, Hm.QMIX_SHAPING)):
            sh = Hm.compute_shaped_rewards(g0, state, cur, acts, trk, len(robots), consts=consts)
            assert isinstance(sh, np.float32) and sh.tobytes() == d[f"sh_{i}"][j].tobytes(), (i, c, j)


@pytest.mark.parametrize("mapname,A,ns", [("map1.txt", 5, 20), ("synthetic64.txt", 16, 60), ("map2.txt", 5, 120),
                                          ("synthetic64.txt", 40, 90)])
def test_helper_record_size_classes(mapname, A, ns):
    """The single-view helpers across the record sizes their paths split on: a view record in
    the small (<= 256 words) or large (<= 768) kernel-argument class, or past it through the
    arena (mdl_host_views_*), each against the oracle's restatement of MAPPO/helper.py."""
    from marl_gpu import helper as Hm
    g = grid(mapname)
    H, W = g.shape
    rs = np.random.RandomState(A * 1000 + ns)
    free = np.argwhere(g == 0)
    t, T = 37, 100
    rows = []
    for k in range(ns):
        s_, d_ = free[rs.randint(len(free))], free[rs.randint(len(free))]
        rows.append([k + 1, 2 if k % 4 == 1 else 1, int(s_[0]), int(s_[1]), int(d_[0]), int(d_[1]),
                     int(rs.randint(0, t + 1)), int(t + rs.randint(-10, 60))])
    transit = [r[0] for r in rows if r[1] == 2]
    cells = free[rs.choice(len(free), 2 * A, replace=False)]
    robots = [(int(cells[i][0]) + 1, int(cells[i][1]) + 1, transit[i] if i < len(transit) and i % 2 else 0)
              for i in range(A)]
    cur = [(int(cells[A + i][0]) + 1, int(cells[A + i][1]) + 1, r[2]) for i, r in enumerate(robots)]
    trk = {r[0]: {"id": r[0], "status": "in_transit" if r[1] == 2 else "waiting", "start_pos": (r[2], r[3]),
                  "target_pos": (r[4], r[5]), "start_time": r[6], "deadline": r[7]} for r in rows}
    glist = g.tolist()
    state = {"time_step": t, "map": glist, "robots": robots, "packages": []}
    for idx in (0, A - 1):
        np.testing.assert_array_equal(Hm.convert_observation(state, trk, idx),
                                      O.convert_observation(g, t, robots, rows, idx))
        np.testing.assert_array_equal(Hm.generate_vector_features(state, trk, idx, T, 30, 100),
                                      O.generate_vector_features(H, W, t, robots, rows, idx, T, 30, 100))
    gm, gv = Hm.convert_global_state(state, trk, T, 50, 120)
    gm0, gv0 = O.convert_global_state(g, t, robots, rows, T, 50, 120)
    np.testing.assert_array_equal(gm, gm0)
    np.testing.assert_array_equal(gv, gv0)
    mv, op = rs.randint(0, 5, A), rs.randint(0, 3, A)
    acts = [("SLRUD"[m], "012"[o]) for m, o in zip(mv, op)]
    curd = {"time_step": t + 1, "map": glist, "robots": cur}
    for consts, oc in ((Hm.MAPPO_SHAPING, O.MAPPO_CONSTS), (Hm.QMIX_SHAPING, O.QMIX_CONSTS)):
        sh = Hm.compute_shaped_rewards(1.5, state, curd, acts, trk, A, consts=consts)
        sh0 = O.compute_shaped_rewards(1.5, t, robots, t + 1, cur, mv, op, rows, A, consts=oc)
        assert sh.tobytes() == sh0.tobytes(), (consts, float(sh), float(sh0))
    with pytest.raises(IndexError):   # fewer actions than agents: the reference indexes past them
        Hm.compute_shaped_rewards(1.5, state, curd, acts[:-1], trk, A)


def test_notebook_kat():
    from marl_gpu import helper as Hm
    k = load_json("kat.json")
    trk = {row[0]: {"id": row[0], "status": "in_transit" if row[1] == 2 else "waiting", "start_pos": (row[2], row[3]),
                    "target_pos": (row[4], row[5]), "start_time": row[6], "deadline": row[7]} for row in k["tracker"]}
    prev = {"robots": [tuple(r) for r in k["prev_robots"]], "time_step": k["prev_t"]}
    cur = {"robots": [tuple(r) for r in k["cur_robots"]], "time_step": k["cur_t"]}
    acts = [tuple(a) for a in k["actions"]]
    m = Hm.compute_shaped_rewards(k["global_reward"], prev, cur, acts, trk, 2)
    q = Hm.compute_shaped_rewards(k["global_reward"], prev, cur, acts, trk, 2, consts=Hm.QMIX_SHAPING)
    assert m.tobytes().hex() == k["mappo_f32_hex"] and float(m) == 215.04000854492188
    assert q.tobytes().hex() == k["qmix_f32_hex"]


# --------------------------------------------------- GPU vs oracle, larger
def _oracle_compare(mapname, E, A, P, T, seed, steps, tracker, check_every=10, rng_seed=0, layout="auto"):
    mg = _mg()
    g = grid(mapname) if isinstance(mapname, str) else mapname
    env = mg.BatchedEnv(g, E, A, P, T, seed=seed, tracker=tracker, shaping="mappo", max_packages_obs=5,
                        step_layout=layout)
    env.reset()
    ob = O.OracleBatch(E, g, A, P, T, seed_base=seed, clear_on_reset=(tracker == "fresh"))
    rs = np.random.RandomState(rng_seed)
    for k in range(steps):
        ints = rs.randint(0, 15, size=(E, A)).astype(np.uint8)
        r, sh, dn = env.step(torch.from_numpy(ints).cuda(), auto_reset=True)
        r0, sh0, d0 = ob.step(ints, auto_reset=True, consts=O.MAPPO_CONSTS)
        np.testing.assert_array_equal(r.cpu().numpy(), r0, err_msg=f"r step {k}")
        np.testing.assert_array_equal(sh.cpu().numpy(), sh0, err_msg=f"shaped step {k}")
        np.testing.assert_array_equal(dn.cpu().numpy().astype(bool), d0, err_msg=f"done step {k}")
        if k % check_every == 0 or k == steps - 1:
            s = snap(env)
            for e in range(E):
                os_ = ob.env(e).state()
                np.testing.assert_array_equal(s["robots"][e], os_["robots"], err_msg=f"robots env {e} step {k}")
                np.testing.assert_array_equal(s["pkgs"][e], os_["pkgs"], err_msg=f"pkgs env {e} step {k}")
                assert s["t"][e] == os_["t"] and s["total_reward"][e] == os_["total_reward"]
                rows = env.tracker_rows(s, e)
                np.testing.assert_array_equal(rows, ob.tracker(e).rows(), err_msg=f"tracker env {e} step {k}")
    env.close()


@pytest.mark.parametrize("layout", ["wave", "rows"])
@pytest.mark.parametrize("tracker", ["mappo", "fresh"])
def test_vs_oracle_map1(tracker, layout):
    _oracle_compare("map1.txt", 64, 5, 50, 60, 1000, 200, tracker, layout=layout)


@pytest.mark.parametrize("mapname,A,P,T", [("map1.txt", 1, 20, 40), ("map1.txt", 3, 50, 40), ("map2.txt", 8, 60, 40),
                                           ("map1.txt", 7, 30, 40), ("map3.txt", 5, 64, 30),
                                           ("synthetic64.txt", 5, 64, 40)])
def test_vs_oracle_rows_layout(mapname, A, P, T):
    """k_step_rows (four envs per wavefront) against the oracle: A < 5, A = 5, A = 8 (numpy's
    8-partial sum), P up to 64, the 64x64 map; 37 envs leave the last wave's rows partly empty."""
    _oracle_compare(mapname, 37, A, P, T, 700 + A, 90, "mappo", layout="rows")


@pytest.mark.parametrize("mapname,A,P,T", [("map1.txt", 1, 20, 40), ("map1.txt", 3, 50, 40), ("map2.txt", 8, 60, 40),
                                           ("map1.txt", 7, 30, 40), ("map2.txt", 5, 100, 40),
                                           ("map2.txt", 5, 200, 40), ("map3.txt", 9, 70, 40)])
def test_vs_oracle_robot_counts(mapname, A, P, T):
    """Every step-kernel specialisation: A == 5 exactly (P <= 128), A <= 8 with the
    robot count at run time (incl. numpy's 8-partial sum at A == 8), the general form."""
    _oracle_compare(mapname, 32, A, P, T, 300 + A, 90, "mappo")


@pytest.mark.parametrize("mapname,A,P,T", [("map2.txt", 8, 130, 50), ("map4.txt", 5, 300, 50),
                                           ("synthetic64.txt", 64, 1024, 40), ("map2.txt", 3, 1024, 30)])
def test_vs_oracle_package_chunks(mapname, A, P, T):
    """Package tables of 2..16 register chunks (NCH = 4, 8, 16) up to MDL_MAX_PACKAGES,
    with MDL_MAX_ROBOTS robots on the 64x64 map."""
    _oracle_compare(mapname, 6, A, P, T, 500 + P, 45, "mappo", check_every=15)


def test_vs_oracle_dense_synthetic():
    _oracle_compare("synthetic64.txt", 16, 16, 100, 50, 77, 120, "mappo", check_every=20)


@pytest.mark.parametrize("H,W", [(3, 255), (255, 3), (2, 1)])
def test_vs_oracle_extreme_map_shapes(H, W):
    """Maps at the 255-row / 255-column limit (the last row / column of the packed-cell
    move-validity table) and a 2x1 strip, 10 % random obstacles."""
    rs = np.random.RandomState(H * 1000 + W)
    g = (rs.rand(H, W) < 0.1).astype(np.uint8) if H * W > 2 else np.zeros((H, W), np.uint8)
    A = 5 if H * W > 2 else 1
    _oracle_compare(g, 8, A, 40, 60, 900 + H, 80, "mappo", check_every=20)


def test_vs_oracle_crowded():
    _oracle_compare("map1.txt", 16, 40, 30, 40, 5, 100, "mappo")
    _oracle_compare("map3.txt", 8, 64, 200, 30, 9, 70, "fresh")


# -------------------------------------------------------- compat dict API
def test_compat_environment_steps_golden():
    from marl_gpu.compat import Environment
    d = npz("steps.npz")
    inv_m = {0: "S", 1: "L", 2: "R", 3: "U", 4: "D", 5: "X"}
    inv_o = {0: "0", 1: "1", 2: "2", 3: "3"}
    for ci, c in enumerate(meta(d)[:3]):
        env = Environment(f"{c['map']}", c["T"], c["A"], c["P"], seed=c["seed"])
        env.reset()
        acts = d[f"acts_{ci}"]
        for k in range(c["n"]):
            a = [(inv_m[int(x[0])], inv_o[int(x[1])]) for x in acts[k]]
            st, r, done, info = env.step(a)
            assert r == d[f"r_{ci}"][k] and isinstance(r, int) == bool(d[f"rint_{ci}"][k])
            assert done == d[f"done_{ci}"][k]
            if done:
                assert info["total_reward"] == env.total_reward and info["total_time_steps"] == env.t
                if c["auto_reset"]:
                    st = env.reset()
            assert [rb[:2] for rb in st["robots"]] == [(int(p[0]) + 1, int(p[1]) + 1) for p in d[f"pos_{ci}"][k]]


def test_readme_random_agent_anchor():
    """README.md:117-121 random-agent row, via the compat Environment."""
    from marl_gpu.compat import Environment
    ref = load_json("eval_anchor.json")
    cfg = ref["config"]
    np.random.seed(10)
    rewards, delivered = [], []
    for ep in range(cfg["episodes"]):
        env = Environment("map1.txt", cfg["max_time_steps"], cfg["n_agents"], cfg["n_packages"], seed=cfg["seed"] + ep)
        state = env.reset()
        n = len(state["robots"])
        done = False
        infos = {}
        while not done:
            actions = []
            for _ in range(n):       # randomagent.py:16-21 draw order
                mv = np.random.choice(["U", "D", "L", "R", "S"])
                op = np.random.choice(["0", "1", "2"])
                actions.append((mv, op))
            state, reward, done, infos = env.step(actions)
        rewards.append(infos.get("total_reward", env.total_reward))
        delivered.append(sum(1 for p in env.packages if p.status == "delivered"))
        env.engine.close()
    assert rewards == ref["random"]["rewards"]
    assert delivered == ref["random"]["delivered"]
    assert round(float(np.mean(rewards)), 2) == -16.50 and round(float(np.std(rewards)), 2) == 6.24
    assert round(float(np.mean(delivered)), 2) == 13.66


@pytest.mark.parametrize("mapname,P,tracker", [("map1.txt", 100, "mappo"), ("map1.txt", 40, "fresh"),
                                               ("map2.txt", 128, "mappo"), ("map3.txt", 64, "fresh"),
                                               ("synthetic64.txt", 17, "mappo")])
def test_vs_oracle_sixteen_robots(mapname, P, tracker):
    """The 16-robot kernel (config 5's robot count: P <= 128, one or two package chunks),
    whose shaped reward finds every agent's nearest waiting package from LDS-packed
    candidates: on map1 sixteen robots share 64 free cells, so equal distances -- and the
    reference's first-in-tracker-order tie-break -- are the common case."""
    _oracle_compare(mapname, 24, 16, P, 45, 4200 + P, 100, tracker, check_every=25)
