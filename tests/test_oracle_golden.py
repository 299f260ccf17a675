"""Pin the CPU oracle to the reference: every fixture produced by running the
reference (tests/golden/gen_golden.py) must be reproduced bit for bit."""
import numpy as np
import pytest

import oracle as O
from golden_io import decode_trainer, grid, load_json, meta, npz


@pytest.fixture(scope="module", autouse=True)
def _build():
    O.build()


def test_numpy_pairwise_sum_model():
    rng = np.random.default_rng(1)
    for _ in range(3000):
        n = int(rng.integers(0, 300))
        a = (rng.standard_normal(n) * 10 ** rng.uniform(-3, 3, n)).astype(np.float32)
        assert O.np_sum_f32(a).tobytes() == a.sum(dtype=np.float32).tobytes()


def test_reset_layouts():
    d = npz("reset.npz")
    cases = meta(d)
    for i, c in enumerate(cases):
        env = O.OracleEnv(grid(c["map"]), c["A"], c["P"], c["T"], seed=c["seed"])
        for k in range(3):
            if k:
                env.reset()
            s = env.state()
            assert s["t"] == 0
            np.testing.assert_array_equal(s["robots"][:, :2], d[f"robots_{i}"][k], err_msg=str(c))
            np.testing.assert_array_equal(s["pkgs"][:, :6], d[f"pkgs_{i}"][k], err_msg=str(c))
            np.testing.assert_array_equal(s["pkgs"][:, 6], np.arange(1, c["P"] + 1))


def test_step_traces():
    d = npz("steps.npz")
    for ci, c in enumerate(meta(d)):
        env = O.OracleEnv(grid(c["map"]), c["A"], c["P"], c["T"], seed=c["seed"])
        env.reset()
        s = env.state()
        np.testing.assert_array_equal(s["robots"][:, :2], d[f"pos0_{ci}"])
        np.testing.assert_array_equal(s["pkgs"][:, :6], d[f"pkgs0_{ci}"])
        acts = d[f"acts_{ci}"]
        for k in range(c["n"]):
            r, rint, done = env.step(acts[k, :, 0], acts[k, :, 1])
            assert r == d[f"r_{ci}"][k] and rint == d[f"rint_{ci}"][k], (c, k)
            assert done == d[f"done_{ci}"][k], (c, k)
            s = env.state()
            assert s["t"] == d[f"t_{ci}"][k] and s["total_reward"] == d[f"total_{ci}"][k], (c, k)
            if done and c["auto_reset"]:
                env.reset()
                s = env.state()
            np.testing.assert_array_equal(s["robots"][:, :2], d[f"pos_{ci}"][k], err_msg=f"{c} step {k}")
            np.testing.assert_array_equal(s["robots"][:, 2], d[f"carry_{ci}"][k], err_msg=f"{c} step {k}")
            np.testing.assert_array_equal(s["pkgs"][:, 7], d[f"status_{ci}"][k], err_msg=f"{c} step {k}")
            np.testing.assert_array_equal(s["pkgs"][:, :6], d[f"pkgs_{ci}"][k], err_msg=f"{c} step {k}")


def _features(env, trk, T, MO, MP, MR, MPs, want_map=True):
    s = env.state()
    rb1 = env.robots1()
    rows = trk.rows()
    A = rb1.shape[0]
    H, W = env.H, env.W
    avec = np.stack([O.generate_vector_features(H, W, s["t"], rb1, rows, a, T, MO, MP) for a in range(A)])
    out = dict(avec=avec)
    if want_map:
        out["amap"] = np.stack([O.convert_observation(env.grid, s["t"], rb1, rows, a) for a in range(A)])
    gm, gv = O.convert_global_state(env.grid, s["t"], rb1, rows, T, MR, MPs)
    out["cmap"], out["cvec"] = gm, gv
    out["rows"], out["rb1"], out["t"] = rows, rb1, s["t"]
    return out


@pytest.mark.parametrize("tag", ["mappo", "mappo_map2", "mappo_syn64"])
def test_mappo_rollout(tag):
    d = npz(f"rollout_{tag}.npz")
    m = meta(d)
    E, A, P, T = m["E"], m["A"], m["P"], m["T"]
    g = grid(m["map"])
    batch = O.OracleBatch(E, g, A, P, T, seed_base=m["seed"], clear_on_reset=False)
    envs = [batch.env(e) for e in range(E)]
    trks = [batch.tracker(e) for e in range(E)]
    map_steps = list(d["map_steps"])
    big_steps = list(d["big_steps"])

    def check(k):
        for e in range(E):
            f = _features(envs[e], trks[e], T, m["MO"], m["MP"], m["MR"], m["MPs"], want_map=k in map_steps)
            np.testing.assert_array_equal(f["avec"], d["avec"][k, e], err_msg=f"avec step {k} env {e}")
            np.testing.assert_array_equal(f["cvec"], d["cvec"][k, e], err_msg=f"cvec step {k} env {e}")
            _, gq = O.convert_global_state(g, f["t"], f["rb1"], f["rows"], T, 10, 20)
            np.testing.assert_array_equal(gq, d["cvec_qmix"][k, e])
            if k in map_steps:
                j = map_steps.index(k)
                np.testing.assert_array_equal(f["amap"], d["amap"][j, e])
                np.testing.assert_array_equal(f["cmap"], d["cmap"][j, e])
            if k in big_steps:
                j = big_steps.index(k)
                big = np.stack([O.generate_vector_features(g.shape[0], g.shape[1], f["t"], f["rb1"], f["rows"], a, T,
                                                           100, 100) for a in range(A)])
                np.testing.assert_array_equal(big, d["avec_big"][j, e])

    check(0)
    for k in range(d["acts"].shape[0]):
        acts = d["acts"][k]
        r, sh, done = batch.step(acts, auto_reset=True, consts=O.MAPPO_CONSTS)
        np.testing.assert_array_equal(r, d["r_env"][k])
        np.testing.assert_array_equal(sh, d["r_shaped"][k], err_msg=f"step {k}")
        np.testing.assert_array_equal(done, d["done"][k])
        check(k + 1)


def test_qmix_rollout():
    """QMIX/trainer.py:333-526: subset stepping, tracker cleared after each iteration."""
    d = npz("rollout_qmix.npz")
    m = meta(d)
    E, A, P, T = m["E"], m["A"], m["P"], m["T"]
    g = grid(m["map"])
    envs = [O.OracleEnv(g, A, P, T, seed=m["seed"] + e) for e in range(E)]
    trks = [O.OracleTracker(P) for _ in range(E)]
    for e in range(E):
        envs[e].reset()
        trks[e].update_from_env(envs[e])
    for k in range(d["active"].shape[0]):
        active = d["active"][k]
        if not active.any():
            # iteration boundary: vec_env.reset() + trackers cleared
            for e in range(E):
                envs[e].reset()
                trks[e].clear()
                trks[e].update_from_env(envs[e])
        else:
            mv, op = decode_trainer(d["acts"][k])
            for e in np.nonzero(active)[0]:
                prev_t, prev1, rows = envs[e].state()["t"], envs[e].robots1(), trks[e].rows()
                r, _, done = envs[e].step(mv[e], op[e])
                sh = O.compute_shaped_rewards(r, prev_t, prev1, envs[e].state()["t"], envs[e].robots1(), mv[e], op[e],
                                              rows, A, O.QMIX_CONSTS)
                trks[e].update_from_env(envs[e])
                assert r == d["r"][k, e] and done == d["done"][k, e]
                assert sh.tobytes() == d["sh"][k, e].tobytes()
        for e in range(E):
            f = _features(envs[e], trks[e], T, m["MO"], m["MP"], m["MR"], m["MPs"])
            np.testing.assert_array_equal(f["avec"], d["avec"][k, e])
            np.testing.assert_array_equal(f["cvec"], d["cvec"][k, e])
            np.testing.assert_array_equal(f["amap"], d["amap"][k, e])


def test_helper_dict_cases():
    d = npz("helpers.npz")
    for i, c in enumerate(meta(d)):
        g = grid(c["map"])
        H, W = g.shape
        rb = d[f"robots_{i}"]
        rows = d[f"trk_{i}"]
        obs = O.convert_observation(g, c["t"], rb, rows, c["idx"])
        np.testing.assert_array_equal(obs, d[f"obs_{i}"], err_msg=str(c))
        vec = O.generate_vector_features(H, W, c["t"], rb, rows, c["idx"], c["T"], c["MO"], c["MP"])
        np.testing.assert_array_equal(vec, d[f"vec_{i}"], err_msg=str(c))
        gm, gv = O.convert_global_state(g, c["t"], rb, rows, c["T"], c["MR"], c["MPs"])
        np.testing.assert_array_equal(gm, d[f"gmap_{i}"])
        np.testing.assert_array_equal(gv, d[f"gvec_{i}"], err_msg=str(c))
        acts = d[f"acts_{i}"]
        g0 = 0 if c["g_int"] else c["g"]
        for j, consts in enumerate((O.MAPPO_CONSTS, O.QMIX_CONSTS)):
            sh = O.compute_shaped_rewards(g0, c["t"], rb, c["t"] + 1, d[f"cur_robots_{i}"], acts[:, 0], acts[:, 1],
                                          rows, c["A"], consts)
            assert sh.tobytes() == d[f"sh_{i}"][j].tobytes(), (i, c, j)


def test_notebook_kat():
    k = load_json("kat.json")
    mv = np.array([O.MOVE_CODES[a[0]] for a in k["actions"]], np.uint8)
    op = np.array([int(a[1]) for a in k["actions"]], np.uint8)
    for consts, key in ((O.MAPPO_CONSTS, "mappo_f32_hex"), (O.QMIX_CONSTS, "qmix_f32_hex")):
        sh = O.compute_shaped_rewards(k["global_reward"], k["prev_t"], k["prev_robots"], k["cur_t"], k["cur_robots"],
                                      mv, op, k["tracker"], 2, consts)
        assert sh.tobytes().hex() == k[key]
    assert float(np.frombuffer(bytes.fromhex(k["mappo_f32_hex"]), np.float32)[0]) == k["notebook_recorded"]


def test_greedy_agent_readme_anchor():
    """greedyagent.py restated in C reproduces the reference's per-episode greedy results
    (evaluation.py:9-66 at the README.md:117-121 settings: 34.04 +- 14.83, 3.79 delivered)."""
    ref = load_json("eval_anchor.json")
    cfg = ref["config"]
    g = grid(cfg["map"])
    rewards, delivered = [], []
    for ep in range(cfg["episodes"]):
        env = O.OracleEnv(g, cfg["n_agents"], cfg["n_packages"], cfg["max_time_steps"], seed=cfg["seed"] + ep)
        env.reset()
        agent = O.OracleGreedy(env)
        done = False
        while not done:
            mv, op = agent.actions(env)
            _, _, done = env.step(mv, op)
        s = env.state()
        rewards.append(s["total_reward"])
        delivered.append(int((s["pkgs"][:, 7] == 3).sum()))
    assert rewards == ref["greedy"]["rewards"]
    assert delivered == ref["greedy"]["delivered"]
    assert round(float(np.mean(rewards)), 2) == 34.04 and round(float(np.std(rewards)), 2) == 14.83


def test_alt_featurizers_golden():
    """IDQ/qmix convert_state, qmix convert_global_state_to_tensor (incl. cropped/padded
    shapes) and IDQ reward_shaping (int and string ops) vs the reference's outputs."""
    d = npz("alt_features.npz")
    for i, c in enumerate(meta(d)):
        g = grid(c["map"])
        rob, trk, t, A = d[f"robots_{i}"], d[f"trk_{i}"], c["t"], c["A"]
        for a in range(A):
            np.testing.assert_array_equal(O.idq_convert_state(g, t, rob, trk, a), d[f"idq_obs_{i}"][a], f"idq {i}/{a}")
        for k, sh in enumerate(c["shapes"]):
            np.testing.assert_array_equal(O.qmix_global_tensor(g, t, rob, trk, sh), d[f"qmix_state_{i}_{k}"],
                                          f"qmix state {i}/{k}")
        cur = d[f"cur_robots_{i}"]
        np.testing.assert_array_equal(O.idq_reward_shaping(t, rob, t + 1, cur, d[f"ops_{i}"], True, trk, A),
                                      d[f"rw_int_{i}"], f"rw int {i}")
        np.testing.assert_array_equal(O.idq_reward_shaping(t, rob, t + 1, cur, d[f"ops_{i}"], False, trk, A),
                                      d[f"rw_str_{i}"], f"rw str {i}")
