"""Randomised parity: the HIP engine against the oracle on seeded random maps and configurations
beyond the reference's own maps -- odd shapes (1-wide corridors, non-square, HW % 32 and % 4 != 0),
obstacle densities up to 45 %, robot counts across every step-kernel specialisation (A = 1..16 and
the general form), package tables of one to two register chunks, short and long episodes, both
tracker modes.  Every step: env reward, shaped reward, done bit for bit; every few steps the full
state and tracker rows; at the end the observation tensors of every env (MAPPO/helper.py:6-255).
Half the cases are driven by the engine's batched greedy agent (greedyagent.py) instead of random
actions, so pick-ups and on-time / late deliveries happen often; the same trainer ints go to the
oracle.  The oracle (oracle/mdl_oracle.c) is pinned to the reference by tests/test_oracle_golden.py."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from golden_io import TRAINER_MOVE_CODES  # noqa: E402

# packed code (move | op << 3) -> the trainer int that decodes to it (golden_io.decode_trainer:
# move = TRAINER_MOVE_CODES[i % 5], op = i // 5)
_CODE_TO_INT = np.zeros(64, np.uint8)
for _i in range(15):
    _CODE_TO_INT[int(TRAINER_MOVE_CODES[_i % 5]) | ((_i // 5) << 3)] = _i


def _snap(env):
    s = env.read_state()
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in s.items()}


def _random_grid(rs, H, W, density):
    """Border walls (when the map is at least 3 cells thick) and random interior obstacles."""
    g = (rs.random_sample((H, W)) < density).astype(np.uint8)
    if H >= 3 and W >= 3:
        g[0, :] = 1
        g[-1, :] = 1
        g[:, 0] = 1
        g[:, -1] = 1
    return g


# (H, W, obstacle density, A, P, T, tracker) -- drawn once, kept literal so failures reproduce
CASES = [
    (1, 12, 0.0, 2, 5, 20, "mappo"),        # one row: every move is L / R or blocked
    (9, 1, 0.0, 3, 4, 25, "fresh"),         # one column
    (7, 13, 0.15, 5, 40, 30, "mappo"),      # A = 5 kernel, HW = 91 (HW % 4 != 0)
    (11, 11, 0.30, 4, 17, 45, "fresh"),     # A <= 8 kernel
    (6, 6, 0.10, 8, 64, 18, "mappo"),       # A = 8 in a crowded 4x4 interior, P = 64 (one chunk)
    (19, 23, 0.45, 6, 65, 35, "mappo"),     # dense obstacles, P = 65 (two chunks)
    (32, 32, 0.20, 16, 100, 40, "mappo"),   # the 16-robot kernel (config 5's), HW = 1024
    (33, 47, 0.05, 16, 128, 30, "fresh"),   # 16 robots, P = 128, odd shape
    (64, 64, 0.25, 12, 90, 25, "mappo"),    # the general kernel (A > 8, A != 16) on the largest map
    (5, 40, 0.10, 1, 1, 12, "fresh"),       # one robot, one package
    (15, 9, 0.20, 7, 30, 60, "mappo"),      # A = 7, several episodes
    (24, 24, 0.35, 10, 120, 22, "fresh"),   # general kernel, fresh tracker, two chunks
]


@pytest.mark.parametrize("greedy", [False, True], ids=["random", "greedy"])
@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}x{c[1]}-A{c[3]}-P{c[4]}-{c[6]}" for c in CASES])
def test_random_map_vs_oracle(case, greedy):
    import marl_gpu as mg
    H, W, dens, A, P, T, tracker = case
    rs = np.random.RandomState(H * 1000 + W * 10 + A)
    g = _random_grid(rs, H, W, dens)
    assert int((g == 0).sum()) >= A + 1, "fixture map has room for the robots"
    E, seed = 24, int(rs.randint(0, 10_000))
    MO, MP, MR, MPs = max(A - 1, 1), 6, A + 2, P // 2 + 1
    env = mg.BatchedEnv(g, E, A, P, T, seed=seed, tracker=tracker, shaping="mappo", max_other_robots=MO,
                        max_packages_obs=MP, max_robots_state=MR, max_packages_state=MPs)
    env.reset()
    if greedy:
        env.greedy_init()
    ob = O.OracleBatch(E, g, A, P, T, seed_base=seed, clear_on_reset=(tracker == "fresh"))
    steps = 2 * T + 7   # through at least two auto-resets
    delivered = 0
    for k in range(steps):
        if greedy:
            ints = _CODE_TO_INT[env.greedy_actions().cpu().numpy()]
        else:
            ints = rs.randint(0, 15, size=(E, A)).astype(np.uint8)
        r, sh, dn = env.step(torch.from_numpy(ints).cuda(), auto_reset=True)
        r0, sh0, d0 = ob.step(ints, auto_reset=True, consts=O.MAPPO_CONSTS)
        np.testing.assert_array_equal(r.cpu().numpy(), r0, err_msg=f"r step {k}")
        np.testing.assert_array_equal(sh.cpu().numpy(), sh0, err_msg=f"shaped step {k}")
        np.testing.assert_array_equal(dn.cpu().numpy().astype(bool), d0, err_msg=f"done step {k}")
        delivered += int((r0 >= 0.5).sum())   # a delivery adds >= delay_reward (1.0) to the step's reward
        if greedy and d0.any():   # the reference re-initialises its agents every episode
            env.greedy_init(env_ids=torch.from_numpy(np.nonzero(d0)[0].astype(np.int32)).cuda())
        if k % 11 == 0 or k == steps - 1:
            s = _snap(env)
            for e in range(E):
                os_ = ob.env(e).state()
                np.testing.assert_array_equal(s["robots"][e], os_["robots"], err_msg=f"robots env {e} step {k}")
                np.testing.assert_array_equal(s["pkgs"][e], os_["pkgs"], err_msg=f"pkgs env {e} step {k}")
                assert s["t"][e] == os_["t"] and s["total_reward"][e] == os_["total_reward"]
                np.testing.assert_array_equal(env.tracker_rows(s, e), ob.tracker(e).rows(),
                                              err_msg=f"tracker env {e} step {k}")
    if greedy and P >= 4 and (g == 0).sum() >= 8:
        assert delivered > 0, "the greedy agents delivered packages"
    o = env.build_obs()
    am, av = o["actor_map"].cpu().numpy(), o["actor_vec"].cpu().numpy()
    cm, cv = o["critic_map"].cpu().numpy(), o["critic_vec"].cpu().numpy()
    for e in range(E):
        oe, ot = ob.env(e), ob.tracker(e)
        st, rb1, rows = oe.state(), oe.robots1(), ot.rows()
        for a in range(A):
            np.testing.assert_array_equal(am[e, a], O.convert_observation(g, st["t"], rb1, rows, a),
                                          err_msg=f"actor map env {e} agent {a}")
            np.testing.assert_array_equal(av[e, a], O.generate_vector_features(H, W, st["t"], rb1, rows, a, T, MO, MP),
                                          err_msg=f"actor vec env {e} agent {a}")
        gm, gv = O.convert_global_state(g, st["t"], rb1, rows, T, MR, MPs)
        np.testing.assert_array_equal(cm[e], gm, err_msg=f"critic map env {e}")
        np.testing.assert_array_equal(cv[e], gv, err_msg=f"critic vec env {e}")
    env.close()
