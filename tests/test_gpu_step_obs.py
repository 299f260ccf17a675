"""mdl_step_obs (BatchedEnv.step_obs): the step followed by the observation build of
the new state -- one kernel for A <= 8, P <= 64, two launches otherwise -- is
bit-identical to mdl_step + mdl_build_obs (themselves pinned to the reference by the
golden fixtures and the oracle), across auto-resets, in both tracker modes, and the
trainer sequence MAPPO/trainer.py:229-286 it replaces."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from golden_io import grid  # noqa: E402

KEYS = ("actor_map", "actor_vec", "critic_map", "critic_vec")


def _mg():
    import marl_gpu
    return marl_gpu


def _pair(mapname, E, A, P, T, **kw):
    mg = _mg()
    g = grid(mapname)
    a = mg.BatchedEnv(g, E, A, P, T, seed=17, **kw)
    b = mg.BatchedEnv(g, E, A, P, T, seed=17, **kw)
    a.reset()
    b.reset()
    return a, b


@pytest.mark.parametrize("mapname,A,P,T,tracker,kw", [
    ("map1.txt", 5, 50, 30, "mappo", dict(max_packages_obs=5)),                       # config 3's builder
    ("map1.txt", 5, 50, 30, "fresh", dict(max_packages_obs=5)),
    ("map1.txt", 5, 50, 25, "mappo", dict(max_other_robots=100, max_packages_obs=100)),   # 1007-dim actor vec
    ("map2.txt", 8, 64, 40, "mappo", dict(max_packages_obs=7, max_robots_state=10, max_packages_state=20)),
    ("map.txt", 3, 20, 20, "fresh", dict(max_packages_obs=5, shaping="qmix")),
    ("map1.txt", 16, 40, 30, "mappo", dict(max_packages_obs=5)),                      # A > 8: two launches
    ("map2.txt", 5, 100, 30, "mappo", dict(max_packages_obs=5)),                      # P > 64: two launches
])
def test_step_obs_equals_step_then_build_obs(mapname, A, P, T, tracker, kw):
    E = 96
    a, b = _pair(mapname, E, A, P, T, tracker=tracker, **kw)
    gen = torch.Generator(device="cuda").manual_seed(3)
    for k in range(2 * T + 7):                      # crosses two synchronized auto-resets
        acts = torch.randint(0, 15, (E, A), dtype=torch.uint8, device="cuda", generator=gen)
        ra, sa, da, oa = a.step_obs(acts)
        rb, sb, db = b.step(acts)
        ob = b.build_obs()
        assert torch.equal(ra, rb) and torch.equal(sa, sb) and torch.equal(da, db), k
        for key in KEYS:
            assert torch.equal(oa[key], ob[key]), (k, key)


def test_step_obs_subset_outputs_and_oracle():
    """Outputs may be skipped (NULL); the built vectors match the oracle's
    generate_vector_features / convert_global_state on the new state."""
    mg = _mg()
    g = grid("map1.txt")
    E, A, P, T = 32, 5, 50, 40
    env = mg.BatchedEnv(g, E, A, P, T, seed=42, tracker="mappo", max_packages_obs=5)
    env.reset()
    O.build()
    ob = O.OracleBatch(E, g, A, P, T, seed_base=42, clear_on_reset=False)
    rs = np.random.RandomState(5)
    for k in range(60):
        ints = rs.randint(0, 15, size=(E, A)).astype(np.uint8)
        r, sh, d, obs = env.step_obs(torch.from_numpy(ints).cuda(), which=("actor_vec", "critic_vec"))
        assert obs["actor_map"] is None and obs["critic_map"] is None   # not written: not returned
        r0, s0, d0 = ob.step(ints, auto_reset=True, consts=O.MAPPO_CONSTS)
        assert np.array_equal(r.cpu().numpy(), r0) and np.array_equal(sh.cpu().numpy(), s0), k
        assert np.array_equal(d.cpu().numpy().astype(bool), d0), k
        if k % 7 == 0:
            vec = obs["actor_vec"].cpu().numpy()
            gv = obs["critic_vec"].cpu().numpy()
            for e in range(0, E, 5):
                oe, ot = ob.env(e), ob.tracker(e)
                st = oe.state()
                for i in range(A):
                    want = O.generate_vector_features(10, 10, st["t"], oe.robots1(), ot.rows(), i, T, A - 1, 5)
                    assert np.array_equal(vec[e, i], want), (k, e, i)
                _, gwant = O.convert_global_state(g, st["t"], oe.robots1(), ot.rows(), T, 100, 100)
                assert np.array_equal(gv[e], gwant), (k, e)


def test_step_obs_refuses_mixed_shapes():
    mg = _mg()
    env = mg.BatchedEnv([grid("map1.txt"), grid("map2.txt")], 8, 5, 20, 30, seed=1, env_map=[0] * 4 + [1] * 4)
    env.reset()
    with pytest.raises(ValueError, match="mix map shapes"):
        env.step_obs(torch.zeros((8, 5), dtype=torch.uint8, device="cuda"))
