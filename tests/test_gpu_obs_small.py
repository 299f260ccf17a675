"""k_obs_small (csrc/mdl_obs_small.hpp) vs the generic k_obs builder and the
oracle: the engine's fast observation path for A <= 8, P <= 64, <= 8 package
slots must produce the same bits as the generic path for every output
(MAPPO/helper.py:6-255) on identical states, across maps (HW % 4 == 0 and
not), both tracker modes, padded and unpadded vector layouts, MR < A, and
obs_max_time_steps <= 0."""
import os

import numpy as np
import pytest
import torch

import oracle as O
from golden_io import grid

pytestmark = pytest.mark.gpu


def _mg():
    import marl_gpu
    return marl_gpu


def _pair(mg, g, E, A, P, T, **kw):
    """Two engines with identical streams: the small builder and the generic one (MdlConfig.obs_builder)."""
    a = mg.BatchedEnv(g, E, A, P, T, **kw)
    b = mg.BatchedEnv(g, E, A, P, T, obs_builder="generic", **kw)
    return a, b


CASES = [
    # map, A, P, T, tracker, MO, MP, MR, MPs, obsT
    ("map1.txt", 5, 50, 60, "mappo", 4, 5, 100, 100, None),      # config 3 sizes (MAPPO trainer)
    ("map1.txt", 5, 50, 60, "fresh", 4, 5, 10, 20, None),        # QMIX config sizes
    ("map.txt", 4, 20, 30, "mappo", 6, 8, 3, 10, None),          # 7x7 (HW % 4 != 0), padded others, MR < A
    ("map2.txt", 3, 64, 40, "fresh", 2, 8, 100, 30, 0),          # P = 64, obsT = 0
    ("map3.txt", 7, 30, 25, "mappo", 6, 1, 8, 30, 17),           # A = 7 (63 tuple lanes), one package slot, obsT < T
    ("map1.txt", 1, 10, 20, "mappo", 0, 3, 1, 5, None),          # one robot
    ("map1.txt", 5, 50, 60, "mappo", 100, 100, 100, 100, None),  # config 3b (helper defaults): bitonic order
    ("map4.txt", 8, 64, 30, "fresh", 7, 64, 8, 64, None),        # A = 8, P = MP = 64: full sort, many tuple passes
    ("map5.txt", 6, 40, 45, "mappo", 3, 9, 4, 25, 50),           # MO < A-1, 9 slots, obsT > T
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-A{c[1]}-P{c[2]}-{c[4]}" for c in CASES])
def test_small_builder_matches_generic(case):
    mg = _mg()
    m, A, P, T, tracker, MO, MP, MR, MPs, obsT = case
    g = grid(m)
    E = 96
    kw = dict(seed=11, tracker=tracker, max_other_robots=MO, max_packages_obs=MP, max_robots_state=MR,
              max_packages_state=MPs, obs_max_time_steps=obsT)
    a, b = _pair(mg, g, E, A, P, T, **kw)
    a.reset()
    b.reset()
    gen = np.random.RandomState(5)
    for k in range(2 * T + 7):
        acts = torch.from_numpy(gen.randint(0, 15, size=(E, A)).astype(np.uint8)).cuda()
        a.step(acts)
        b.step(acts)
        if k % 9 == 4:
            oa, ob = a.build_obs(), b.build_obs()
            for key in ("actor_map", "actor_vec", "critic_map", "critic_vec"):
                x, y = oa[key].cpu().numpy(), ob[key].cpu().numpy()
                assert x.shape == y.shape
                # bitwise (also the sign of zeros)
                assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), (key, k)
    a.close()
    b.close()


def test_small_builder_config3_vs_oracle():
    """Config 3 featurizer sizes along a MAPPO rollout (stale tracker, auto-reset), checked
    against the oracle's literal restatement of the three helpers."""
    mg = _mg()
    g = grid("map1.txt")
    E, A, P, T = 16, 5, 50, 40
    env = mg.BatchedEnv(g, E, A, P, T, seed=42, tracker="mappo", max_other_robots=4, max_packages_obs=5)
    env.reset()
    ob = O.OracleBatch(E, g, A, P, T, seed_base=42, clear_on_reset=False)
    gen = np.random.RandomState(3)
    for k in range(90):
        ints = gen.randint(0, 15, size=(E, A)).astype(np.uint8)
        env.step(torch.from_numpy(ints).cuda())
        ob.step(ints, auto_reset=True, consts=O.MAPPO_CONSTS)
        if k % 15 == 7:
            o = env.build_obs()
            av, cv = o["actor_vec"].cpu().numpy(), o["critic_vec"].cpu().numpy()
            am, cm = o["actor_map"].cpu().numpy(), o["critic_map"].cpu().numpy()
            for e in range(E):
                oe, ot = ob.env(e), ob.tracker(e)
                st, rb1, rows = oe.state(), oe.robots1(), ot.rows()
                for a in range(A):
                    np.testing.assert_array_equal(
                        av[e, a], O.generate_vector_features(10, 10, st["t"], rb1, rows, a, T, 4, 5))
                    np.testing.assert_array_equal(am[e, a], O.convert_observation(g, st["t"], rb1, rows, a))
                gm, gv = O.convert_global_state(g, st["t"], rb1, rows, T, 100, 100)
                np.testing.assert_array_equal(cv[e], gv)
                np.testing.assert_array_equal(cm[e], gm)
    env.close()


@pytest.mark.parametrize("case", [("map.txt", 4, 20, 30, 6, 8, 3, 10), ("map1.txt", 5, 50, 60, 100, 100, 100, 100),
                                  ("map4.txt", 3, 30, 40, 2, 5, 4, 7)],
                         ids=["7x7", "config3b", "19x20"])
def test_flat_emission_any_alignment_and_range(case):
    """The builder writes every float of each tensor exactly once, wherever the tensor starts
    inside a 16-B line (1..3 floats in: the unaligned emission paths), with float4s that straddle
    envs / planes / agents (HW % 4 != 0, vector lengths % 4 != 0), and for an env sub-range:
    bit-identical to the aligned full build, the sentinels around each tensor intact."""
    mg = _mg()
    m, A, P, T, MO, MP, MR, MPs = case
    g = grid(m)
    H, W = g.shape
    E = 37
    env = mg.BatchedEnv(g, E, A, P, T, seed=3, tracker="mappo", max_other_robots=MO, max_packages_obs=MP,
                        max_robots_state=MR, max_packages_state=MPs)
    env.reset()
    gen = np.random.RandomState(8)
    for _ in range(T // 2 + 3):
        env.step(torch.from_numpy(gen.randint(0, 15, size=(E, A)).astype(np.uint8)).cuda())
    ref = {k: v.clone() for k, v in env.build_obs().items()}
    shapes = {k: tuple(v.shape) for k, v in ref.items()}
    for lead in (1, 2, 3):
        for b, n in ((0, E), (5, 20), (36, 1)):
            out, raw = {}, {}
            for k, shp in shapes.items():
                cnt = int(np.prod((n,) + shp[1:]))
                buf = torch.full((lead + cnt + 5,), -7.0, dtype=torch.float32, device="cuda")
                raw[k] = buf
                out[k] = buf[lead:lead + cnt].view((n,) + shp[1:])
            env.build_obs(env_begin=b, n=n, out=out)
            torch.cuda.synchronize()
            for k in shapes:
                got = out[k].cpu().numpy()
                want = ref[k][b:b + n].cpu().numpy()
                assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (k, lead, b, n)
                r = raw[k].cpu().numpy()
                assert (r[:lead] == -7.0).all() and (r[lead + got.size:] == -7.0).all(), (k, lead, b, n)
    # one tensor alone (the others not requested)
    o = env.build_obs(which=("critic_vec",))
    assert torch.equal(o["critic_vec"], ref["critic_vec"])
    env.close()
