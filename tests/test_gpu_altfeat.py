"""IDQ / qmix featurizers and IDQ reward shaping on the device:
the dict-API drop-ins against the reference-generated fixture (bit for bit, incl.
cropped / padded state-tensor shapes and the trainer's string-op quirk), and the
batched engine builder against the oracle along random rollouts."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from golden_io import grid, meta, npz  # noqa: E402


def _trk_dict(rows):
    return {int(r[0]): {"id": int(r[0]), "status": "waiting" if r[1] == 1 else "in_transit",
                        "start_pos": (int(r[2]), int(r[3])), "target_pos": (int(r[4]), int(r[5])),
                        "start_time": int(r[6]), "deadline": int(r[7])} for r in rows}


def test_alt_helpers_golden():
    import marl_gpu.alt_helper as AH
    d = npz("alt_features.npz")
    for i, c in enumerate(meta(d)):
        g = grid(c["map"])
        rob = [tuple(int(x) for x in r) for r in d[f"robots_{i}"]]
        trk = _trk_dict(d[f"trk_{i}"])
        state = {"time_step": c["t"], "map": g.tolist(), "robots": rob, "packages": []}
        for a in range(c["A"]):
            np.testing.assert_array_equal(AH.convert_state(state, trk, a), d[f"idq_obs_{i}"][a], f"idq {i}/{a}")
        np.testing.assert_array_equal(AH.convert_state(state, trk, c["A"]), d[f"idq_obs_{i}"][0] * 0 +
                                      np.concatenate([g[None].astype(np.float32), np.zeros((5,) + g.shape,
                                                                                           np.float32)]))
        for k, sh in enumerate(c["shapes"]):
            np.testing.assert_array_equal(AH.convert_global_state_to_tensor(state, trk, sh),
                                          d[f"qmix_state_{i}_{k}"], f"qmix state {i}/{k}")
        cur = {"time_step": c["t"] + 1, "map": g.tolist(),
               "robots": [tuple(int(x) for x in r) for r in d[f"cur_robots_{i}"]], "packages": []}
        ops = d[f"ops_{i}"]
        r_int = AH.reward_shaping(state, cur, [("S", int(o)) for o in ops], trk, c["A"])
        r_str = AH.reward_shaping(state, cur, [("S", str(int(o))) for o in ops], trk, c["A"])
        assert r_int == d[f"rw_int_{i}"].tolist(), i
        assert r_str == d[f"rw_str_{i}"].tolist(), i


@pytest.mark.parametrize("mapname,A,P,T", [("map1.txt", 5, 50, 60), ("map3.txt", 8, 40, 45)])
def test_batched_alt_obs_vs_oracle(mapname, A, P, T):
    import marl_gpu
    g = grid(mapname)
    E, steps = 24, 90
    env = marl_gpu.BatchedEnv(g, E, A, P, T, seed=77, tracker="fresh")
    env.reset()
    ob = O.OracleBatch(E, g, A, P, T, seed_base=77, clear_on_reset=True)
    rs = np.random.RandomState(3)
    H, W = g.shape
    for k in range(steps):
        if k % 15 == 0 or k == steps - 1:
            out = env.build_obs_alt()
            out2 = env.build_obs_alt(state_shape=(7, H + 3, W - 2), which=("qmix_state",))
            idq = out["idq_obs"].cpu().numpy()
            qst = out["qmix_state"].cpu().numpy()
            qst2 = out2["qmix_state"].cpu().numpy()
            for e in range(E):
                s = ob.env(e).state()
                r1 = s["robots"].copy()
                r1[:, :2] += 1
                rows = ob.tracker(e).rows()
                for a in range(A):
                    np.testing.assert_array_equal(idq[e, a], O.idq_convert_state(g, s["t"], r1, rows, a),
                                                  f"idq env {e} agent {a} step {k}")
                np.testing.assert_array_equal(qst[e], O.qmix_global_tensor(g, s["t"], r1, rows, (7, H, W)))
                np.testing.assert_array_equal(qst2[e], O.qmix_global_tensor(g, s["t"], r1, rows, (7, H + 3, W - 2)))
        ints = rs.randint(0, 15, size=(E, A)).astype(np.uint8)
        env.step(torch.from_numpy(ints).cuda(), auto_reset=True)
        ob.step(ints, auto_reset=True, consts=O.QMIX_CONSTS)
    env.close()
