"""Batched greedy baseline: the reference's 100 greedy evaluation
episodes (evaluation.py:9-66 at the README.md:117-121 settings) run as 100 envs at once on
the device must reproduce every per-episode total reward and delivered count that the
reference produced; and at a larger scale the device agent matches the oracle's literal
greedyagent.py restatement action for action."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from golden_io import grid, load_json  # noqa: E402


def _mg():
    import marl_gpu
    return marl_gpu


def run_greedy_episodes(mg, g, E, A, P, T, seeds):
    env = mg.BatchedEnv(g, E, A, P, T, seeds=seeds)
    env.reset()
    env.greedy_init()
    active = np.arange(E)
    totals = np.zeros(E)
    delivered = np.zeros(E, np.int64)
    while active.size:
        ids = torch.from_numpy(active.astype(np.int32)).cuda()
        acts = env.greedy_actions(env_ids=ids)
        _, _, done = env.step(acts, env_ids=ids, auto_reset=False, action_format="codes")
        d = done.cpu().numpy().astype(bool)
        if d.any():
            s = env.read_state()
            tot = s["total_reward"].cpu().numpy()
            st = s["pkgs"][:, :, 7].cpu().numpy()
            for e in active[d]:
                totals[e] = tot[e]
                delivered[e] = int((st[e] == 3).sum())
            active = active[~d]
    env.close()
    return totals, delivered


def test_greedy_readme_anchor_batched():
    mg = _mg()
    ref = load_json("eval_anchor.json")
    cfg = ref["config"]
    E = cfg["episodes"]
    tot, dl = run_greedy_episodes(mg, grid(cfg["map"]), E, cfg["n_agents"], cfg["n_packages"],
                                  cfg["max_time_steps"], [cfg["seed"] + ep for ep in range(E)])
    assert tot.tolist() == ref["greedy"]["rewards"]
    assert dl.tolist() == ref["greedy"]["delivered"]
    assert round(float(np.mean(tot)), 2) == 34.04 and round(float(np.std(tot)), 2) == 14.83


@pytest.mark.parametrize("mapname,A,P,T", [("map2.txt", 8, 60, 300), ("map4.txt", 5, 40, 200)])
def test_greedy_vs_oracle_actions(mapname, A, P, T):
    mg = _mg()
    g = grid(mapname)
    E = 48
    seeds = [500 + i for i in range(E)]
    env = mg.BatchedEnv(g, E, A, P, T, seeds=seeds)
    env.reset()
    env.greedy_init()
    envs = []
    for s in seeds:
        o = O.OracleEnv(g, A, P, T, seed=s)
        o.reset()
        envs.append((o, O.OracleGreedy(o)))
    for k in range(T):
        acts = env.greedy_actions().cpu().numpy()
        for e, (o, ag) in enumerate(envs):
            mv, op = ag.actions(o)
            np.testing.assert_array_equal(acts[e] & 7, mv, err_msg=f"move env {e} step {k}")
            np.testing.assert_array_equal(acts[e] >> 3, op, err_msg=f"op env {e} step {k}")
            o.step(mv, op)
        env.step(torch.from_numpy(acts).cuda(), auto_reset=False, action_format="codes")
    env.close()
