"""Device-resident rollout glue: MappoRollout replays the
reference-generated MAPPO rollout fixture through on-device sampling, stepping and
featurization into the rollout buffers (bit-exact vs the fixture), GAE matches the
reference's float32 expression bit for bit, and the sampler is checked against its
numpy restatement (Philox4x32-10 + inverse CDF) and against softmax statistics."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from golden_io import grid, meta, npz  # noqa: E402

GAMMA, GAE_LAMBDA = 0.99, 0.95  # MAPPO/trainer.py:53-54


def _mg():
    import marl_gpu
    import marl_gpu.rollout as R
    return marl_gpu, R


def ref_gae(rewards, values, next_value, dones):
    """MAPPO/trainer.py:266-276 restated on CPU torch tensors (float32, same expression order)."""
    T = rewards.shape[0]
    advantages = torch.zeros_like(rewards)
    last = 0
    for t in reversed(range(T)):
        nnt = 1.0 - dones[t].float()
        nv = next_value if t == T - 1 else values[t + 1]
        delta = rewards[t] + GAMMA * nv * nnt - values[t]
        advantages[t] = last = delta + GAMMA * GAE_LAMBDA * nnt * last
    return advantages, advantages + values


def test_gae_bitwise_vs_reference_expression():
    _, R = _mg()
    g = torch.Generator().manual_seed(0)
    T, n = 97, 3001
    r = torch.randn(T, n, generator=g) * 3
    v = torch.randn(T, n, generator=g)
    nv = torch.randn(n, generator=g)
    d = torch.rand(T, n, generator=g) < 0.05
    a0, ret0 = ref_gae(r, v, nv, d)
    a1, ret1 = R.gae(r.cuda(), v.cuda(), nv.cuda(), d.cuda(), GAMMA, GAE_LAMBDA)
    assert torch.equal(a1.cpu().view(torch.int32), a0.view(torch.int32))
    assert torch.equal(ret1.cpu().view(torch.int32), ret0.view(torch.int32))


def philox(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 on numpy uint32 arrays (restatement for the sampler test)."""
    c = [np.asarray(x, np.uint64) for x in (c0, c1, c2, c3)]
    k0, k1 = np.uint64(k0), np.uint64(k1)
    M = np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c[0]
        p1 = np.uint64(0xCD9E8D57) * c[2]
        c = [((p1 >> np.uint64(32)) ^ c[1] ^ k0) & M, p1 & M, ((p0 >> np.uint64(32)) ^ c[3] ^ k1) & M, p0 & M]
        k0 = (k0 + np.uint64(0x9E3779B9)) & M
        k1 = (k1 + np.uint64(0xBB67AE85)) & M
    return c[0].astype(np.uint32)


def test_sampler_matches_restatement_and_softmax():
    _, R = _mg()
    N, K = 200_000, 15
    g = torch.Generator().manual_seed(1)
    logits = torch.randn(N, K, generator=g) * 2
    seed, off = 0x1234_5678_9ABC_DEF0, 7
    a, lp = R.sample_actions(logits.cuda(), seed, off)
    a, lp = a.cpu().numpy(), lp.cpu()
    a2, _ = R.sample_actions(logits.cuda(), seed, off)
    assert np.array_equal(a, a2.cpu().numpy())                       # deterministic
    # log_prob == log_softmax gather (float32 tolerance)
    ref_lp = torch.log_softmax(logits, dim=1).gather(1, torch.from_numpy(a.astype(np.int64))[:, None])[:, 0]
    assert torch.allclose(lp, ref_lp, atol=3e-6, rtol=0)
    # inverse CDF on the restated Philox uniform (fp64), skipping rows within 1e-5 of a bin edge
    rows = np.arange(N, dtype=np.uint64)
    u = (philox(off & 0xFFFFFFFF, off >> 32, rows & 0xFFFFFFFF, rows >> 32, seed & 0xFFFFFFFF, seed >> 32) >> 8)
    u = u.astype(np.float64) * 2.0 ** -24
    x = logits.double().numpy()
    p = np.exp(x - x.max(1, keepdims=True))
    cdf = np.cumsum(p, 1) / p.sum(1, keepdims=True)
    ref = (u[:, None] >= cdf).sum(1)
    safe = np.abs(cdf - u[:, None]).min(1) > 1e-5
    assert safe.mean() > 0.99
    assert np.array_equal(a[safe], ref[safe])
    # statistics: one logit row repeated, chi-square against softmax
    row = torch.tensor([[0.3, -1.0, 2.0, 0.0, 0.5, -3.0, 1.0, 0.2, -0.5, 0.7, 0.0, -2.0, 1.5, 0.1, -0.1]])
    b, _ = R.sample_actions(row.repeat(N, 1).cuda(), 99, 0)
    cnt = np.bincount(b.cpu().numpy(), minlength=K)
    exp = torch.softmax(row.double(), 1)[0].numpy() * N
    chi2 = ((cnt - exp) ** 2 / exp).sum()
    assert chi2 < 45.0  # 14 dof: p ~ 5e-5


def test_sampler_masked_logits_exact():
    _, R = _mg()
    N, K = 4096, 15
    pick = torch.randint(0, K, (N,), generator=torch.Generator().manual_seed(2))
    logits = torch.full((N, K), float("-inf"))
    logits[torch.arange(N), pick] = 0.0
    a, lp = R.sample_actions(logits.cuda(), 5, 3)
    assert torch.equal(a.cpu().long(), pick)
    assert torch.equal(lp.cpu(), torch.zeros(N))


def test_mappo_rollout_replays_reference_fixture():
    """MAPPO/trainer.py:154-290 with a policy that replays the fixture's actions: every
    buffer the reference fills must equal the reference-generated fixture."""
    mg, R = _mg()
    d = npz("rollout_mappo.npz")
    m = meta(d)
    E, A, P, T = m["E"], m["A"], m["P"], m["T"]
    env = mg.BatchedEnv(grid(m["map"]), E, A, P, T, seed=m["seed"], tracker="mappo", shaping="mappo",
                        max_other_robots=m["MO"], max_packages_obs=m["MP"], max_robots_state=m["MR"],
                        max_packages_state=m["MPs"])
    env.reset()
    acts = torch.from_numpy(d["acts"].astype(np.int64)).cuda()
    k_total = acts.shape[0]
    half = k_total // 2
    state = {"k": 0}

    def actor(obs, vec):
        lg = torch.full((E * A, 15), float("-inf"), device="cuda")
        lg[torch.arange(E * A, device="cuda"), acts[state["k"]].reshape(-1)] = 0.0
        state["k"] += 1
        return lg

    def critic(gmap, gvec):
        return gvec[:, -1] * 0.5 + gvec[:, 0]

    for seg, steps in ((0, half), (half, k_total - half)):
        ro = R.MappoRollout(env, steps, seed=11)
        out = ro.collect(actor, critic)
        torch.cuda.synchronize()
        for j in range(steps):
            k = seg + j
            np.testing.assert_array_equal(ro.mb_obs[j].cpu().numpy(), d["amap"][k].astype(np.float32), f"amap {k}")
            np.testing.assert_array_equal(ro.mb_vector_obs[j].cpu().numpy(), d["avec"][k], f"avec {k}")
            np.testing.assert_array_equal(ro.mb_global_states[j].cpu().numpy(), d["cmap"][k].astype(np.float32))
            np.testing.assert_array_equal(ro.mb_global_vector[j].cpu().numpy(), d["cvec"][k], f"cvec {k}")
            np.testing.assert_array_equal(ro.mb_actions[j].cpu().numpy(), d["acts"][k])
            np.testing.assert_array_equal(ro.mb_rewards[j].cpu().numpy(), d["r_shaped"][k], f"reward {k}")
            np.testing.assert_array_equal(ro.mb_dones[j].cpu().numpy().astype(bool), d["done"][k], f"done {k}")
        assert torch.equal(ro.mb_log_probs.cpu(), torch.zeros_like(ro.mb_log_probs.cpu()))
        k_next = seg + steps
        np.testing.assert_array_equal(ro.next_obs["critic_vec"].cpu().numpy(), d["cvec"][k_next])
        # GAE against the reference expression on CPU with the same (exact) critic values
        cv = torch.from_numpy(d["cvec"][seg:k_next + 1])
        vals = cv[:, :, -1] * 0.5 + cv[:, :, 0]
        a0, r0 = ref_gae(torch.from_numpy(d["r_shaped"][seg:k_next]), vals[:-1], vals[-1],
                         torch.from_numpy(d["done"][seg:k_next]))
        b_adv, b_ret = out[6], out[7]
        assert torch.equal(b_ret.cpu().view(torch.int32), r0.reshape(-1).view(torch.int32))
        assert torch.equal(b_adv.cpu().view(torch.int32),
                           a0.reshape(steps * E, 1).repeat(1, A).reshape(-1).view(torch.int32))
        assert out[0].shape == (steps * E * A, 6, 10, 10) and out[4].dtype == torch.long
    env.close()


def test_graph_rollout_bitwise_equals_eager():
    """collect(graph=True) -- the whole rollout captured once and replayed, with the
    sampler's offset base on the device -- produces exactly the eager rollouts."""
    mg, R = _mg()
    g = grid("map1.txt")
    E, A, P, T, steps = 64, 5, 50, 60, 24

    def make():
        env = mg.BatchedEnv(g, E, A, P, T, seed=7, tracker="mappo", shaping="mappo", max_other_robots=A - 1,
                            max_packages_obs=5)
        env.reset()
        return env

    gen = torch.Generator(device="cuda").manual_seed(3)
    env0 = make()
    wa = torch.randn(env0.actor_vec_dim, 15, device="cuda", generator=gen)
    wc = torch.randn(env0.critic_vec_dim, device="cuda", generator=gen) * 0.01

    def actor(obs, vec):
        return vec @ wa + obs.sum(dim=(1, 2, 3)).unsqueeze(1) * 0.01

    def critic(gmap, gvec):
        return gvec @ wc

    eager = R.MappoRollout(env0, steps, seed=5)
    env1 = make()
    graphed = R.MappoRollout(env1, steps, seed=5)
    for k in range(4):   # call 0 runs eagerly and captures; calls 1..3 replay the graph
        a = [x.clone() for x in eager.collect(actor, critic)]
        b = [x.clone() for x in graphed.collect(actor, critic, graph=True)]
        torch.cuda.synchronize()
        for i, (x, y) in enumerate(zip(a, b)):
            assert torch.equal(x, y), f"rollout {k}, output {i}"
    assert graphed._graph is not None and eager.offset == graphed.offset
    s0, s1 = env0.read_state(), env1.read_state()
    for key in s0:
        assert torch.equal(s0[key], s1[key]), key
    env0.close()
    env1.close()
