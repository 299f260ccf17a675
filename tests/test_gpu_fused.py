"""Bench mode: mdl_step_fused must equal K mdl_step calls
bit for bit -- rewards, shaped rewards, done flags and the whole final state,
across auto-resets, in both tracker modes and for P > 64 (two package chunks)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from golden_io import grid  # noqa: E402


def _mg():
    import marl_gpu
    return marl_gpu


def snap(env):
    s = env.read_state()
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in s.items()}


@pytest.mark.parametrize("tracker,P,T,E", [("mappo", 50, 23, 512), ("fresh", 50, 23, 512), ("mappo", 100, 17, 256)])
def test_fused_equals_sequential(tracker, P, T, E):
    mg = _mg()
    g = grid("map1.txt")
    K = 60
    kw = dict(seed=7, tracker=tracker)
    a = mg.BatchedEnv(g, E, 5, P, T, **kw)
    b = mg.BatchedEnv(g, E, 5, P, T, **kw)
    a.reset()
    b.reset()
    gen = torch.Generator(device="cuda").manual_seed(3)
    acts = torch.randint(0, 15, (K, E, 5), dtype=torch.uint8, device="cuda", generator=gen)
    rs, shs, ds = [], [], []
    for k in range(K):
        r, sh, d = a.step(acts[k])
        rs.append(r.clone())
        shs.append(sh.clone())
        ds.append(d.clone())
    r2, sh2, d2 = b.step_fused(acts)
    torch.cuda.synchronize()
    assert torch.equal(torch.stack(rs), r2)
    assert torch.equal(torch.stack(shs).view(torch.int32), sh2.view(torch.int32))
    assert torch.equal(torch.stack(ds), d2)
    assert int(d2.sum()) > 0  # the window crosses auto-resets
    sa, sb = snap(a), snap(b)
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    # and both keep stepping identically afterwards
    r, sh, d = a.step(acts[0])
    r3, sh3, d3 = b.step(acts[0])
    assert torch.equal(r, r3) and torch.equal(sh.view(torch.int32), sh3.view(torch.int32))


def test_fused_env_subset():
    mg = _mg()
    g = grid("map1.txt")
    E, K = 300, 25
    a = mg.BatchedEnv(g, E, 5, 50, 11, seed=5, tracker="mappo")
    b = mg.BatchedEnv(g, E, 5, 50, 11, seed=5, tracker="mappo")
    a.reset()
    b.reset()
    ids = torch.arange(3, E, 7, dtype=torch.int32, device="cuda")
    n = ids.numel()
    gen = torch.Generator(device="cuda").manual_seed(9)
    acts = torch.randint(0, 15, (K, n, 5), dtype=torch.uint8, device="cuda", generator=gen)
    for k in range(K):
        a.step(acts[k], env_ids=ids)
    b.step_fused(acts, env_ids=ids)
    sa, sb = snap(a), snap(b)
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
