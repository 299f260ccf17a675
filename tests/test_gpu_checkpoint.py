"""Engine checkpoint: save, keep stepping, restore into a fresh
engine and replay -> identical rewards, done flags, observations and state, across
auto-resets (the MT19937 streams are part of the checkpoint); mismatched engines
refuse the blob."""
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


@pytest.mark.parametrize("tracker", ["mappo", "fresh"])
def test_checkpoint_resume_is_exact(tracker, tmp_path):
    mg = _mg()
    g = grid("map2.txt")
    E, A, P, T = 200, 5, 50, 37
    kw = dict(seed=123, tracker=tracker, max_packages_obs=5)
    a = mg.BatchedEnv(g, E, A, P, T, **kw)
    a.reset()
    gen = torch.Generator(device="cuda").manual_seed(4)
    acts = torch.randint(0, 15, (150, E, A), dtype=torch.uint8, device="cuda", generator=gen)
    for k in range(50):
        a.step(acts[k])
    path = tmp_path / "ckpt.npy"
    blob = a.save_state(path)
    rs, ds, obs = [], [], []
    for k in range(50, 150):                      # crosses several auto-resets (T=37)
        r, sh, d = a.step(acts[k])
        rs.append(torch.stack([r.float(), sh]).cpu())
        ds.append(d.clone().cpu())
    obs_a = {k: v.cpu() for k, v in a.build_obs().items()}
    end_a = snap(a)
    b = mg.BatchedEnv(g, E, A, P, T, **kw)        # never reset: everything comes from the blob
    b.load_state(str(path))
    for i, k in enumerate(range(50, 150)):
        r, sh, d = b.step(acts[k])
        assert torch.equal(torch.stack([r.float(), sh]).cpu(), rs[i]), k
        assert torch.equal(d.cpu(), ds[i]), k
    obs_b = {k: v.cpu() for k, v in b.build_obs().items()}
    for k in obs_a:
        assert torch.equal(obs_a[k], obs_b[k]), k
    end_b = snap(b)
    for k in end_a:
        assert np.array_equal(end_a[k], end_b[k]), k
    # the in-memory blob equals the file
    assert np.array_equal(blob, np.load(path, allow_pickle=False))


@pytest.mark.parametrize("tracker", ["mappo", "fresh"])
def test_checkpoint_restore_matches_oracle(tracker):
    """The restored stream against the CPU oracle (the reference cannot checkpoint, so the
    oracle run from the same seeds through the same actions is the external anchor): an
    engine restored from a blob taken after 50 steps is stepped through 100 more, across
    several auto-resets (T = 37: each reset draws from the restored MT19937 states), and its
    env / shaped rewards, done flags, robot and package state and tracker rows equal the
    oracle's (MAPPO/trainer.py:194-286 semantics, both tracker modes)."""
    import oracle as O
    O.build()
    mg = _mg()
    g = grid("map2.txt")
    E, A, P, T, seed = 48, 5, 50, 37, 123
    kw = dict(seed=seed, tracker=tracker, shaping="mappo", max_packages_obs=5)
    a = mg.BatchedEnv(g, E, A, P, T, **kw)
    a.reset()
    ob = O.OracleBatch(E, g, A, P, T, seed_base=seed, clear_on_reset=(tracker == "fresh"))
    rs = np.random.RandomState(11)
    acts = rs.randint(0, 15, size=(150, E, A)).astype(np.uint8)
    for k in range(50):
        a.step(torch.from_numpy(acts[k]).cuda(), auto_reset=True)
        ob.step(acts[k], auto_reset=True, consts=O.MAPPO_CONSTS)
    blob = a.save_state()
    a.close()
    b = mg.BatchedEnv(g, E, A, P, T, **kw)        # never reset: everything comes from the blob
    b.load_state(blob)
    n_done = 0
    for k in range(50, 150):
        r, sh, d = b.step(torch.from_numpy(acts[k]).cuda(), auto_reset=True)
        r0, sh0, d0 = ob.step(acts[k], auto_reset=True, consts=O.MAPPO_CONSTS)
        np.testing.assert_array_equal(r.cpu().numpy(), r0, err_msg=f"r step {k}")
        np.testing.assert_array_equal(sh.cpu().numpy(), sh0, err_msg=f"shaped step {k}")
        np.testing.assert_array_equal(d.cpu().numpy().astype(bool), d0, err_msg=f"done step {k}")
        n_done += int(d0.sum())
        if k % 10 == 0 or k == 149:
            s = snap(b)
            for e in range(E):
                os_ = ob.env(e).state()
                np.testing.assert_array_equal(s["robots"][e], os_["robots"], err_msg=f"robots env {e} step {k}")
                np.testing.assert_array_equal(s["pkgs"][e], os_["pkgs"], err_msg=f"pkgs env {e} step {k}")
                assert s["t"][e] == os_["t"] and s["total_reward"][e] == os_["total_reward"], (e, k)
                np.testing.assert_array_equal(b.tracker_rows(s, e), ob.tracker(e).rows(),
                                              err_msg=f"tracker env {e} step {k}")
    assert n_done >= 2 * E   # every env auto-reset at least twice after the restore
    b.close()


def test_checkpoint_refuses_other_configuration():
    mg = _mg()
    a = mg.BatchedEnv(grid("map1.txt"), 16, 5, 50, 100, seed=1)
    a.reset()
    blob = a.save_state()
    for other in (mg.BatchedEnv(grid("map2.txt"), 16, 5, 50, 100, seed=1),
                  mg.BatchedEnv(grid("map1.txt"), 16, 4, 50, 100, seed=1),
                  mg.BatchedEnv(grid("map1.txt"), 16, 5, 50, 100, seed=1, tracker="fresh")):
        with pytest.raises(mg.MdlError):
            other.load_state(blob)
    bad = blob.copy()
    bad[:8] = 0
    with pytest.raises(mg.MdlError):
        mg.BatchedEnv(grid("map1.txt"), 16, 5, 50, 100, seed=1).load_state(bad)


def test_checkpoint_refuses_other_constants_and_obs_dims():
    """Reward constants, shaping constants and observation dims are part of the
    checkpoint's configuration fingerprint (a snapshot used to load into
    an engine that would then compute other rewards / features)."""
    mg = _mg()
    base = dict(seed=1)
    a = mg.BatchedEnv(grid("map1.txt"), 16, 5, 50, 100, **base)
    a.reset()
    blob = a.save_state()
    mg.BatchedEnv(grid("map1.txt"), 16, 5, 50, 100, **base).load_state(blob)   # same configuration: loads
    for kw in (dict(move_cost=-0.02), dict(delivery_reward=5.0), dict(delay_reward=2.0), dict(shaping="qmix"),
               dict(max_packages_obs=100), dict(max_other_robots=10), dict(max_robots_state=10),
               dict(max_packages_state=20), dict(obs_max_time_steps=50)):
        other = mg.BatchedEnv(grid("map1.txt"), 16, 5, 50, 100, **base, **kw)
        with pytest.raises(mg.MdlError, match="constants or observation"):
            other.load_state(blob)


def test_checkpoint_carries_greedy_agents():
    """The greedy agents' records travel with the checkpoint: a restored engine's
    greedy_actions continue the saved run action for action.  A checkpoint without
    them makes an engine's own greedy records stale until greedy_init."""
    mg = _mg()
    g = grid("map1.txt")
    E, A, P, T = 64, 5, 40, 60
    a = mg.BatchedEnv(g, E, A, P, T, seed=9, tracker="fresh")
    a.reset()
    a.greedy_init()
    for _ in range(20):
        a.step(a.greedy_actions(), auto_reset=False, action_format="codes")
    blob = a.save_state()
    want = []
    for _ in range(30):
        act = a.greedy_actions()
        want.append(act.cpu())
        a.step(act, auto_reset=False, action_format="codes")
    b = mg.BatchedEnv(g, E, A, P, T, seed=9, tracker="fresh")
    b.load_state(blob)
    for k in range(30):
        act = b.greedy_actions()
        assert torch.equal(act.cpu(), want[k]), k
        b.step(act, auto_reset=False, action_format="codes")
    # a checkpoint taken before greedy_init has no greedy section
    c = mg.BatchedEnv(g, E, A, P, T, seed=9, tracker="fresh")
    c.reset()
    plain = c.save_state()
    assert plain.nbytes < blob.nbytes
    b.load_state(plain)
    with pytest.raises(mg.MdlError, match="greedy_init"):
        b.greedy_actions()
    b.greedy_init()
    b.greedy_actions()
