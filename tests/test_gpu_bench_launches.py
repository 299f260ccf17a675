"""The exact launches bench.py times, at the sizes it times them, against the oracle (VERDICT r05
item 1).

* Config 3: ``bench.py --config 3`` times ``BatchedEnv.step_obs`` over 16,384 map1 envs -- the
  fused ``k_step_obs<true, 5>`` launch (step + MAPPO shaped reward + tracker + auto-reset, then the
  6-ch actor maps, 52-dim actor vectors, 4-ch critic map and 1301-dim critic vector of the new
  state; MAPPO/trainer.py:229-286, MAPPO/helper.py:6-255).  Here the same launch runs 45 steps
  across an auto-reset (T = 30); 16 envs spread over workgroups and XCD slots (2,048-env slot
  ranges) are replayed by the oracle from their seeds: rewards, shaped rewards and dones every
  step, all four observation tensors every step.
* Config 4: ``bench.py --config 4`` at one GPU times ONE ``k_step_rows<true, 5, 4, 3>`` launch over
  65,536 envs of map1..map5 (contiguous map groups, seeds 42 + global id).  Here that batch runs 45
  steps across an auto-reset with oracle windows at the start, at every map-group boundary
  (13,108, 26,215, 39,322, 52,429) and at the last wave; state, tracker rows and vectors at the end.
* Config 5: ``bench.py --config 5`` at one GPU times ONE ``k_step_halves<true, 3>`` launch over 131,072
  envs (64x64, 16 robots, 100 packages); the same batch runs 45 steps across an auto-reset with
  oracle windows at the start, the middle, an XCD-slot boundary and the last wave.
* The tests assert which kernel the engine launched (``mdl_last_step_layout`` /
  ``mdl_step_kernel_name``), the record bench.py labels its roofline with.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from golden_io import grid  # noqa: E402

OBS3 = dict(max_other_robots=4, max_packages_obs=5, max_robots_state=100, max_packages_state=100)


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    O.build()


def test_config3_fused_step_obs_16384_vs_oracle():
    import marl_gpu as mg
    g = grid("map1.txt")
    E, A, P, T, W = 16384, 5, 50, 30, 2
    env = mg.BatchedEnv(g, E, A, P, T, seed=42, tracker="mappo", shaping="mappo", **OBS3)
    env.reset()
    assert env.step_kernel_name(with_obs=True) == "mdl::k_step_obs<true, 5>"
    # 8 windows of 2 envs: the first / last envs, workgroup (4 envs) and XCD-slot (2,048 envs) boundaries
    starts = [0, 1023, 2047, 4095, 6143, 8191, 12286, E - W]
    wins = [(s, O.OracleBatch(W, g, A, P, T, seed_base=42 + s, clear_on_reset=False)) for s in starts]
    sel = torch.tensor([s + i for s in starts for i in range(W)], dtype=torch.int64, device="cuda")
    bufs = env.obs_buffers()
    gen = np.random.RandomState(33)
    dones = 0
    for k in range(45):
        ints = gen.randint(0, 15, size=(E, A)).astype(np.uint8)
        r, sh, d, o = env.step_obs(torch.from_numpy(ints).cuda(), obs_out=bufs)
        rh, shh, dh = r.cpu().numpy(), sh.cpu().numpy(), d.cpu().numpy().astype(bool)
        got = {key: o[key].index_select(0, sel).cpu().numpy() for key in ("actor_map", "actor_vec", "critic_map",
                                                                          "critic_vec")}
        dones += int(dh.sum())
        for i, (s, ob) in enumerate(wins):
            r0, s0, d0 = ob.step(ints[s:s + W], auto_reset=True, consts=O.MAPPO_CONSTS)
            np.testing.assert_array_equal(rh[s:s + W], r0, err_msg=f"r_env step {k} envs {s}+")
            np.testing.assert_array_equal(shh[s:s + W], s0, err_msg=f"shaped step {k} envs {s}+")
            np.testing.assert_array_equal(dh[s:s + W], d0, err_msg=f"done step {k} envs {s}+")
            want = ob.obs(T, OBS3["max_other_robots"], OBS3["max_packages_obs"], OBS3["max_robots_state"],
                          OBS3["max_packages_state"])
            for key in got:
                np.testing.assert_array_equal(got[key][i * W:(i + 1) * W], want[key],
                                              err_msg=f"{key} step {k} envs {s}+")
    assert dones == E   # every env crossed its auto-reset at t = T inside the checked steps
    env.close()


def test_config4_rows_65536_five_maps_vs_oracle():
    import marl_gpu as mg
    from marl_gpu import dist as D
    total, A, P, T, W = 65536, 5, 50, 30, 8
    sizes = D.map_group_sizes(total, 5)
    bounds = np.cumsum([0] + sizes)
    grids = [grid(f"map{i}.txt") for i in range(1, 6)]
    env_map = np.repeat(np.arange(5), sizes)
    seeds = [42 + e for e in range(total)]
    env = mg.BatchedEnv(grids, total, A, P, T, seeds=seeds, env_map=env_map, tracker="mappo", shaping="mappo",
                        max_packages_obs=5)
    env.reset()
    assert env.step_layout() == "rows" and env.step_kernel_name() == "mdl::k_step_rows<true, 5, 4, 3>"
    # windows inside one map group each: the first envs, both sides of every group boundary, the last wave
    wins = [(0, 0)]
    for m in range(1, 5):
        wins += [(m - 1, int(bounds[m]) - W), (m, int(bounds[m]))]
    wins.append((4, total - W))
    wins = [(m, s, O.OracleBatch(W, grids[m], A, P, T, seed_base=42 + s, clear_on_reset=False)) for m, s in wins]
    gen = np.random.RandomState(44)
    dones = 0
    for k in range(45):
        ints = gen.randint(0, 15, size=(total, A)).astype(np.uint8)
        r, sh, d = env.step(torch.from_numpy(ints).cuda())
        assert env.last_step_layout() == "rows"
        rh, shh, dh = r.cpu().numpy(), sh.cpu().numpy(), d.cpu().numpy().astype(bool)
        dones += int(dh.sum())
        for m, s, ob in wins:
            r0, s0, d0 = ob.step(ints[s:s + W], auto_reset=True, consts=O.MAPPO_CONSTS)
            np.testing.assert_array_equal(rh[s:s + W], r0, err_msg=f"r_env step {k} envs {s}+ (map{m + 1})")
            np.testing.assert_array_equal(shh[s:s + W], s0, err_msg=f"shaped step {k} envs {s}+ (map{m + 1})")
            np.testing.assert_array_equal(dh[s:s + W], d0, err_msg=f"done step {k} envs {s}+ (map{m + 1})")
    assert dones == total
    st = env.read_state()
    torch.cuda.synchronize()
    st = {k: v.cpu().numpy() for k, v in st.items()}
    for m, s, ob in wins:
        H, Wd = grids[m].shape
        o = env.build_obs(env_begin=s, n=W)
        av, cv = o["actor_vec"].cpu().numpy(), o["critic_vec"].cpu().numpy()
        for i in range(W):
            oe, ot = ob.env(i), ob.tracker(i)
            os_ = oe.state()
            assert st["t"][s + i] == os_["t"]
            np.testing.assert_array_equal(st["robots"][s + i], os_["robots"])
            np.testing.assert_array_equal(st["pkgs"][s + i], os_["pkgs"])
            assert st["total_reward"][s + i] == os_["total_reward"]
            np.testing.assert_array_equal(env.tracker_rows(st, s + i), ot.rows(), err_msg=f"tracker env {s + i}")
            rb1, rows = oe.robots1(), ot.rows()
            want = np.stack([O.generate_vector_features(H, Wd, os_["t"], rb1, rows, a, T, A - 1, 5) for a in range(A)])
            np.testing.assert_array_equal(av[i], want)
            _, gv = O.convert_global_state(grids[m], os_["t"], rb1, rows, T, 100, 100)
            np.testing.assert_array_equal(cv[i], gv)
    env.close()


def test_config5_halves_131072_vs_oracle():
    """Config 5 at one GPU: ``bench.py --config 5`` times ONE ``k_step_halves<true, 3>`` launch over
    131,072 envs of the 64x64 map (16 robots, 100 packages; the layout AUTO takes there).  Here that
    batch runs 45 steps across an auto-reset (T = 30) with oracle windows at the start, around the
    middle, at an XCD-slot boundary and at the last wave: rewards, shaped rewards and dones every
    step, state and tracker rows at the end."""
    import marl_gpu as mg
    g = grid("synthetic64.txt")
    E, A, P, T, W = 131072, 16, 100, 30, 6
    env = mg.BatchedEnv(g, E, A, P, T, seed=42, tracker="mappo", shaping="mappo", max_other_robots=15,
                        max_packages_obs=20, max_robots_state=16, max_packages_state=100)
    env.reset()
    assert env.step_layout() == "halves" and env.step_kernel_name() == "mdl::k_step_halves<true, 3>"
    starts = [0, 16381, 65533, 98304 - 3, E - W]
    wins = [(s, O.OracleBatch(W, g, A, P, T, seed_base=42 + s, clear_on_reset=False)) for s in starts]
    gen = np.random.RandomState(55)
    dones = 0
    for k in range(45):
        ints = gen.randint(0, 15, size=(E, A)).astype(np.uint8)
        r, sh, d = env.step(torch.from_numpy(ints).cuda())
        assert env.last_step_layout() == "halves"
        rh, shh, dh = r.cpu().numpy(), sh.cpu().numpy(), d.cpu().numpy().astype(bool)
        dones += int(dh.sum())
        for s, ob in wins:
            r0, s0, d0 = ob.step(ints[s:s + W], auto_reset=True, consts=O.MAPPO_CONSTS)
            np.testing.assert_array_equal(rh[s:s + W], r0, err_msg=f"r_env step {k} envs {s}+")
            np.testing.assert_array_equal(shh[s:s + W], s0, err_msg=f"shaped step {k} envs {s}+")
            np.testing.assert_array_equal(dh[s:s + W], d0, err_msg=f"done step {k} envs {s}+")
    assert dones == E
    st = env.read_state()
    torch.cuda.synchronize()
    st = {k: v.cpu().numpy() for k, v in st.items()}
    for s, ob in wins:
        for i in range(W):
            os_ = ob.env(i).state()
            assert st["t"][s + i] == os_["t"] and st["total_reward"][s + i] == os_["total_reward"]
            np.testing.assert_array_equal(st["robots"][s + i], os_["robots"])
            np.testing.assert_array_equal(st["pkgs"][s + i], os_["pkgs"])
            np.testing.assert_array_equal(env.tracker_rows(st, s + i), ob.tracker(i).rows(), err_msg=f"env {s + i}")
    env.close()
