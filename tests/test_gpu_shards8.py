"""The driver's 8-GPU layouts at full size, one rank at a time on the HIP engine, against the
oracle at the same global seeds.

BASELINE config 4 (65,536 mixed-map envs over 8 ranks): rank r owns the contiguous global ids
``dist.shard_mixed(65536, 5, r, 8, 42)`` deals it, seeded ``42 + global id``
(MAPPO/env_vectorized.py:4-10).  Rank 1 (global ids 8192-16383) crosses the map1 -> map2 group
boundary at 13108; rank 7 is all map5.  Each rank's shard is stepped on the GPU for 520 steps
(past the T = 500 auto-reset) and windows of envs at the start, the middle and the end of every
same-map run are replayed by the oracle from their global seeds: env reward, shaped reward and
done bit for bit every step, state and tracker rows and the actor / critic vectors at the end.

Also: bench.py under torch.distributed.run on the RCCL (nccl) backend with one rank, the code
path the driver's multi-GPU run takes (process group on the device, device-tensor MAX)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402
from golden_io import grid  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAPS = [f"map{i}.txt" for i in range(1, 6)]


@pytest.fixture(scope="module", autouse=True)
def _setup():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device")
    O.build()


@pytest.mark.parametrize("rank", [1, 7])
def test_config4_rank_of_eight_vs_oracle(rank):
    import marl_gpu as mg
    from marl_gpu import dist as D
    total, world, A, P, T, W = 65536, 8, 5, 50, 500, 12
    ids, seeds, env_map, runs = D.shard_mixed(total, 5, rank, world, 42)
    E = len(ids)
    assert E == total // world and ids == list(range(rank * E, (rank + 1) * E))
    assert seeds == [42 + g for g in ids]
    if rank == 1:   # the map1 group is global ids [0, 13108): the shard holds its tail and map2's head
        assert [(m, b, n) for m, b, n in runs] == [(0, 0, 13108 - 8192), (1, 13108 - 8192, 16384 - 13108)]
    else:
        assert [m for m, _, _ in runs] == [4]
    grids = [grid(m) for m in MAPS]
    env = mg.BatchedEnv(grids, E, A, P, T, seeds=seeds, env_map=env_map, tracker="mappo", shaping="mappo",
                        max_packages_obs=5)
    env.reset()
    # oracle windows: W consecutive envs at the start, middle and end of every same-map run
    wins = []
    for m, b, n in runs:
        for s in sorted({b, b + n // 2 - W // 2, b + n - W}):
            wins.append((m, s, O.OracleBatch(W, grids[m], A, P, T, seed_base=int(seeds[s]), clear_on_reset=False)))
    gen = np.random.RandomState(100 + rank)
    dones = 0
    for k in range(520):
        ints = gen.randint(0, 15, size=(E, A)).astype(np.uint8)
        r, sh, d = env.step(torch.from_numpy(ints).cuda(), auto_reset=True)
        rh, shh, dh = r.cpu().numpy(), sh.cpu().numpy(), d.cpu().numpy().astype(bool)
        for m, s, ob in wins:
            r0, s0, d0 = ob.step(ints[s:s + W], auto_reset=True, consts=O.MAPPO_CONSTS)
            np.testing.assert_array_equal(rh[s:s + W], r0, err_msg=f"r_env step {k} envs {s}+")
            np.testing.assert_array_equal(shh[s:s + W], s0, err_msg=f"shaped step {k} envs {s}+")
            np.testing.assert_array_equal(dh[s:s + W], d0, err_msg=f"done step {k} envs {s}+")
        dones += int(dh.sum())
    assert dones == E   # every env finished its episode at t = T and was reset
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
            rb1, rows = oe.robots1(), ot.rows()
            want = np.stack([O.generate_vector_features(H, Wd, os_["t"], rb1, rows, a, T, A - 1, 5) for a in range(A)])
            np.testing.assert_array_equal(av[i], want)
            _, gv = O.convert_global_state(grids[m], os_["t"], rb1, rows, T, 100, 100)
            np.testing.assert_array_equal(cv[i], gv)
    env.close()


def test_bench_torchrun_rccl_one_rank():
    """bench.py's RCCL path (bench.py: init_process_group("nccl", device_id=...) and the device-tensor
    all_reduce MAX of the per-rank clocks) under the driver's launcher, one rank on the one GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29571", os.path.join(REPO, "bench.py"),
           "--gpus", "1", "--backend", "nccl", "--steps", "40", "--warmup", "5", "--cpu-seconds", "0"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["steps"] == 40 and d["scaling"] == "weak"
    assert d["value"] == pytest.approx(4096 * 5 * 40 / (d["ms_per_step"] * 40 / 1e3), rel=1e-9)
    assert d["roofline"]["achieved"] > 0 and d["cpu_baseline"] is None   # --cpu-seconds 0
