"""world_size-2 gloo check of the multi-GPU sharding (CPU only).

Each rank takes its shard of global env ids / seeds from marl_gpu.dist, runs
that shard's env streams (here through the CPU oracle, standing in for the
per-GPU engine) and the ranks all-gather their rewards; the result must equal
one process running every env -- i.e. sharding changes no env's stream.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, out_q):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(repo, "marl-delivery_amd"), os.path.join(repo, "oracle"), os.path.join(repo, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from marl_gpu import dist as D
    import oracle as O
    from golden_io import grid
    r, w, _ = D.world()
    assert (r, w) == (rank, world)
    base, per, total = 42, 6, 11
    if mode == "weak":
        ids, seeds = D.shard(per, r, base)
    else:
        ids, seeds = D.shard_strong(total, r, w, base)
    g = grid("map1.txt")
    E = len(ids)
    ob = O.OracleBatch(E, g, 5, 20, 30, seed_base=seeds[0], clear_on_reset=False)
    rs = np.random.RandomState(3)
    n_global = per * w if mode == "weak" else total
    rewards = []
    for k in range(45):
        acts = rs.randint(0, 15, size=(n_global, 5)).astype(np.uint8)
        rr, sh, dn = ob.step(acts[ids[0]:ids[0] + E], auto_reset=True, consts=O.MAPPO_CONSTS)
        rewards.append(np.stack([rr, sh.astype(np.float64), dn.astype(np.float64)], 1))
    mine = torch.from_numpy(np.stack(rewards, 0))            # [K, E, 3]
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(w)]
    dist.all_gather(sizes, torch.tensor([E]))
    mx = int(max(s.item() for s in sizes))
    pad = torch.zeros(mine.shape[0], mx, 3, dtype=mine.dtype)
    pad[:, :E] = mine
    parts = [torch.zeros_like(pad) for _ in range(w)]
    dist.all_gather(parts, pad)
    t_max = D.max_over_ranks([float(rank + 1), 2.0])
    if rank == 0:
        full = torch.cat([p[:, :int(s.item())] for p, s in zip(parts, sizes)], 1).numpy()
        out_q.put((full, t_max))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["weak", "strong"])
def test_sharded_streams_equal_single_process(mode):
    import oracle as O
    from golden_io import grid
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    full, t_max = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert t_max == [2.0, 2.0]
    n = 12 if mode == "weak" else 11
    ob = O.OracleBatch(n, grid("map1.txt"), 5, 20, 30, seed_base=42, clear_on_reset=False)
    rs = np.random.RandomState(3)
    for k in range(45):
        acts = rs.randint(0, 15, size=(n, 5)).astype(np.uint8)
        rr, sh, dn = ob.step(acts, auto_reset=True, consts=O.MAPPO_CONSTS)
        np.testing.assert_array_equal(full[k, :, 0], rr)
        np.testing.assert_array_equal(full[k, :, 1], sh.astype(np.float64))
        np.testing.assert_array_equal(full[k, :, 2], dn.astype(np.float64))


def test_shard_partitions():
    from marl_gpu import dist as D
    for total in (1, 7, 4096, 65536):
        for w in (1, 2, 3, 8):
            ids = []
            for r in range(w):
                i, s = D.shard_strong(total, r, w, 10)
                assert s == [10 + x for x in i]
                ids += i
            assert ids == list(range(total))
    i, s = D.shard(4096, 3, 42)
    assert i[0] == 3 * 4096 and s[0] == 42 + 3 * 4096 and len(i) == 4096
