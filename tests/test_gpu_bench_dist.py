"""bench.py's multi-rank path (the driver's `torch.distributed.run --nproc-per-node N
bench.py --gpus N`) rehearsed on one GPU: two ranks with the gloo backend share the
device, each steps its own env shard (weak scaling) or its part of one batch (strong
scaling), and rank 0 prints one JSON line with the whole-job value."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(extra, port):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "40", "--warmup", "5", "--cpu-seconds", "0", "--fused-k", "0",
           "--backend", "gloo", "--envs", "512"] + extra
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout   # rank 0 only
    return json.loads(lines[0])


def test_bench_two_ranks_weak_scaling():
    d = _run([], 29561)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["steps"] == 40
    assert d["config"]["total_envs"] == 1024 and d["config"]["envs_per_gpu"] == 512
    assert d["value"] > 0 and d["value"] == pytest.approx(1024 * 5 * 40 / (d["ms_per_step"] * 40 / 1e3), rel=1e-9)
    assert d["cpu_baseline"] is None   # rank 0 at N = 1 only


def test_bench_two_ranks_strong_scaling():
    d = _run(["--total-envs", "1000"], 29563)
    assert d["scaling"] == "strong" and d["config"]["total_envs"] == 1000
    assert d["config"]["envs_per_gpu"] == 500


def test_bench_two_ranks_config4_mixed_maps():
    """BASELINE config 4's command at rehearsal size: map1..map5 groups over the ranks."""
    d = _run(["--config", "4", "--total-envs", "2000"], 29565)
    assert d["scaling"] == "strong" and d["config"]["total_envs"] == 2000 and d["config"]["envs_per_gpu"] == 1000
    assert d["config"]["maps"] == [f"map{i}.txt" for i in range(1, 6)]
    assert d["config"]["map_runs_rank0"] == [["map1.txt", 0, 400], ["map2.txt", 400, 400], ["map3.txt", 800, 200]]
    assert d["value"] > 0


def test_bench_two_ranks_config5():
    """BASELINE config 5's command at rehearsal size: 64x64, 16 agents, 100 packages."""
    d = _run(["--config", "5", "--total-envs", "1024"], 29567)
    assert d["config"]["agents"] == 16 and d["config"]["packages"] == 100 and d["config"]["envs_per_gpu"] == 512
    assert d["value"] > 0

