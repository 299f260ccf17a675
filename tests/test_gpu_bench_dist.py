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
    assert d["cpu_baseline"] is None   # --cpu-seconds 0
    assert d["ranks_seen"] == 2


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



def _plain(args, timeout=300):
    """bench.py as the driver's plain command (no torchrun around it)."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=env,
                         capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), out.stdout   # exactly rank 0's JSON line
    return json.loads(lines[0])


def test_bench_plain_command_two_gpus_self_launches():
    """`python3 bench.py --gpus 2 --backend gloo --steps 40 --warmup 5` as a plain
    command starts torch.distributed.run itself; the line says how many ranks the process group saw,
    which devices they ran on, and carries the CPU baseline (timed on rank 0 after the timed region)."""
    d = _plain(["--gpus", "2", "--backend", "gloo", "--steps", "40", "--warmup", "5", "--cpu-seconds", "1",
                "--fused-k", "0", "--gather"])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["launcher"] == "self"
    assert d["process_group_backend"] == "gloo"
    assert sorted(x["rank"] for x in d["devices"]) == [0, 1] and all("gfx950" in x["arch"] for x in d["devices"])
    assert d["distinct_devices"] == 1   # gloo rehearsal: both ranks share the box's one GPU
    assert d["config"]["total_envs"] == 2 * 4096 and d["scaling"] == "weak"
    cpu = d["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["host"]["nproc"] >= 1
    assert d["cpu_baseline_1thread"]["threads_note"].startswith("single thread")
    # the launch floor beside the step: an empty kernel in the step's launch shape
    assert 0 < d["launch_floor_ms_per_step"] and d["over_floor_us"] == pytest.approx(
        (d["ms_per_step"] - d["launch_floor_ms_per_step"]) * 1e3)
    # the metric's own workload at N ranks -- 4,096 envs in TOTAL split over them --
    # as a second timed region beside the weak one, and the reference's CPU figures, labelled
    s = d["strong_4096"]
    assert s["total_envs"] == 4096 and s["envs_per_rank"] == [2048, 2048] and s["scaling"] == "strong"
    assert s["value"] == pytest.approx(4096 * 5 * s["steps"] / (s["ms_per_step"] * s["steps"] / 1e3), rel=1e-9)
    assert s["launch_floor_ms_per_step"] > 0 and s["step_layout"] == "wave"
    rc = d["reference_cpu"]
    assert rc["serial_1core"] == 195453.0 and rc["processes_8"] == 1650597.0 and "BASELINE.md" in rc["source"]
    # the optional rollout gather leg (gloo here: a rehearsal through host memory)
    g = d["rollout_gather"]
    assert g["gathered_bytes"] == 2 * 4096 * 1301 * 4 and g["bytes_per_rank"] == 4096 * 1301 * 4
    assert g["ms_per_gather"] > 0 and g["backend"] == "gloo"
    # the kernel label and layout come from the engine (mdl_step_kernel_name / mdl_last_step_layout)
    assert d["roofline"]["kernel"] == "mdl::k_step<true, 1, false, 5>"
    assert d["config"]["step_layout"].startswith("wave")


def test_bench_one_gpu_launch_floor_and_config3_leg():
    """The default line carries the launch floor; `--config 3` times mdl_step_obs (step + full
    observations) with the write-bytes roofline and the CPU leg that builds the same observations."""
    d = _plain(["--steps", "40", "--warmup", "5", "--cpu-seconds", "0", "--fused-k", "0"])
    assert d["ranks_seen"] == 1 and d["launcher"] == "none" and d["launch_floor"]["ms_per_step"] > 0
    assert d["launch_floor_ms_per_step"] < d["ms_per_step"]
    d3 = _plain(["--config", "3", "--envs", "2048", "--steps", "20", "--warmup", "5", "--cpu-seconds", "0.5"])
    assert d3["config"]["obs_dims"] == {"actor_vec": 52, "critic_vec": 1301, "obs_bytes_per_env_step": 19844}
    assert d3["roofline"]["algorithmic_bytes_per_env_step"] == 19844 + 586
    assert d3["roofline"]["kernel"] == "mdl::k_step_obs<true, 5>" and d3["launch_floor"] is None
    assert d3["cpu_baseline"]["value"] > 0 and "full observations" in d3["cpu_baseline"]["sample"]
