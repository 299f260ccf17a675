"""Benchmark of the marl-delivery hot path on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): map1.txt, 5 agents, 4096 batched envs per
GPU, step + reward kernel: one ``mdl_step`` per env-step = movement with
shared-cell priority, package pickup/drop/spawn, fp64 env reward, float32
MAPPO shaped reward with the never-cleared tracker, tracker update and
reset-on-done.  P=50 packages, T=500 (MAPPO/trainer.py:41-47), env seeds
42 + global env index, actions uint8 uniform in [0, 15) pre-generated on the
device (Philox, seed 0) -- inputs resident in HBM before the timed region.

A "step" = one ``mdl_step`` over all local envs.  The K timed steps are
replayed from hipGraphs of G steps each (launch-bound loop; the same kernels
as eager launches).  value = agent-steps/s over all ranks (weak scaling: 4096
envs per GPU, no collective on the step path; ``--total-envs N`` splits N envs
over the ranks instead: strong scaling, SURVEY.md 8(e), global env ids and seeds
unchanged).  ``--config 3`` times the trainer's per-step cost instead: one
``mdl_step_obs`` (step + the full 6ch/4ch maps and vectors of the new state) over
16,384 envs per GPU.

Multi-GPU: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) the
process is one rank.  A plain ``python bench.py --gpus N`` (N > 1, no WORLD_SIZE)
starts ``python -m torch.distributed.run --nproc-per-node N bench.py ...`` as a
child process -- the parent makes no GPU call -- forwards rank 0's JSON line and
exits with the child's return code.

Extra fields: the ranks the process group saw and their devices, eager
(un-captured) throughput, the launch floor (an empty kernel in the step's launch
shape replayed the same way), the roofline record of the step kernel (HIP-event
timed), and the CPU baseline (the oracle's C restatement on a bounded sample of
the same workload, timed on rank 0 after the timed region).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "marl-delivery_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

STEP_BYTES_PER_ENV = lambda A, P: 9 * A + 10 * P + 41  # SURVEY.md §8(d) / A.7  # noqa: E731
HBM_PEAK_GBS = 8000.0                                     # MI355X_MICROARCH.md: 8.0 TB/s spec

# config 3's observation dims (MAPPO/trainer.py:250-280: generate_vector_features(..., A-1, 5),
# convert_global_state with the defaults MR = MPs = 100)
OBS3 = dict(max_other_robots=4, max_packages_obs=5, max_robots_state=100, max_packages_state=100)
OBS5 = dict(max_other_robots=15, max_packages_obs=20, max_robots_state=16, max_packages_state=100)

# BASELINE.json configs run by --config (configs[1] is the headline; 4 and 5 are the
# fixed-size multi-GPU batches, split over the ranks: strong scaling of one global batch)
CONFIGS = {
    "2": dict(maps=["map1.txt"], agents=5, packages=50, T=500, total=0, envs=4096,
              metric="agent-steps/sec (whole node), map1 5-agent 4096 envs, 1/2/4/8 MI355X"),
    "3": dict(maps=["map1.txt"], agents=5, packages=50, T=500, total=0, envs=16384,
              metric="agent-steps/sec (whole node), map1 5-agent 16384 envs per GPU, step + full 6ch/4ch "
                     "spatial + vector observations, 1/2/4/8 MI355X"),
    "4": dict(maps=[f"map{i}.txt" for i in range(1, 6)], agents=5, packages=50, T=500, total=65536, envs=4096,
              metric="agent-steps/sec (whole node), map1-map5 mixed 5-agent 65536 envs, 1/2/4/8 MI355X"),
    "5": dict(maps=["synthetic64.txt"], agents=16, packages=100, T=500, total=131072, envs=4096,
              metric="agent-steps/sec (whole node), synthetic 64x64 16-agent 131072 envs, 1/2/4/8 MI355X"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (= ranks, one process each); N > 1 without torch.distributed.run starts it as a child")
    ap.add_argument("--config", default="2", choices=sorted(CONFIGS),
                    help="BASELINE.json config: 2 = map1 4096 envs per GPU (the headline), 3 = map1 16384 envs per "
                         "GPU with full observations every step, 4 = 65536 mixed-map envs over all ranks, "
                         "5 = 131072 synthetic 64x64 16-agent envs over all ranks")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default: 4096; config 3: 16384)")
    ap.add_argument("--total-envs", type=int, default=0,
                    help="strong scaling: this many envs in total, split over the ranks (0 = weak: --envs per GPU)")
    ap.add_argument("--map", default=None, help="configs 2 / 3 only (default map1.txt)")
    ap.add_argument("--agents", type=int, default=None)
    ap.add_argument("--packages", type=int, default=None)
    ap.add_argument("--T", type=int, default=None)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--graph-steps", type=int, default=100)
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline budget per leg (0 = skip)")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--fused-k", type=int, default=100, help="bench mode (ii): steps per fused launch (0 = skip)")
    ap.add_argument("--no-floor", action="store_true", help="skip the launch-floor leg")
    ap.add_argument("--no-graph", action="store_true", help="eager launches only (PMC profiling passes)")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="process-group backend under torchrun (gloo: rehearse N ranks on fewer GPUs)")
    ap.add_argument("--step-layout", default="auto", choices=("auto", "wave", "rows", "halves"),
                    help="mdl_step's env-to-wavefront mapping (MdlConfig.step_layout; same results): auto = four "
                         "envs per wavefront where A <= 8 and P <= 64 (>= 7,168 envs), two where A == 16 and "
                         "P <= 128 (>= 12,288 envs)")
    ap.add_argument("--host-wait", default="auto", choices=("auto", "spin", "yield", "blocking"),
                    help="how the host waits for the GPU in synchronize (hipSetDeviceFlags schedule mode)")
    ap.add_argument("--no-strong", action="store_true",
                    help="N > 1, config 2: skip the second timed region of 4,096 envs in total split over the ranks")
    ap.add_argument("--gather", action="store_true",
                    help="N > 1: after the timed regions, all-gather one step of critic vectors (the optional "
                         "rollout collation, marl_gpu.dist.gather_rollout) and report its rate")
    ap.add_argument("--graph-only", action="store_true",
                    help="skip the eager, isolated-launch and floor legs (rocprof kernel-trace pass: the trace then "
                         "holds only the warmup and the timed graph replay, so its average is the timed region's)")
    a = ap.parse_args(argv)
    c = CONFIGS[a.config]
    if a.map is not None and a.config not in ("2", "3"):
        ap.error("--map applies to configs 2 and 3 only")
    a.maps = [a.map] if a.map is not None else c["maps"]
    a.agents = c["agents"] if a.agents is None else a.agents
    a.packages = c["packages"] if a.packages is None else a.packages
    a.T = c["T"] if a.T is None else a.T
    a.envs = c["envs"] if a.envs is None else a.envs
    if c["total"] and a.total_envs == 0:
        a.total_envs = c["total"]
    a.metric = c["metric"]
    return a


# ---------------------------------------------------------------- self-launch (N > 1, plain command)
def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(n, argv, port):
    """The torch.distributed.run command that runs this bench as n ranks (one per GPU)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def forward_child(cmd, env=None):
    """Run `cmd`; its JSON result line goes to our stdout, every other line to stderr (progress
    stays visible while it runs).  Returns the child's exit code."""
    p = subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in p.stdout:
        s = line.strip()
        if s.startswith("{") and '"metric"' in s:
            sys.stdout.write(s + "\n")
            sys.stdout.flush()
        else:
            sys.stderr.write(line)
    return p.wait()


def self_launch(args, argv):
    """`python bench.py --gpus N` (N > 1) outside torchrun: N ranks as a child torchrun job.
    Nothing here touches the GPU (the children select and initialise their own devices)."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this pool (RCCL)
    env["MDL_BENCH_LAUNCHER"] = "self"
    return forward_child(launcher_cmd(args.gpus, argv, free_port()), env)


# ---------------------------------------------------------------- CPU baseline
CPU_THREAD_CAP = 16   # a one-GPU box's CPU share (the pool's limit: nproc shows the whole machine)


def host_cpu_info():
    """What the CPU leg ran on: ``nproc`` (the whole machine on a GPU box), this process's
    affinity count, the ``lscpu`` model name, and the thread cap applied."""
    def run(cmd):
        try:
            return subprocess.run(cmd, capture_output=True, text=True, timeout=10).stdout
        except (OSError, subprocess.SubprocessError):
            return ""
    nproc = run(["nproc", "--all"]).strip()
    model = ""
    for line in run(["lscpu"]).splitlines():
        if line.startswith("Model name:"):
            model = line.split(":", 1)[1].strip()
            break
    if not model:
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
        except OSError:
            model = platform.processor()
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    return {"nproc": int(nproc) if nproc.isdigit() else os.cpu_count(), "affinity_cpus": aff,
            "lscpu_model_name": model, "thread_cap": CPU_THREAD_CAP,
            "threads_used": max(1, min(CPU_THREAD_CAP, aff))}


def cpu_baseline(args, grid, seeds0, budget_s, n_threads, E, map_name, host, with_obs=False):
    """The oracle's C restatement on the same workload: the first rank's first same-map run of
    E envs, same seeds, uniform trainer-int actions, for as many steps as fit in ~budget_s of
    wall time, on `n_threads` OpenMP threads (envs split statically across threads, SURVEY.md
    §8(d) CPU leg (ii)).  with_obs (config 3): every step also builds the full observations
    of the new state (MAPPO/trainer.py:261-280)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    A = args.agents
    ob = O.OracleBatch(E, grid, A, args.packages, args.T, seed_base=int(seeds0), clear_on_reset=False)
    obs_out = None
    gen = torch.Generator().manual_seed(0)
    t_all = 0.0
    steps = 0
    while t_all < budget_s:
        ints = torch.randint(0, 15, (E, A), generator=gen, dtype=torch.uint8).numpy()
        t0 = time.perf_counter()
        ob.step(ints, auto_reset=True, consts=O.MAPPO_CONSTS, n_threads=n_threads)
        if with_obs:
            obs_out = ob.obs(args.T, OBS3["max_other_robots"], OBS3["max_packages_obs"], OBS3["max_robots_state"],
                             OBS3["max_packages_state"], out=obs_out, n_threads=n_threads)
        t_all += time.perf_counter() - t0
        steps += 1
    how = "single thread" if n_threads == 1 else f"{n_threads} OpenMP threads"
    what = "step + full observations" if with_obs else "step"
    rec = {"value": E * A * steps / t_all, "unit": "agent-steps/s", "cores": n_threads, "kind": "port",
           "sample": f"{E} envs ({map_name}) x {steps} steps ({E * A * steps} agent-steps, {t_all:.1f} s) of the "
                     f"same workload ({what}), oracle/mdl_oracle.c, {how}, host {host['lscpu_model_name']}",
           "host": host}
    rec["threads_note"] = ("single thread (one core of the host)" if n_threads == 1 else
                           f"threads = min(affinity {host['affinity_cpus']}, cap {host['thread_cap']}): the cap is a "
                           f"one-GPU box's CPU share; nproc {host['nproc']} counts the whole machine")
    return rec


# The reference's own CPU figures (MAPPO/env_vectorized.py VectorizedEnv, env.step only, 4096 map1
# envs), measured in the build container because the reference never travels to the GPU box
# (BASELINE.md §2): static numbers, labelled as measured elsewhere -- not this host.
REFERENCE_CPU = {
    "what": "reference MAPPO/env_vectorized.py VectorizedEnv(Environment, 4096) map1 A=5 P=50 T=500, env.step only, "
            "uniform random trainer-int actions, auto-reset",
    "serial_1core": 195453.0, "processes_8": 1650597.0, "unit": "agent-steps/s",
    "host": "build container: Intel Xeon, 8 cores, 1 thread/core, Python 3.10.12, NumPy 2.2.6",
    "source": "BASELINE.md section 2 (measured in the build container, NOT on this GPU host: the reference does not "
              "travel; cpu_baseline is the same workload through the C restatement timed on this host)",
}

HIP_SCHEDULE = {"auto": 0, "spin": 1, "yield": 2, "blocking": 4}   # hipDeviceSchedule* flags


def set_host_wait(mode):
    """hipSetDeviceFlags(schedule mode) on the current device: how a synchronize waits for
    the GPU (spin: the host thread polls the completion signal instead of sleeping on it).
    Returns the hipError_t (None for the HIP default, which is left untouched)."""
    if mode == "auto":
        return None
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    return int(hip.hipSetDeviceFlags(ctypes.c_uint(HIP_SCHEDULE[mode])))


def device_record(rank, local, dev_index):
    pr = torch.cuda.get_device_properties(dev_index)
    bus = "%04x:%02x:%02x" % (getattr(pr, "pci_domain_id", 0), getattr(pr, "pci_bus_id", 0),
                              getattr(pr, "pci_device_id", 0))
    return {"rank": rank, "local_rank": local, "device": dev_index, "pci": bus, "name": pr.name,
            "arch": getattr(pr, "gcnArchName", "")}


def strong_region(args, D, marl_gpu, grid, rank, world, dev, graph_region, obs_dims, G, K, dist):
    """4,096 envs in total over the ranks (the metric's workload at N GPUs, strong scaling): each
    rank steps its shard_strong share (global ids and seeds as one process would give them), timed
    like the headline region; the MAX over ranks of the wall time sets the rate."""
    A, P = args.agents, args.packages
    total = 4096
    ids, seeds = D.shard_strong(total, rank, world, args.seed)
    E = len(ids)
    env = marl_gpu.BatchedEnv(grid, E, A, P, args.T, seeds=seeds, tracker="mappo", shaping="mappo", device=dev,
                              step_layout=args.step_layout, **obs_dims)
    env.reset()
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    acts = torch.randint(0, 15, (G, E, A), generator=gen, device=dev, dtype=torch.int32).to(torch.uint8)
    out = (torch.zeros(E, dtype=torch.float64, device=dev), torch.zeros(E, dtype=torch.float32, device=dev),
           torch.zeros(E, dtype=torch.uint8, device=dev))
    wall, gpu_ms = graph_region(lambda k: env.step(acts[k % G], auto_reset=True, out=out))
    layout = env.last_step_layout()
    wall_f = 0.0
    if not args.no_floor and not args.graph_only:
        wall_f, _ = graph_region(lambda k: env.step_floor())
    mx = D.max_over_ranks([wall, wall_f], device=dev if args.backend == "nccl" else None)
    env.close()
    sizes = [len(D.shard_strong(total, r, world, 0)[0]) for r in range(world)]
    return {"total_envs": total, "envs_per_rank": sizes, "value": total * A * K / mx[0], "unit": "agent-steps/s",
            "ms_per_step": mx[0] / K * 1e3, "gpu_event_ms_per_step_rank0": gpu_ms / K,
            "launch_floor_ms_per_step": (mx[1] / K * 1e3) if wall_f else None,
            "step_layout": layout, "steps": K, "scaling": "strong",
            "note": "second timed region after the weak one: BASELINE.json's metric workload (4096 map1 envs) split "
                    "over the ranks, replayed and timed like the headline (graphs, warmup, barrier, MAX over ranks)"}


def gather_leg(args, D, env, run0, dev, dist, world, reps=20):
    """The optional RCCL rollout collation, off the timed step region: the critic
    vectors of this rank's envs for one step (convert_global_state's vector, 1301 floats per env at
    the MAPPO dims) all-gathered to every rank with marl_gpu.dist.gather_rollout."""
    _, b0, n0 = run0
    cv = env.build_obs(b0, n0, which=("critic_vec",))["critic_vec"]
    torch.cuda.synchronize()
    full = D.gather_rollout(cv)   # warm (communicator set-up)
    full = D.gather_rollout(cv)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        full = D.gather_rollout(cv)
    torch.cuda.synchronize()
    dt = D.max_over_ranks([time.perf_counter() - t0], device=dev if args.backend == "nccl" else None)[0]
    per = dt / reps
    nbytes = full.numel() * full.element_size()
    return {"tensor": f"critic_vec [{n0}, {cv.shape[1]}] float32 per rank", "bytes_per_rank": cv.numel() * 4,
            "gathered_bytes": nbytes, "ms_per_gather": per * 1e3, "gathered_GBps": nbytes / per / 1e9,
            "received_GBps_per_rank": nbytes * (world - 1) / world / per / 1e9, "reps": reps,
            "backend": dist.get_backend(),
            "note": ("RCCL all_gather_into_tensor on device tensors (xGMI)" if dist.get_backend() == "nccl" else
                     "gloo: through host memory -- rehearsal of the code path only, not an xGMI figure")}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(args, argv)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:   # one process per GPU: N GPUs need N ranks
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    dist = None
    if world > 1 or "TORCHELASTIC_RUN_ID" in os.environ:   # under torchrun: always a process group
        import torch.distributed as dist
        if args.backend == "nccl":   # RCCL: one rank per GPU
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:   # gloo (rehearsal of the multi-rank path on fewer GPUs than ranks): ranks share GPUs
            torch.cuda.set_device(local % torch.cuda.device_count())
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    host_wait_rc = set_host_wait(args.host_wait)
    ranks_seen = dist.get_world_size() if dist is not None else 1
    me = device_record(rank, local, dev.index)
    if dist is not None:
        devices = [None] * ranks_seen
        dist.all_gather_object(devices, me)
    else:
        devices = [me]

    import marl_gpu
    from marl_gpu.maps import grid_array, load_map, map_path
    grids = [grid_array(load_map(map_path(m))) for m in args.maps]
    A, P = args.agents, args.packages
    from marl_gpu import dist as D
    # global env g is seeded args.seed + g (MAPPO/env_vectorized.py:8-9); each rank's ids are contiguous
    if len(grids) > 1:        # config 4: map groups back to back, dealt to ranks in contiguous blocks
        ids, seeds, env_map, runs = D.shard_mixed(args.total_envs, len(grids), rank, world, args.seed)
        E_all = args.total_envs
    elif args.total_envs > 0:   # strong scaling: the ranks split one batch (lower ranks take the remainder)
        ids, seeds = D.shard_strong(args.total_envs, rank, world, args.seed)
        env_map, runs, E_all = None, [(0, 0, len(ids))], args.total_envs
    else:
        ids, seeds = D.shard(args.envs, rank, args.seed)
        env_map, runs, E_all = None, [(0, 0, len(ids))], args.envs * world
    E = len(ids)
    if E == 0:
        raise SystemExit(f"bench.py: rank {rank} has no envs (--total-envs {args.total_envs} < {world} ranks)")
    obs_cfg = args.config == "3"
    obs_dims = OBS5 if args.config == "5" else OBS3
    env = marl_gpu.BatchedEnv(grids if len(grids) > 1 else grids[0], E, A, P, args.T, seeds=seeds, env_map=env_map,
                              tracker="mappo", shaping="mappo", device=dev, step_layout=args.step_layout, **obs_dims)
    env.reset()

    G = max(1, min(args.graph_steps, args.steps))
    n_graph = (args.steps + G - 1) // G
    K = n_graph * G
    gen = torch.Generator(device=dev).manual_seed(0 + rank)
    acts = torch.randint(0, 15, (G, E, A), generator=gen, device=dev, dtype=torch.int32).to(torch.uint8)
    r = torch.zeros(E, dtype=torch.float64, device=dev)
    sh = torch.zeros(E, dtype=torch.float32, device=dev)
    dn = torch.zeros(E, dtype=torch.uint8, device=dev)
    obs_bufs = env.obs_buffers(E) if obs_cfg else None

    if obs_cfg:
        def one(k):   # the trainer's per-step cost: step + the observations of the new state
            env.step_obs(acts[k % G], auto_reset=True, out=(r, sh, dn), obs_out=obs_bufs)
    else:
        def one(k):
            env.step(acts[k % G], auto_reset=True, out=(r, sh, dn))

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def stop_clock(t_start):
        """End of a timed region: this rank's GPU work drained, then its clock read, then
        the barrier -- the collective's own latency stays outside the measured time (the
        start is aligned by the opening barrier; the MAX over ranks below covers skew)."""
        torch.cuda.synchronize()
        dt = time.perf_counter() - t_start
        if dist is not None:
            dist.barrier()
        return dt

    side = torch.cuda.Stream(device=dev)

    def graph_region(fn):
        """K calls of fn(k): captured as a G-call hipGraph (torch's stream capture covers the
        ctypes launches), replayed once untimed (the first launch of a fresh graph uploads it),
        then W warmup calls as one replay of a W-call graph (launched the way the timed calls
        are, right before the timed region), then barrier + the timed n_graph replays.
        Returns (max-over-ranks is applied by the caller) wall seconds and HIP-event ms."""
        side.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            fn(0)  # prime on the side stream
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=side):
                for k in range(G):
                    fn(k)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        if args.warmup > 0:
            wg = torch.cuda.CUDAGraph()
            with torch.cuda.stream(side):
                with torch.cuda.graph(wg, stream=side):
                    for k in range(args.warmup):
                        fn(k)
            torch.cuda.synchronize()
            wg.replay()
            torch.cuda.synchronize()
            del wg
        barrier()
        # the opening HIP event is enqueued on the idle stream before the clock starts: it marks the
        # GPU-side start of the region and is not part of the K steps' work
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        for _ in range(n_graph):
            g.replay()
        e1.record()
        w = stop_clock(t0)
        return w, e0.elapsed_time(e1)

    # ---- timed region: K steps replayed from graphs ----
    if not args.no_graph:
        wall, gpu_ms = graph_region(one)
    else:
        for k in range(args.warmup):
            one(k)
        barrier()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        t0 = time.perf_counter()
        for k in range(K):
            one(k)
        ev1.record()
        wall = stop_clock(t0)
        gpu_ms = ev0.elapsed_time(ev1)

    # the layout of the launches just timed, as the engine recorded it (step_obs: its fused wave kernel)
    layout = "wave" if obs_cfg else env.last_step_layout()

    # ---- eager throughput (same kernels, one ctypes launch per step) ----
    wall_eager = None
    if not args.graph_only:
        barrier()
        t1 = time.perf_counter()
        for k in range(K):
            one(k)
        wall_eager = stop_clock(t1)

    # ---- launch floor: an empty kernel in mdl_step's launch shape (grid, workgroup, LDS,
    # kernel-argument layout), replayed exactly as the timed steps are ----
    wall_floor = gpu_ms_floor = None
    if not obs_cfg and not args.no_graph and not args.graph_only and not args.no_floor:
        wall_floor, gpu_ms_floor = graph_region(lambda k: env.step_floor())

    # ---- bench mode: fused_k steps per launch, each env's
    # state in registers between steps; same action stream; not the API path ----
    wall_f, nf, Kf = None, 0, (0 if obs_cfg else args.fused_k)
    if Kf > 0:
        facts = acts.repeat((Kf + G - 1) // G, 1, 1)[:Kf].contiguous()
        fr = torch.empty((Kf, E), dtype=torch.float64, device=dev)
        fsh = torch.empty((Kf, E), dtype=torch.float32, device=dev)
        fdn = torch.empty((Kf, E), dtype=torch.uint8, device=dev)
        env.step_fused(facts, out=(fr, fsh, fdn))  # warm
        nf = max(1, K // Kf)
        barrier()
        t2 = time.perf_counter()
        for _ in range(nf):
            env.step_fused(facts, out=(fr, fsh, fdn))
        wall_f = stop_clock(t2)

    # ---- per-launch kernel duration: HIP events on the launch stream around the
    # timed region (back-to-back launches, so this includes the ~1 us dispatch
    # gap between kernels and is an upper bound on the rocprof kernel time);
    # plus an isolated per-launch event pair for reference ----
    kdur_us = gpu_ms / K * 1e3
    kdur_iso_us = None
    if not args.graph_only:
        nk = min(K, 200)
        starts = [torch.cuda.Event(enable_timing=True) for _ in range(nk)]
        ends = [torch.cuda.Event(enable_timing=True) for _ in range(nk)]
        for k in range(nk):
            starts[k].record()
            one(k)
            ends[k].record()
        torch.cuda.synchronize()
        kdur_iso_us = float(np.mean([a.elapsed_time(b) for a, b in zip(starts, ends)]) * 1e3)

    if dist is not None:
        t = torch.tensor([wall, wall_eager or 0.0, wall_f or 0.0, wall_floor or 0.0], dtype=torch.float64,
                         device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t[0])
        wall_eager = float(t[1]) if wall_eager is not None else None
        wall_f = float(t[2]) if wall_f is not None else None
        wall_floor = float(t[3]) if wall_floor is not None else None

    # ---- N > 1, config 2: a second timed region on the metric's own workload -- 4,096 envs in
    # TOTAL split over the ranks (strong scaling; shard_strong, seeds 42 + global id)
    strong = None
    if dist is not None and world > 1 and args.config == "2" and args.total_envs == 0 and not args.no_strong:
        strong = strong_region(args, D, marl_gpu, grids[0], rank, world, dev, graph_region, obs_dims, G, K, dist)

    # ---- optional rollout collation (N > 1): one step of critic vectors all-gathered over the ranks
    gather = None
    if args.gather and dist is not None and world > 1:
        gather = gather_leg(args, D, env, runs[0], dev, dist, world)

    total_agent_steps = E_all * A * K
    value = total_agent_steps / wall
    if rank == 0:
        H0, W0 = grids[runs[0][0]].shape
        obs_bytes_env = 4 * (A * 6 * H0 * W0 + A * env.actor_vec_dim + 4 * H0 * W0 + env.critic_vec_dim)
        # algorithmic bytes per launch: the step's SoA traffic; config 3 adds the
        # observation bytes it writes (the fused launch builds them from the step's registers, so
        # the 474 B per env of state that SURVEY §8(d) counts for a separate builder's reload are
        # not moved and not counted)
        per_env = STEP_BYTES_PER_ENV(A, P) + (obs_bytes_env if obs_cfg else 0)
        per_launch_bytes = per_env * E
        achieved = per_launch_bytes / (kdur_us * 1e-6) / 1e9
        # the kernel the engine launched (its own record and symbol: no Python mirror of its rules)
        kname = env.step_kernel_name(layout, with_obs=obs_cfg) + (" (mixed maps)" if len(grids) > 1 else "")
        traffic, traffic_rec = None, None
        if os.path.exists(args.traffic_json):
            try:
                tj = json.load(open(args.traffic_json))
                want = {"envs": E, "agents": A, "packages": P, "maps": args.maps}
                for rec in tj.get("records", []):
                    # the PMC pass of the kernel timed here: same workload, same kernel (name prefix)
                    if rec.get("config") == want and bool(rec.get("obs")) == obs_cfg and \
                            kname.startswith(rec.get("kernel", "?")):
                        traffic, traffic_rec = rec.get("hbm_bytes_per_launch"), rec
            except (OSError, ValueError):
                traffic = None
        cpu = cpu1 = None
        if args.cpu_seconds > 0:   # after every rank's timed region (the others wait in the closing barrier)
            host = host_cpu_info()
            nt = host["threads_used"]
            m0, b0, n0 = runs[0]
            Ec = min(n0, 4096)   # the first same-map run, at most 4096 envs (a bounded sample)
            cpu = cpu_baseline(args, grids[m0], seeds[b0], args.cpu_seconds, nt, Ec, args.maps[m0], host, obs_cfg)
            cpu1 = cpu if nt == 1 else cpu_baseline(args, grids[m0], seeds[b0], args.cpu_seconds, 1, Ec,
                                                     args.maps[m0], host, obs_cfg)
        ms_step = wall / K * 1e3
        floor = None
        if wall_floor is not None:
            floor = {"kernel": "mdl::k_step_floor (empty; mdl_step's grid, workgroup size, LDS request and "
                               "kernel-argument layout)",
                     "ms_per_step": wall_floor / K * 1e3, "gpu_event_us_per_step": gpu_ms_floor / K * 1e3,
                     "note": "replayed like the timed steps (G-node graphs, same warmup, same K); over_floor_us = "
                             "the step's wall time per step minus this floor's: the step kernel's own cost"}
        what = ("mdl_step_obs (step + MAPPO shaped reward + tracker + auto-reset, then the 6ch actor maps, "
                f"{env.actor_vec_dim}-dim actor vectors, 4ch critic map and {env.critic_vec_dim}-dim critic vector "
                "of the new state)") if obs_cfg else \
            "mdl_step (move+packages+env reward+MAPPO shaped reward+tracker+auto-reset)"
        out = {
            "metric": args.metric,
            "value": value,
            "unit": "agent-steps/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,
            "devices": devices,
            "distinct_devices": len({d["pci"] for d in devices}),
            "launcher": os.environ.get("MDL_BENCH_LAUNCHER", "torch.distributed.run" if dist is not None else "none"),
            "process_group_backend": None if dist is None else dist.get_backend(),
            "steps": K,
            "warmup": args.warmup,
            "graph_upload_replay_steps": 0 if args.no_graph else G,
            "graph_steps": 0 if args.no_graph else G,
            "host_wait": args.host_wait if host_wait_rc in (None, 0) else f"{args.host_wait} (hipError {host_wait_rc})",
            "ms_per_step": ms_step,
            "launch_floor_ms_per_step": None if floor is None else floor["ms_per_step"],
            "over_floor_us": None if floor is None else (ms_step - floor["ms_per_step"]) * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if args.total_envs > 0 else "weak",
            "vs_baseline": None,
            "dtype": "int32+fp64" + (" (state, rewards) + f32 (observations)" if obs_cfg else ""),
            "data": "synthetic: uniform random trainer-int actions (Philox, on device), env seeds 42+global index",
            "config": {"workload": f"BASELINE config {args.config}: {'+'.join(args.maps)} A={A} P={P} T={args.T} "
                                   f"{E} envs/GPU, {what}, "
                                   + ("eager launches" if args.no_graph else "hipGraph replay"),
                       "envs_per_gpu": E, "total_envs": E_all, "agents": A, "packages": P, "max_time_steps": args.T,
                       "maps": args.maps, "map_runs_rank0": [[args.maps[m], b, n] for m, b, n in runs],
                       "obs_dims": ({"actor_vec": env.actor_vec_dim, "critic_vec": env.critic_vec_dim,
                                     "obs_bytes_per_env_step": obs_bytes_env} if obs_cfg else None),
                       "parallelism": f"env-shard x{world}",
                       "step_layout": {"rows": "rows (4 envs per wavefront)", "halves": "halves (2 envs per wavefront)"}
                                      .get(layout, "wave (1 env per wavefront)"),
                       "step_layout_source": "engine (mdl_last_step_layout of the timed launches)"},
            "gpu_event_ms_per_step": gpu_ms / K,
            "eager": None if wall_eager is None else {"value": total_agent_steps / wall_eager,
                                                       "ms_per_step": wall_eager / K * 1e3},
            "launch_floor": floor,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_over_algorithmic": None if traffic is None else traffic / per_launch_bytes,
                         "traffic_source": None if traffic_rec is None else traffic_rec.get("source"),
                         "kernel": kname, "kernel_us": kdur_us,
                         "kernel_us_isolated_event_pair": kdur_iso_us,
                         "algorithmic_bytes_per_env_step": per_env,
                         "algorithmic_bytes_per_launch": per_launch_bytes},
            "fused_bench_mode": None if wall_f is None else {
                "k_steps_per_launch": Kf, "launches": nf, "value": E_all * A * Kf * nf / wall_f,
                "ms_per_step": wall_f / (Kf * nf) * 1e3,
                "note": "SURVEY.md 8(d)(ii) bench mode: mdl_step_fused, K steps per launch on pre-generated device "
                        "actions (bit-exact with K mdl_step calls); not the API path, not the headline value"},
            "cpu_baseline": cpu,
            "cpu_baseline_1thread": cpu1,
            "reference_cpu": REFERENCE_CPU,
            "strong_4096": strong,
            "rollout_gather": gather,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    env.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
