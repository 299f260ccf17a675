#!/bin/bash
# Bench checks on one GPU box: the driver's command (20 steps), the torchrun path with
# one rank (RCCL process group, the N>1 code path), and a long run.  Results under
# gpurun_out/$TAG/.
set -u
OUT=gpurun_out/${TAG:-benchcheck}
mkdir -p $OUT
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/bench_torchrun1.json \
    2> $OUT/bench_torchrun1.err || exit $?
timeout -k 10 300 python bench.py --cpu-seconds 0 --steps 2000 --warmup 100 > $OUT/bench_long.json 2> $OUT/bench_long.err || exit $?
python3 - <<EOF
import json
for f in ("bench_driver", "bench_torchrun1", "bench_long"):
    d = json.loads(open("$OUT/%s.json" % f).read().strip().splitlines()[-1])
    print(f, "value %.3e" % d["value"], "wall us/step %.3f" % (d["ms_per_step"] * 1e3),
          "event us/step %.3f" % (d["gpu_event_ms_per_step"] * 1e3), "frac %.4f" % d["roofline"]["frac"],
          "eager %.3e" % d["eager"]["value"])
EOF
