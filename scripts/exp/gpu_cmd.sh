mkdir -p gpurun_out/r03x
timeout -k 10 120 build/slab_bw > gpurun_out/r03x/slab_bw.jsonl 2>&1; rc=$?; cat gpurun_out/r03x/slab_bw.jsonl; exit $rc
