#!/bin/bash
# r4b: host probe, the multi-rank GPU tests (incl. C3 world 8), bench N=1 (new roofline and
# cycle with transposes), bench --gpus 2 over gloo on one GPU
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4b; mkdir -p $O
{ nproc; python3 -c "import os;print(len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>&1; lscpu | grep -E "Model name|Thread|Core|Socket"; } > $O/host.txt 2>&1
timeout -k 10 500 python -u -m pytest tests/test_gpu_multi_rank.py tests/test_gpu_parity.py -k "multi_rank or ranks or pipelined" -x -v --timeout 300 --timeout-method thread > $O/multi.log 2>&1 || { tail -30 $O/multi.log; exit 3; }
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench1.log 2>&1 || { tail -20 $O/bench1.log; exit 4; }
CWBL_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --no-detail-configs > $O/bench2.log 2>&1 || { tail -20 $O/bench2.log; exit 5; }
tail -3 $O/multi.log; cat $O/host.txt
