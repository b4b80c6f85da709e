#!/bin/bash
# bench.py's N>1 path on one GPU (two ranks on cuda:0 over gloo: RCCL refuses two ranks per
# device), then rank 0's share of the C2 grid timed alone at world 1, 2, 4, 8
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
CWBL_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cycle --no-detail-configs > gpurun_out/bench_n2_gloo.log 2>&1 || { echo "n2 failed"; tail -20 gpurun_out/bench_n2_gloo.log; exit 3; }
grep '^{' gpurun_out/bench_n2_gloo.log | cut -c1-700
timeout -k 10 300 python scripts/shard_rehearsal.py 1 2 4 8 2>&1 | grep world
