#!/bin/bash
# r4end: the per-rank shard rehearsal and a 20-step C2 bench line with the final library
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 240 python3 -u scripts/shard_rehearsal.py > gpurun_out/r4end_shard.log 2>&1 || { tail -5 gpurun_out/r4end_shard.log; exit 4; }
grep world gpurun_out/r4end_shard.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-cycle --no-detail-configs > gpurun_out/r4end_c2.log 2>&1 || { tail -5 gpurun_out/r4end_c2.log; exit 5; }
tail -1 gpurun_out/r4end_c2.log | cut -c1-700
