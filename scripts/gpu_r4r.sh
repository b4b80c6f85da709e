#!/bin/bash
# r4r: final per-kernel profiles (kernel statistics, HBM traffic, executed FP64 work) of C2/C4/C5,
# and the per-rank shard rehearsal (rank 0's share at world 1/2/4/8)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r4q timeout -k 10 900 bash scripts/profile_r4.sh > gpurun_out/r4q_profile.log 2>&1 || { tail -5 gpurun_out/r4q_profile.log; exit 3; }
grep "^==" -A1 gpurun_out/r4q_profile.log | cut -c1-200
timeout -k 10 240 python3 -u scripts/shard_rehearsal.py > gpurun_out/r4q_shard.log 2>&1 || { tail -5 gpurun_out/r4q_shard.log; exit 4; }
cat gpurun_out/r4q_shard.log
