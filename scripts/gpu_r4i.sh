#!/bin/bash
# r4i: batch-size A/B on C2 with the one-stream record path
cd "$GRAFT_REPO_ROOT"
ENVS="CWBL_MAX_BATCH=160000 CWBL_MAX_BATCH=240000 CWBL_MAX_BATCH=320000 CWBL_TQ40_STREAMS=1" CFG=c2 REPS=2 STEPS=8 timeout -k 10 500 bash scripts/ab_env.sh 2>&1 | tee gpurun_out/r4i_batch.txt
ENVS="CWBL_BIN_DIV=4 CWBL_BIN_DIV=5 CWBL_BIN_DIV=6" CFG=c5 REPS=2 STEPS=2 timeout -k 10 500 bash scripts/ab_env.sh 2>&1 | tee gpurun_out/r4i_bindiv_c5.txt
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-detail-configs --no-cycle > gpurun_out/r4i_bench.log 2>&1
grep -o '"roofline": {[^}]*' gpurun_out/r4i_bench.log | cut -c1-300
# the full N>1 bench path (all legs: transposes, cycle, C4, C5) as 4 gloo ranks on one GPU
CWBL_DIST_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 4 --steps 2 --warmup 1 > gpurun_out/r4i_gloo4.log 2>&1; echo "gloo4 rc=$?"
tail -c 400 gpurun_out/r4i_gloo4.log
