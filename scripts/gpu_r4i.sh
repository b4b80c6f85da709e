#!/bin/bash
# r4i: batch-size A/B on C2 with the one-stream record path
cd "$GRAFT_REPO_ROOT"
ENVS="CWBL_MAX_BATCH=160000 CWBL_MAX_BATCH=240000 CWBL_MAX_BATCH=320000 CWBL_TQ40_STREAMS=1" CFG=c2 REPS=2 STEPS=8 timeout -k 10 500 bash scripts/ab_env.sh 2>&1 | tee gpurun_out/r4i_batch.txt
