#!/bin/bash
# r4s: the next batch's search beside this batch's solve instead of its assembly (CWBL_SEARCH_AFTER_ASM=1)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/abenv
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "c2_full or batch_plan" --timeout 120 --timeout-method thread > gpurun_out/r4s_tests.log 2>&1; tail -2 gpurun_out/r4s_tests.log
ENVS="CWBL_SEARCH_AFTER_ASM=0 CWBL_SEARCH_AFTER_ASM=1" CFG=c2 REPS=3 STEPS=6 timeout -k 10 400 bash scripts/ab_env.sh || exit 5
mkdir -p gpurun_out/abenv_s2 && mv gpurun_out/abenv/*.log gpurun_out/abenv_s2/
ENVS="CWBL_SEARCH_AFTER_ASM=0 CWBL_SEARCH_AFTER_ASM=1" CFG=c5 REPS=2 STEPS=2 timeout -k 10 400 bash scripts/ab_env.sh || exit 6
