#!/bin/bash
# r4za: event overhead on the solve stream: kernel timing on/off x stats events timed / dependency-only
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/abenv
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "c2_full or batch_plan or pipelined" --timeout 120 --timeout-method thread > gpurun_out/r4za_tests.log 2>&1; tail -1 gpurun_out/r4za_tests.log
CWBL_LEAN_EVENTS=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "c2_full or batch_plan or pipelined" --timeout 120 --timeout-method thread > gpurun_out/r4za_tests_lean.log 2>&1; tail -1 gpurun_out/r4za_tests_lean.log
ENVS="CWBL_BENCH_KT=1 CWBL_BENCH_KT=0 CWBL_BENCH_KT=1,CWBL_LEAN_EVENTS=1 CWBL_BENCH_KT=0,CWBL_LEAN_EVENTS=1" CFG=c2 REPS=3 STEPS=10 timeout -k 10 600 bash scripts/ab_env.sh || exit 5
