#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi_rank.py -x -v -k bench_two_ranks --timeout 900 --timeout-method thread > gpurun_out/r4t_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4t_tests.log; exit $rc
