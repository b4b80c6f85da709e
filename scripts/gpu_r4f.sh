#!/bin/bash
# r4f: the binned-search tests alone (a hang in r4e), verbose, short limits
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "binned_search_equals_tree_search or driver_variable_matches" -x -v --timeout 60 --timeout-method thread 2>&1 | tee $O/tests.log
