#!/bin/bash
# r4last: the round's last check on the final tree: the GPU suite, smoke(), the default bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4last_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4last_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4last_smoke.log 2>&1 || { tail -5 gpurun_out/r4last_smoke.log; exit 3; }
tail -1 gpurun_out/r4last_smoke.log
timeout -k 10 500 python3 bench.py > gpurun_out/r4last_bench.log 2>&1 || { tail -5 gpurun_out/r4last_bench.log; exit 4; }
tail -1 gpurun_out/r4last_bench.log | cut -c1-400
