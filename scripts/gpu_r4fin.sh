#!/bin/bash
# r4fin: final checks of the round: the GPU suite, smoke(), and the default bench under rocprofv3 kernel statistics
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4fin_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4fin_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4fin_smoke.log 2>&1 || { tail -5 gpurun_out/r4fin_smoke.log; exit 3; }
tail -1 gpurun_out/r4fin_smoke.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4fin_bench -o kt --output-format csv -- python3 bench.py > gpurun_out/r4fin_bench.log 2>&1 || { tail -5 gpurun_out/r4fin_bench.log; exit 4; }
f=$(find gpurun_out/prof_r4fin_bench -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r4fin_bench_kernel_stats.csv
grep -E "assemble_record|solve_tq40|search_binned" gpurun_out/r4fin_bench_kernel_stats.csv | cut -d, -f1-8
tail -1 gpurun_out/r4fin_bench.log | cut -c1-600
