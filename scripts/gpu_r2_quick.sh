#!/bin/bash
# GPU suite (stop at first failure) + one default bench line
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^FAILED|^E  " gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g ms/step %.2f solve %.2f search %.2f frac %.3f' % (d['value'], d['ms_per_step'], d['detail']['ms_solve_per_step'], d['detail']['ms_search_per_step'], d['roofline']['frac']))"
