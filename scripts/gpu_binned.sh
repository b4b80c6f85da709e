#!/bin/bash
# binned analysis search: parity tests, then C2 (and C5 with C5=1) with the bins and with
# the k-d tree search only
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "${TESTK:-binned or driver or synthetic or dense or batch_plan or c2_full}" > gpurun_out/pytest_binned.log 2>&1
rc=$?; tail -22 gpurun_out/pytest_binned.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_binned.log | head -20; exit $rc; }
for cfg in c2 ${C5:+c5}; do
  for mode in bins tree; do
    CWBL_SEARCH=$mode timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-cycle > gpurun_out/bench_${cfg}_$mode.log 2>&1 || { echo "bench $cfg $mode failed"; tail -5 gpurun_out/bench_${cfg}_$mode.log; exit 4; }
    echo -n "$cfg $mode: "; tail -1 gpurun_out/bench_${cfg}_$mode.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g ms/step %.2f solve %.1f search %.2f' % (d['value'], d['ms_per_step'], d['detail']['ms_solve_per_step'], d['detail']['ms_search_per_step']))"
  done
done
