#!/bin/bash
# k = 128 (configs[3]): large-ensemble parity tests, then the C4 bench with the timing
# ablations of solve_tq_big_kernel (CWBL_DEBUG_TQ_STOP=1/2/3: stop after assembly /
# tridiagonalisation / quadrature)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu ${PYX--x} -q --timeout 300 --timeout-method thread -k "${TESTK:-128 or 80 or big or k128}" > gpurun_out/pytest_big.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_big.log
tail -6 gpurun_out/pytest_big.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then echo "stop: pytest rc=$rc"; exit $rc; fi
for st in ${STOPS:-0 1 2 3}; do
  CWBL_DEBUG_TQ_STOP=$st timeout -k 10 300 python bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline --no-cycle > gpurun_out/bench_big.log 2>&1 || { echo "bench stop=$st failed"; tail -5 gpurun_out/bench_big.log; exit 4; }
  echo -n "stop=$st: "; tail -1 gpurun_out/bench_big.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g ms/step %.1f solve %.1f search %.1f TF %.2f' % (d['value'], d['ms_per_step'], d['detail']['ms_solve_per_step'], d['detail']['ms_search_per_step'], d['roofline']['achieved']))"
done
