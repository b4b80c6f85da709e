#!/bin/bash
# KP = 40 split paths: parity test, then bench A/B (CWBL_TQ4 = 1 new record path, 8 old hand-off)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "split_kp40 or c2_full or driver or ragged" > gpurun_out/pytest_tq40.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_tq40.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E  " gpurun_out/pytest_tq40.log | head -30; exit $rc; }
for m in ${MODES:-1 8}; do
  CWBL_TQ4=$m timeout -k 10 300 python bench.py --no-cpu-baseline --no-cycle --steps 5 > gpurun_out/bench_tq$m.log 2>&1 || { echo "bench $m failed"; tail -5 gpurun_out/bench_tq$m.log; exit 4; }
  echo "mode $m: $(tail -1 gpurun_out/bench_tq$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g ms/step %.2f solve %.2f' % (d['value'], d['ms_per_step'], d['detail']['ms_solve_per_step']))")"
done
