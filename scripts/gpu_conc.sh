#!/bin/bash
# record path with the solves on their own stream: parity tests, then bench A/B
# (CWBL_TQ40_STREAMS = 1 / 0) twice in one run
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "split_kp40 or ragged or batch_plan or c2_full or driver" > gpurun_out/pytest_conc.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_conc.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E  " gpurun_out/pytest_conc.log | head -20; exit $rc; }
for i in 1 2 3 4; do for m in 1 0; do
  CWBL_TQ40_STREAMS=$m timeout -k 10 300 python bench.py --no-cpu-baseline --no-cycle --steps 10 > gpurun_out/conc_$m.log 2>&1 || { tail -5 gpurun_out/conc_$m.log; exit 4; }
  echo "streams $m: $(tail -1 gpurun_out/conc_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g ms/step %.2f solve %.2f frac %.3f' % (d['value'], d['ms_per_step'], d['detail']['ms_solve_per_step'], d['roofline']['frac']))")"
done; done
