#!/bin/bash
# C4 (k = 128) tridiagonalisation cost per step range: CWBL_DEBUG_TQ_STOP=2 (stop after the
# tridiagonalisation) with CWBL_DEBUG_TQ_STEPS=n (only the first n Householder steps)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for s in ${STEPLIST:-1 32 64 96 0}; do
  CWBL_DEBUG_TQ_STOP=${STOP:-2} CWBL_DEBUG_TQ_STEPS=$s timeout -k 10 300 python bench.py --config ${CFG:-c4} --steps 1 --warmup 1 --no-cpu-baseline --no-cycle > gpurun_out/bench_steps.log 2>&1 || { echo "bench steps=$s failed"; tail -5 gpurun_out/bench_steps.log; exit 4; }
  echo -n "steps=$s: "; tail -1 gpurun_out/bench_steps.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step %.1f solve %.1f search %.1f' % (d['ms_per_step'], d['detail']['ms_solve_per_step'], d['detail']['ms_search_per_step']))"
done
