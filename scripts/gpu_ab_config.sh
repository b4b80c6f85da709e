#!/bin/bash
# Interleaved A/B of prebuilt libraries (_ab/*.so, untracked) on one bench configuration
# (CONFIG, default c5): one line per library run.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
CONFIG=${CONFIG:-c5}
i=0
for lib in ${LIBS:-_ab/*.so}; do
  i=$((i + 1))
  log=gpurun_out/ab_${CONFIG}_${i}_$(basename $lib .so).log
  CWBL_LIBRARY=$PWD/$lib timeout -k 10 300 python bench.py --config $CONFIG --steps ${STEPS:-1} \
    --warmup 1 --no-cpu-baseline --no-cycle > $log 2>&1 || { echo "fail $lib"; tail -5 $log; exit 4; }
  tail -1 $log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$CONFIG $lib', round(d['value']/1e6,3), 'M/s ms/step', round(d['ms_per_step'],1), 'solve', round(d['detail']['ms_solve_per_step'],1), 'search', round(d['detail']['ms_search_per_step'],1))"
done
