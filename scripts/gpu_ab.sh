#!/bin/bash
# A/B of prebuilt libraries (_ab/*.so, untracked) on the C2 bench: one line per library.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for lib in ${LIBS:-_ab/*.so}; do
  CWBL_LIBRARY=$PWD/$lib timeout -k 10 400 python bench.py --steps ${STEPS:-3} --warmup 1 \
    --no-cpu-baseline > gpurun_out/ab_$(basename $lib .so).log 2>&1 || { echo "fail $lib"; exit 4; }
  tail -1 gpurun_out/ab_$(basename $lib .so).log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['value']/1e6,3), 'M/s solve', round(d['detail']['ms_solve_per_step'],2), 'search', round(d['detail']['ms_search_per_step'],2))"
done
