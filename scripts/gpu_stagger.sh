#!/bin/bash
cd "$GRAFT_REPO_ROOT"
for S in ${STAG:-0 20000 40000}; do
  CWBL_DEBUG_STAGGER=$S timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/stag$S.log 2>&1 || exit 4
  echo "stagger=$S $(tail -1 gpurun_out/stag$S.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['detail']['ms_solve_per_step'])")"
done
