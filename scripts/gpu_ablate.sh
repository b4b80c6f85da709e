#!/bin/bash
cd "$GRAFT_REPO_ROOT"
for sw in 30 0 1 2; do
  CWBL_DEBUG_MAX_SWEEPS=$sw timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$sw.log 2>&1 || exit 4
  echo "sweeps<=$sw: $(tail -1 gpurun_out/ab_$sw.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['detail']['ms_solve_per_step'],1), 'ms solve', round(d['detail']['mean_sweeps'],2), 'mean sweeps')")"
done
