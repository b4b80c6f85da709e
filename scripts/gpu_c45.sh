#!/bin/bash
# C5 and C4 bench lines
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for cfg in c5 c4; do
  timeout -k 10 400 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-cycle > gpurun_out/bench_$cfg.log 2>&1 || { echo "$cfg failed"; tail -5 gpurun_out/bench_$cfg.log; exit 2; }
  tail -1 gpurun_out/bench_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg value %.4g ms/step %.1f solve %.1f search %.1f mean_p %.0f frac %.3f' % (d['value'], d['ms_per_step'], d['detail']['ms_solve_per_step'], d['detail']['ms_search_per_step'], d['config']['mean_p'], d['roofline']['frac']))"
done
