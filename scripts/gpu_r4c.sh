#!/bin/bash
# r4c: bench N=1 (all legs but the CPU baseline), record-path stream A/B, gloo N=2
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench1.log 2>&1 || { tail -20 $O/bench1.log; exit 4; }
for r in 1 2; do for S in 0 1; do
  CWBL_TQ40_STREAMS=$S timeout -k 10 120 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-cycle --no-detail-configs --no-transposes > $O/ab_${S}_$r.log 2>&1 || exit 5
  echo "streams=$S run $r $(grep -o '"value": [0-9.]*' $O/ab_${S}_$r.log | head -1)"
done; done
CWBL_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --no-detail-configs > $O/bench2.log 2>&1 || { tail -20 $O/bench2.log; exit 6; }
