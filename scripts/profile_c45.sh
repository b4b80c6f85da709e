#!/bin/bash
# Kernel statistics of the C4 (k = 128) and C5 (dense radar) bench configurations, one step
# each after a warmup -> gpurun_out/prof_${TAG}_c4, _c5 (kt_kernel_stats.csv)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for C in c4 c5; do
  OUT=gpurun_out/prof_${TAG:-r3}_$C
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --config $C --steps 1 --warmup 1 --no-cpu-baseline --no-cycle --no-detail-configs > $OUT/kt_bench.log 2>&1 || { tail -5 $OUT/kt_bench.log; exit 5; }
  f=$(find $OUT/kt -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kt/
  tail -1 $OUT/kt_bench.log | cut -c1-300
done
