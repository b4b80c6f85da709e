#!/bin/bash
# A/B of the C2 solve kernels under rocprofv3 kernel statistics: library $LIBS (new in-tree,
# scratch/old) x CWBL_DEBUG_TQ_STOP in $STOPS
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for lib in ${LIBS:-new old}; do
  if [ $lib = old ]; then export CWBL_LIBRARY=$PWD/scratch/old/libcwbl.so; else unset CWBL_LIBRARY; fi
  for st in ${STOPS:-1 0}; do
    d=gpurun_out/ab_${lib}_$st
    CWBL_DEBUG_TQ_STOP=$st timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o kt --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-cycle ${BENCH_ARGS} > $d.log 2>&1 || { echo "$lib stop=$st failed"; tail -3 $d.log; exit 1; }
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    echo "$lib stop=$st"; python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if float(r['TotalDurationNs']) > 1e6: print('  %-45s calls %4s avg %.3f ms total %.1f ms' % (r['Name'].split('(')[0][:45], r['Calls'], float(r['AverageNs'])/1e6, float(r['TotalDurationNs'])/1e6))"
  done
done
