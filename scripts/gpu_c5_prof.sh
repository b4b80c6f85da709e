#!/bin/bash
# C5 (dense radar) kernel statistics: overlapped and with the searches serialised
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
cd /tmp
for ser in 0 1; do
  CWBL_DEBUG_SERIAL=$ser timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5_$ser -o c5 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-cycle > $GRAFT_REPO_ROOT/gpurun_out/prof_c5_$ser.log 2>&1 || { echo "prof $ser failed"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof_c5_$ser.log; exit 5; }
  echo "serial=$ser: $(tail -1 $GRAFT_REPO_ROOT/gpurun_out/prof_c5_$ser.log | cut -c1-200)"
  f=$(find $GRAFT_REPO_ROOT/gpurun_out/prof_c5_$ser -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print('  ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3), round(float(r['TotalDurationNs'])/1e6,1))
"
done
