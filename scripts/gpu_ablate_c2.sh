#!/bin/bash
# C2 assembly-kernel ablations under rocprofv3 kernel statistics: CWBL_DEBUG_TQ_STOP=11
# (staging only), 1 (staging + MFMA assembly), 0 (full)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for st in ${STOPS:-11 1 0}; do
  CWBL_DEBUG_TQ_STOP=$st timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abl_$st -o kt --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-cycle > gpurun_out/abl_$st.log 2>&1 || { echo "stop=$st failed"; tail -3 gpurun_out/abl_$st.log; exit 1; }
  f=$(find gpurun_out/abl_$st -name "*kernel_stats.csv" | head -1)
  echo "stop=$st"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print('  %-45s calls %4s avg %.3f ms total %.1f ms' % (r['Name'].split('(')[0][-45:], r['Calls'], float(r['AverageNs'])/1e6, float(r['TotalDurationNs'])/1e6))"
done
