#!/bin/bash
# Kernel statistics with the searches overlapped (default) and serialized (CWBL_DEBUG_SERIAL=1)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for ser in 0 1; do
  d=gpurun_out/serial_$ser
  CWBL_DEBUG_SERIAL=$ser timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o kt --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cycle ${BENCH_ARGS} > $d.log 2>&1 || { echo "serial=$ser failed"; tail -3 $d.log; exit 1; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  echo "serial=$ser $(tail -1 $d.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("ms/step %.2f" % d["ms_per_step"])')"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if float(r['TotalDurationNs']) > 1e6: print('  %-45s calls %4s avg %.3f ms total %.1f ms' % (r['Name'].split('(')[0][:45], r['Calls'], float(r['AverageNs'])/1e6, float(r['TotalDurationNs'])/1e6))"
done
