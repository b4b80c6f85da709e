#!/bin/bash
# rocprofv3 kernel statistics of a short bench run (env passes through: CWBL_*)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/kstats_${TAG:-x}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o kt --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cycle > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 5; }
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-60s calls %4s avg %9.3f ms  pct %6s" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])/1e6, r["Percentage"]))
PY
