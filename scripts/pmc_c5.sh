#!/bin/bash
# C5 gather locality: HBM bytes (FETCH_SIZE) and L2 hit rate (TCC_HIT/MISS) per kernel, one
# step, serial streams -> gpurun_out/pmc_c5/
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_c5${TAG:+_$TAG}
mkdir -p $OUT
B="python3 bench.py --config ${CFG:-c5} --steps 1 --warmup 0 --no-cpu-baseline --no-cycle --no-detail-configs"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "assemble|tq40|search" -d $OUT/f -o f --output-format csv -- $B > $OUT/f.log 2>&1 || { tail -3 $OUT/f.log; exit 5; }
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "assemble|tq40|search" -d $OUT/h -o h --output-format csv -- $B > $OUT/h.log 2>&1 || { tail -3 $OUT/h.log; exit 6; }
python3 - $OUT <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    hit = m.get("TCC_HIT_sum", 0); miss = m.get("TCC_MISS_sum", 0)
    print(k[:50], "FETCH GB/launch x2 = %.2f" % (2 * m.get("FETCH_SIZE", 0) * 1024 / 1e9),
          "L2 hit %.3f" % (hit / max(hit + miss, 1)), "launches", len(d.get("FETCH_SIZE", [])))
PY
