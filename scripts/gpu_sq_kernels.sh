#!/bin/bash
# SQ counter passes (issue / wait / MFMA breakdown) for the kernels matching $KRE, one bench step
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/sq_${TAG:-x}
mkdir -p $OUT
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM" ; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $P --kernel-include-regex "${KRE:-solve}" -d $OUT/p$i -o p$i --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-cycle ${BENCH_ARGS} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print("  %-28s %14.4g (avg of %d)" % (c, sum(v) / len(v), len(v)))
PY
