#!/bin/bash
# SQ counters of the C2 solve pair (assemble_record_kernel, solve_tq40_kernel), one bench
# step, two rocprofv3 --pmc passes of <= 8 SQ counters -> gpurun_out/sq_$TAG/summary.txt
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/sq_${TAG:-r3}
mkdir -p $OUT

B="python3 bench.py --config ${CFG:-c2} --steps 1 --warmup 0 --no-cpu-baseline --no-cycle --no-detail-configs"
PA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_VALU_CVT SQ_WAVE_CYCLES"
PB="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
# cache pass (optional: a counter this ROCm does not know fails the pass, not the script)
PC="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
i=0
for P in "$PA" "$PB"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "${KREGEX:-assemble|tq40}" -d $OUT/p$i -o p$i --output-format csv -- $B > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --pmc $PC --kernel-include-regex "${KREGEX:-assemble|tq40}" -d $OUT/p3 -o p3 --output-format csv -- $B > $OUT/p3.log 2>&1 || { echo "cache pass failed"; tail -3 $OUT/p3.log; }
python3 - $OUT <<'PY' | tee $OUT/summary.txt
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    w = m.get("SQ_WAVES", 1.0)
    print(k, "per wave:", ", ".join(f"{c[3:]}={v / w:.0f}" for c, v in sorted(m.items()) if c != "SQ_WAVES"),
          f"| waves/launch={w:.0f}")
PY
