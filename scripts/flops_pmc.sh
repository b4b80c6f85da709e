#!/bin/bash
# Executed FP64 work of the C2 solve kernels (one bench step): FP64 VALU instruction counts
# and F64 MFMA ops, one rocprofv3 --pmc pass (6 SQ counters), summarised per launch and per
# wave into gpurun_out/flops/summary.json
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/flops
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1
grep -E "^[[:space:]]*SQ_INSTS_VALU_(FMA|ADD|MUL|TRANS)_F64|MFMA_MOPS_F64" $OUT/counters_list.txt | head -20
P="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES"
timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "solve|assemble" -d $OUT/p1 -o p1 --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-cycle --no-detail-configs > $OUT/p1.log 2>&1 || { echo "pmc pass failed"; tail -5 $OUT/p1.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys, json, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p1/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, d in agg.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    waves = m.get("SQ_WAVES", 1.0)
    valu = 64 * (2 * m.get("SQ_INSTS_VALU_FMA_F64", 0) + m.get("SQ_INSTS_VALU_ADD_F64", 0)
                 + m.get("SQ_INSTS_VALU_MUL_F64", 0) + m.get("SQ_INSTS_VALU_TRANS_F64", 0))
    mfma = 512 * m.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0)
    out[k] = dict(counters_per_launch=m, launches=len(d.get("SQ_WAVES", [])),
                  fp64_valu_flops_per_launch=valu, fp64_mfma_flops_per_launch=mfma,
                  fp64_flops_per_launch=valu + mfma)
    print(k, json.dumps({c: round(v / waves, 1) for c, v in m.items()}),
          "valu GF %.3g mfma GF %.3g per launch" % (valu / 1e9, mfma / 1e9))
json.dump(out, open(sys.argv[1] + "/summary.json", "w"), indent=1)
PY
