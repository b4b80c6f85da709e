#!/bin/bash
# Effective clock of the solve kernels: GRBM_GUI_ACTIVE (GPU busy cycles) per launch over the
# launch's duration (the counter CSV's timestamps), one bench step, one rocprofv3 --pmc pass
# -> gpurun_out/clock_$TAG/summary.txt
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/clock_${TAG:-r6}_${CFG:-c2}
mkdir -p $OUT
B="python3 bench.py --config ${CFG:-c2} --steps 1 --warmup 0 --no-cpu-baseline --no-cycle --no-detail-configs --no-transposes"
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "${KREGEX:-assemble|tq40|rows|tail}" -d $OUT/p -o p --output-format csv -- $B > $OUT/p.log 2>&1 || { echo "clock pass failed"; tail -5 $OUT/p.log; exit 1; }
python3 - $OUT <<'PY' | tee $OUT/summary.txt
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            agg[k]["_ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
for k, d in agg.items():
    n = max(len(d["GRBM_GUI_ACTIVE"]), 1)
    g = sum(d["GRBM_GUI_ACTIVE"]) / n
    c = sum(d.get("GRBM_COUNT", [0])) / max(len(d.get("GRBM_COUNT", [])), 1)
    ns = sum(d["_ns"]) / max(len(d["_ns"]), 1)
    print(k, f"launches={n} GRBM_GUI_ACTIVE={g:.0f} GRBM_COUNT={c:.0f} avg_ns={ns:.0f} "
          f"clock_GHz={g / ns if ns else 0:.3f}")
PY
