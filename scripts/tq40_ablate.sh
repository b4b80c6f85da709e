#!/bin/bash
# solve_tq40_kernel time split on the C2 bench (CWBL_DEBUG_TQ_STOP ablations: 5 = the record
# loads only, 4 = + phase 1, 2 = + phase 2 (the whole tridiagonalisation), 3 = + quadrature,
# 0 = whole kernel), kernel statistics per ablation -> gpurun_out/tq40_ablate/<stop>/
# (needs a library built with the knobs, make DEBUG_KNOBS=1, e.g. in a copy of the tree and
# passed as CWBL_LIBRARY=<copy>/cwbnwp-letkf_amd/lib/libcwbl.so)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/tq40_ablate
mkdir -p $OUT
for S in ${STOPS:-0 5 4 2 3}; do
  CWBL_DEBUG_TQ_STOP=$S timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/$S -o kt --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cycle --no-detail-configs > $OUT/$S.log 2>&1 || { tail -5 $OUT/$S.log; exit 5; }
  f=$(find $OUT/$S -name "*kernel_stats.csv" | head -1)
  echo "== stop $S"; grep -E "solve_tq40|assemble_record" "$f" | cut -d, -f1-8
done
