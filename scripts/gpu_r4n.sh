#!/bin/bash
# r4n: where the k = 128 hand-off kernel's time goes: SQ counters of the C4 pair, and the
# assembly/staging ablations of a DEBUG_KNOBS library (_ab/dbg, CWBL_DEBUG_TQ_STOP 12 = staging
# only, 1 = staging + MFMA assembly; the tail then runs on an unfinished hand-off)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r4n CFG=c4 KREGEX="tq_big|tqb_tail" timeout -k 10 600 bash scripts/sq_c2.sh || exit 3
for S in 0 12 1; do
  CWBL_LIBRARY=$PWD/_ab/dbg/libcwbl.so CWBL_DEBUG_TQ_STOP=$S timeout -k 10 200 python3 bench.py --config c4 --steps 1 --warmup 1 \
    --no-cpu-baseline --no-cycle --no-detail-configs > gpurun_out/r4n_stop$S.log 2>&1 || { tail -5 gpurun_out/r4n_stop$S.log; exit 4; }
  python3 - gpurun_out/r4n_stop$S.log $S <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d.get('detail',{}).get('kernels_rank0',{})
print('stop', sys.argv[2], {n: (v['launches'], round(v['avg_launch_ms'],3)) for n,v in k.items() if 'big' in n or 'tail' in n or 'tqb' in n})
PY
done
