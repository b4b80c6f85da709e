#!/bin/bash
# r4p: tail kernel matvec from LDS broadcasts (tlds) vs readlane (base2, = the r4o swz step): k > 64 parity tests, then C4 A/B + SQ counters of the tail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "big or large or c4 or k128 or solve_batch or eigen" --timeout 120 --timeout-method thread > gpurun_out/r4p_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4p_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for L in base2 tlds tlds2; do
    CWBL_LIBRARY=$PWD/_ab/$L/libcwbl.so timeout -k 10 200 python3 bench.py --config c4 --steps 2 --warmup 1 \
      --no-cpu-baseline --no-cycle --no-detail-configs > gpurun_out/r4p_$L.$rep.log 2>&1 || { tail -5 gpurun_out/r4p_$L.$rep.log; exit 4; }
    python3 - gpurun_out/r4p_$L.$rep.log $L $rep <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d.get('detail',{}).get('kernels_rank0',{})
print(sys.argv[2], sys.argv[3], round(d['value']/1e6,3), 'M', {n: round(v['avg_launch_ms'],3) for n,v in k.items() if 'big' in n or 'tqb' in n})
PY
  done
done
TAG=r4p CFG=c4 KREGEX="tqb_tail" timeout -k 10 600 bash scripts/sq_c2.sh
