#!/bin/bash
# r4y: binned search look-ahead 8 (r4) vs 16 vs 4 points per round
# at once instead of assembled into int4 groups (sb2; half the VALU of the kernel body) vs r4 (sb0)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "binned or search or driver or c5 or c2_full or oracle_block or batch_plan" --timeout 120 --timeout-method thread > gpurun_out/r4y_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4y_tests.log; [ $rc -eq 0 ] || exit $rc
for C in c2 c5; do
  for rep in 1 2 3; do
    for L in ba8 ba16 ba4; do
      [ $C = c5 ] && [ $rep = 3 ] && continue
      CWBL_LIBRARY=$PWD/_ab/$L/libcwbl.so timeout -k 10 200 python3 bench.py --config $C --steps $([ $C = c5 ] && echo 2 || echo 6) --warmup 1 \
        --no-cpu-baseline --no-cycle --no-detail-configs > gpurun_out/r4y_$C.$L.$rep.log 2>&1 || { tail -5 gpurun_out/r4y_$C.$L.$rep.log; exit 4; }
      python3 - gpurun_out/r4y_$C.$L.$rep.log $C $L $rep <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d.get('detail',{}).get('kernels_rank0',{})
print(sys.argv[2], sys.argv[3], sys.argv[4], round(d['value']/1e6,3), 'M', {n: round(v['avg_launch_ms'],4) for n,v in k.items() if 'search' in n or 'assemble' in n or 'tq40' in n})
PY
    done
  done
done
