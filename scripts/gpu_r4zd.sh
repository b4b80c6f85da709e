#!/bin/bash
# r4zd: the flag counters zeroed by the previous batch's flagged search (m1) instead of a memset launch per batch (m0)

cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4zd_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4zd_tests.log; [ $rc -eq 0 ] || exit $rc
for C in c2 c5; do
  for rep in 1 2 3; do
    [ $C = c5 ] && [ $rep = 3 ] && continue
    for L in m0 m1; do
      CWBL_LIBRARY=$PWD/_ab/$L/libcwbl.so timeout -k 10 200 python3 bench.py --config $C --steps $([ $C = c5 ] && echo 2 || echo 10) --warmup 1 \
        --no-cpu-baseline --no-cycle --no-detail-configs > gpurun_out/r4zd_$C.$L.$rep.log 2>&1 || { tail -5 gpurun_out/r4zd_$C.$L.$rep.log; exit 4; }
      python3 - gpurun_out/r4zd_$C.$L.$rep.log $C $L $rep <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=d.get('roofline') or {}
print(sys.argv[2], sys.argv[3], sys.argv[4], round(d['value']/1e6,3), 'M', round(d['ms_per_step'],2), 'ms', round(r.get('avg_launch_ms') or 0,4), round(r.get('frac') or 0,4), 'nonconv', d['detail'].get('nonconverged'), 'solved', d['detail'].get('solved_per_step'))
PY
    done
  done
done
