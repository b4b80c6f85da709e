#!/bin/bash
# r4w: full GPU suite on the leaner binned search, then C2 / C5 bench lines
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4w_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4w_tests.log; [ $rc -eq 0 ] || exit $rc
for C in c2 c5; do
  timeout -k 10 200 python3 bench.py --config $C --steps $([ $C = c5 ] && echo 2 || echo 10) --warmup 1 --no-cpu-baseline --no-cycle --no-detail-configs > gpurun_out/r4w_$C.log 2>&1 || { tail -5 gpurun_out/r4w_$C.log; exit 4; }
  python3 - gpurun_out/r4w_$C.log $C <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d.get('detail',{}).get('kernels_rank0',{})
print(sys.argv[2], round(d['value']/1e6,3), 'M', round(d['ms_per_step'],2), 'ms', 'frac', round(d['roofline']['frac'],4), {n: round(v['avg_launch_ms'],4) for n,v in k.items() if 'search' in n or 'assemble' in n or 'tq40' in n})
PY
done
