#!/bin/bash
# r4zb: kernel timing with the record path's pair timed between events the call records anyway
# (kt2: one extra event per batch) vs two pairs of events (kt4); C2, timing on; and off for reference
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi_rank.py -x -q -k "c2_full or batch_plan or pipelined or kernel_tim or bench_two" --timeout 300 --timeout-method thread > gpurun_out/r4zb_tests.log 2>&1; tail -1 gpurun_out/r4zb_tests.log
for rep in 1 2 3; do
  for L in kt4 kt2; do
    for KT in 1 0; do
      CWBL_BENCH_KT=$KT CWBL_LIBRARY=$PWD/_ab/$L/libcwbl.so timeout -k 10 200 python3 bench.py --steps 10 --warmup 1 \
        --no-cpu-baseline --no-cycle --no-detail-configs > gpurun_out/r4zb_$L.$KT.$rep.log 2>&1 || { tail -5 gpurun_out/r4zb_$L.$KT.$rep.log; exit 4; }
      python3 - gpurun_out/r4zb_$L.$KT.$rep.log $L $KT $rep <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=d.get('roofline') or {}
print(sys.argv[2], 'KT', sys.argv[3], sys.argv[4], round(d['value']/1e6,3), 'M', round(d['ms_per_step'],2), 'ms', r.get('kernel'), round(r.get('avg_launch_ms') or 0,4), round(r.get('frac') or 0,4))
PY
    done
  done
done
