#!/bin/bash
# r4t2: world-1 transposes pack/unpack straight into/out of the slab (no self-copy)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_transpose.py tests/test_gpu_multi_rank.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4t2_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r4t2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-detail-configs > gpurun_out/r4t2_bench.log 2>&1 || { tail -5 gpurun_out/r4t2_bench.log; exit 4; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/r4t2_bench.log').read().strip().splitlines()[-1])
print(round(d['value']/1e6,3), 'M', d['detail']['transposes'], {k: v for k, v in d['detail']['cycle'].items() if k.endswith('_ms')})
PY
