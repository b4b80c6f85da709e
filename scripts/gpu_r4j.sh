#!/bin/bash
# r4j: LDS-staged binned search (search_binned_stage_kernel) — parity, then A/B against the per-lane form
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "binned or search or driver or c5 or c2_full or oracle_block" > gpurun_out/r4j_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4j_tests.log; [ $rc -eq 0 ] || exit $rc
ENVS="CWBL_SEARCH_LANE=0 CWBL_SEARCH_LANE=1" CFG=c2 REPS=2 STEPS=6 timeout -k 10 300 bash scripts/ab_env.sh || exit 5
for f in gpurun_out/abenv/CWBL_SEARCH_LANE_*.log; do
  python3 - "$f" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d.get('detail',{}).get('kernels_rank0',{})
print(sys.argv[1].split('/')[-1], {n: round(v['avg_launch_ms'],4) for n,v in k.items() if 'search' in n or 'assemble' in n})
PY
done
mkdir -p gpurun_out/abenv_c2 && mv gpurun_out/abenv/CWBL_SEARCH_LANE_* gpurun_out/abenv_c2/
ENVS="CWBL_SEARCH_LANE=0 CWBL_SEARCH_LANE=1" CFG=c5 REPS=1 STEPS=2 timeout -k 10 300 bash scripts/ab_env.sh || exit 6
for f in gpurun_out/abenv/CWBL_SEARCH_LANE_*.log; do
  python3 - "$f" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d.get('detail',{}).get('kernels_rank0',{})
print(sys.argv[1].split('/')[-1], {n: round(v['avg_launch_ms'],4) for n,v in k.items() if 'search' in n or 'assemble' in n})
PY
done
