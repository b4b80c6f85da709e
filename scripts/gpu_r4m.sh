#!/bin/bash
# r4l: record kernel with the 4x4-block cover (assemble_record_blocks_kernel): full GPU suite, then A/B
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "driver or c2 or oracle or pipelined" --timeout 120 --timeout-method thread > gpurun_out/r4l_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4l_tests.log; [ $rc -eq 0 ] || exit $rc
summ() {
  for f in gpurun_out/abenv/*.log; do
    python3 - "$f" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d.get('detail',{}).get('kernels_rank0',{})
print(sys.argv[1].split('/')[-1], {n: round(v['avg_launch_ms'],4) for n,v in k.items() if 'search_binned' in n or 'assemble' in n or 'tq40' in n})
PY
  done
}
rm -rf gpurun_out/abenv
ENVS="CWBL_ASM_COVER=0 CWBL_ASM_COVER=1" CFG=c2 REPS=3 STEPS=6 timeout -k 10 400 bash scripts/ab_env.sh || exit 5
summ
mkdir -p gpurun_out/abenv_l2 && mv gpurun_out/abenv/*.log gpurun_out/abenv_l2/
summ
