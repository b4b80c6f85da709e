#!/bin/bash
# record sub-batch sweep (CWBL_TQ4_SUB) on the two-stream record path, alternating
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for i in 1 2; do for sb in 0 50000 25000; do
  CWBL_TQ4_SUB=$sb timeout -k 10 300 python bench.py --no-cpu-baseline --no-cycle --steps 6 > gpurun_out/sub_$sb.log 2>&1 || exit 1
  echo "sub $sb: $(tail -1 gpurun_out/sub_$sb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step %.2f' % d['ms_per_step'])")"
done; done
