#!/bin/bash
# C2 step time (world 1) under batch caps, alternating, in one run
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for i in 1 2; do for mb in 160000 120000 100000; do
  CWBL_MAX_BATCH=$mb timeout -k 10 300 python bench.py --no-cpu-baseline --no-cycle --steps 8 > gpurun_out/bs_$mb.log 2>&1 || exit 1
  echo "max_batch $mb: $(tail -1 gpurun_out/bs_$mb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step %.2f' % d['ms_per_step'])")"
done; done
