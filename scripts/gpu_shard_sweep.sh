#!/bin/bash
# rank-0 share of the C2 grid at world 8 (and 1) under batch-plan settings (CWBL_MAX_BATCH,
# CWBL_LEAD_DIV): the per-rank step time of the strong-scaling bench
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for cfg in ${CFGS:-"160000:0" "160000:8" "120000:0" "100000:0" "100000:10" "80000:0"}; do
  mb=${cfg%%:*}; ld=${cfg##*:}
  echo -n "max_batch=$mb lead_div=$ld: "
  CWBL_MAX_BATCH=$mb CWBL_LEAD_DIV=$ld timeout -k 10 300 python scripts/shard_rehearsal.py ${WORLDS:-8} 2>&1 | grep world || exit 1
done
