#!/bin/bash
# lead-batch sweep at an 8-GPU rank's C2 share (scripts/call_overhead.py), alternating
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for i in 1 2; do for ld in 0 12 24; do
  echo "lead_div $ld: $(CWBL_LEAD_DIV=$ld timeout -k 10 200 python scripts/call_overhead.py 2>&1 | grep wall | tail -3 | awk '{s+=$2} END {printf "%.2f ms (mean of last 3 calls)", s/3}')"
done; done
