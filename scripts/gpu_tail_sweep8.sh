#!/bin/bash
# short-tail sweep at an 8-GPU rank's C2 share (scripts/call_overhead.py), alternating
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for i in 1 2; do for td in 0 2 4; do
  echo "tail_div $td: $(CWBL_TAIL_DIV=$td timeout -k 10 200 python scripts/call_overhead.py 2>&1 | grep wall | tail -3 | awk '{s+=$2} END {printf "%.2f ms (mean of last 3 calls)", s/3}')"
done; done
