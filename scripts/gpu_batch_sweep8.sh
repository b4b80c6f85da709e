cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for mb in default 160000 100000; do
  echo "max_batch $mb: $($( [ $mb = default ] && echo env || echo env CWBL_MAX_BATCH=$mb ) timeout -k 10 200 python scripts/call_overhead.py 2>&1 | grep wall | tail -3 | awk '{s+=$2} END {printf "%.2f ms (mean of last 3 calls)", s/3}')"
done
