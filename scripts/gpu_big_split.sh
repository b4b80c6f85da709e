#!/bin/bash
# k = 128 split path (solve_tq_big_kernel<128,false,64> + solve_tqb_tail_kernel): parity
# tests, then the C4 bench split and one-kernel, then a kernel-trace profile of the split
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
[ "$TESTK" = none ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "${TESTK:-split_big or large_ensemble or c4_full}" > gpurun_out/pytest_split.log 2>&1
rc=$?; [ "$TESTK" = none ] || tail -12 gpurun_out/pytest_split.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_split.log | head -20; exit $rc; }
for sp in ${SPLITS:-1 0}; do
  CWBL_BIG_SPLIT=$sp timeout -k 10 300 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-cycle > gpurun_out/bench_c4_$sp.log 2>&1 || { echo "bench split=$sp failed"; tail -5 gpurun_out/bench_c4_$sp.log; exit 4; }
  echo -n "split=$sp: "; tail -1 gpurun_out/bench_c4_$sp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g ms/step %.1f solve %.1f search %.1f TF %.2f' % (d['value'], d['ms_per_step'], d['detail']['ms_solve_per_step'], d['detail']['ms_search_per_step'], d['roofline']['achieved']))"
done
if [ -n "$PROF" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4 -o c4 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-cycle > $GRAFT_REPO_ROOT/gpurun_out/prof_c4.log 2>&1
  echo "prof rc=$?"; cd $GRAFT_REPO_ROOT
  f=$(find gpurun_out/prof_c4 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -8
fi
