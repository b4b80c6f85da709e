#!/bin/bash
# split KP=40 path (assembly hand-off + four-points-per-wave solve): parity tests, then the
# bench with the split path on/off and hand-off batch sizes
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: pytest rc=$rc"; exit $rc; fi
for cfg in "CWBL_TQ4=0" "CWBL_TQ4=1" ${EXTRA_CFGS}; do
  env $cfg timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_tq4.log 2>&1 || { echo "bench $cfg failed"; tail -5 gpurun_out/bench_tq4.log; exit 4; }
  echo -n "$cfg: "; tail -1 gpurun_out/bench_tq4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.4g ms/step %.1f solve %.1f search %.1f TF %.2f' % (d['value'], d['ms_per_step'], d['detail']['ms_solve_per_step'], d['detail']['ms_search_per_step'], d['roofline']['achieved']))"
done
