#!/bin/bash
# Round check on one MI355X: the GPU test suite, smoke(), the default bench line, the
# rocprofv3 kernel statistics + HBM counters of C2 (gpu_profile.sh), and the kernel
# statistics of C4 (k = 128)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_default.log; exit 4; }
tail -1 gpurun_out/bench_default.log | cut -c1-400
TAG=$TAG scripts/gpu_profile.sh || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt_c4 -o kt --output-format csv -- python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline --no-cycle > $OUT/kt_c4_bench.log 2>&1 || exit 8
tail -1 $OUT/kt_c4_bench.log | cut -c1-300
