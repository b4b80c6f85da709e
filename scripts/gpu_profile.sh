#!/bin/bash
# rocprofv3: kernel trace + stats of the bench, then HBM PMC counters in separate passes
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-r1}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cycle > $OUT/kt_bench.log 2>&1 || exit 5
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-cycle > $OUT/fetch_bench.log 2>&1 || exit 6
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-cycle > $OUT/write_bench.log 2>&1 || exit 7
find $OUT -name "*.csv" | head -20
tail -1 $OUT/kt_bench.log | cut -c1-300
