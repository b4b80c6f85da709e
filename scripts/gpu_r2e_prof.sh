#!/bin/bash
# Round-2 profile of the default bench path: kernel statistics, HBM PMC passes (FETCH_SIZE,
# WRITE_SIZE), executed FP64 work (SQ counters) -> gpurun_out/prof_$TAG, gpurun_out/flops
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-r2e}
# kernel durations with the solves on the assembly stream (CWBL_TQ40_STREAMS=0): with two
# streams the two kernels overlap and each launch looks longer
export CWBL_TQ40_STREAMS=${CWBL_TQ40_STREAMS:-0}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cycle > $OUT/kt_bench.log 2>&1 || { tail -5 $OUT/kt_bench.log; exit 5; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-cycle > $OUT/fetch_bench.log 2>&1 || { tail -5 $OUT/fetch_bench.log; exit 6; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-cycle > $OUT/write_bench.log 2>&1 || { tail -5 $OUT/write_bench.log; exit 7; }
for d in kt fetch write; do f=$(find $OUT/$d -name "*.csv" | grep -E "kernel_stats|counter_collection" | head -1); [ -n "$f" ] && cp "$f" $OUT/$d/; done
ls $OUT/kt $OUT/fetch $OUT/write
bash scripts/gpu_flops_pmc.sh || exit 8
tail -1 $OUT/kt_bench.log | cut -c1-400
