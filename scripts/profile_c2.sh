#!/bin/bash
# Profile of the default C2 bench path: kernel statistics, HBM PMC passes (FETCH_SIZE,
# WRITE_SIZE), executed FP64 work (SQ counters) -> gpurun_out/prof_$TAG, gpurun_out/flops
# (then: python scripts/pmc_summary.py gpurun_out/prof_$TAG $TAG -> profiles/)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-r3}
# kernel durations with the solves on the assembly stream (CWBL_TQ40_STREAMS=0): with two
# streams the two kernels overlap and each launch looks longer
export CWBL_TQ40_STREAMS=${CWBL_TQ40_STREAMS:-0}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-cycle --no-detail-configs > $OUT/kt_bench.log 2>&1 || { tail -5 $OUT/kt_bench.log; exit 5; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-cycle --no-detail-configs > $OUT/fetch_bench.log 2>&1 || { tail -5 $OUT/fetch_bench.log; exit 6; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-cycle --no-detail-configs > $OUT/write_bench.log 2>&1 || { tail -5 $OUT/write_bench.log; exit 7; }
for d in kt fetch write; do f=$(find $OUT/$d -name "*.csv" | grep -E "kernel_stats|counter_collection" | head -1); [ -n "$f" ] && cp "$f" $OUT/$d/; done
ls $OUT/kt $OUT/fetch $OUT/write
bash scripts/flops_pmc.sh || exit 8
tail -1 $OUT/kt_bench.log | cut -c1-400
