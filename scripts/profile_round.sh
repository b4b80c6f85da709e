#!/bin/bash
# Per-kernel profile of the bench configurations (CONFIGS, default "c2 c4 c5"), one timed step
# each: kernel statistics (rocprofv3 --kernel-trace --stats), then separate --pmc passes for
# HBM traffic (FETCH_SIZE, WRITE_SIZE) and executed FP64 work (SQ FP64 VALU + MFMA ops) ->
# gpurun_out/prof_$TAG/<config>/; then scripts/pmc_kernels.py gpurun_out/prof_$TAG $TAG
# writes profiles/pmc_kernels.json and profiles/${TAG}_<config>_*.  SUFFIX / BENCH_EXTRA: e.g.
# SUFFIX=_one BENCH_EXTRA='--big-path 0' CONFIGS=c4 profiles the one-kernel k = 128 path.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r5}
B="--steps 1 --warmup 0 --no-cpu-baseline --no-cycle --no-detail-configs --no-transposes"
F64="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES"
for C in ${CONFIGS:-c2 c4 c5}; do
  OUT=gpurun_out/prof_$TAG/$C${SUFFIX:-}
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --config $C $B ${BENCH_EXTRA:-} > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 5; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 bench.py --config $C $B ${BENCH_EXTRA:-} > $OUT/fetch.log 2>&1 || { tail -5 $OUT/fetch.log; exit 6; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 bench.py --config $C $B ${BENCH_EXTRA:-} > $OUT/write.log 2>&1 || { tail -5 $OUT/write.log; exit 7; }
  timeout -s KILL 300 rocprofv3 --pmc $F64 --kernel-include-regex "solve|assemble" -d $OUT/f64 -o f64 --output-format csv -- python3 bench.py --config $C $B ${BENCH_EXTRA:-} > $OUT/f64.log 2>&1 || { tail -5 $OUT/f64.log; exit 8; }
  for d in kt fetch write f64; do f=$(find $OUT/$d -name "*.csv" | grep -E "kernel_stats|counter_collection" | head -1); [ -n "$f" ] && cp "$f" $OUT/$d/; done
  echo "== $C"; tail -1 $OUT/kt.log | cut -c1-300
done
python3 scripts/pmc_kernels.py gpurun_out/prof_$TAG $TAG
