#!/bin/bash
# r4d: host-slab tests, bench N=1 (all legs but the CPU baseline), then the r4 profiles
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench1.log 2>&1 || { tail -20 $O/bench1.log; exit 4; }
grep -o '"host_memory": {.*' $O/bench1.log | cut -c1-600
timeout -k 10 60 ./scripts/microbench/mb_i8 > $O/mb_i8.txt 2>&1; cat $O/mb_i8.txt
TAG=r4a bash scripts/profile_r4.sh > $O/profile.log 2>&1 || { tail -30 $O/profile.log; exit 5; }
tail -40 $O/profile.log
# C4 library A/B: round-3 step vs four-chain row sums vs + no vb barrier
LIBS="_ab/base _ab/rs4 _ab/vbc" REPS=2 STEPS=3 WARMUP=1 BENCH_ARGS="--config c4 --no-transposes" timeout -k 10 400 bash scripts/ab_libs.sh 2>&1 | tee $O/ab_c4.txt
# C4 two-stream split path (tail beside the next hand-off kernel), env A/B on the current library
ENVS="CWBL_BIG_STREAMS=0 CWBL_BIG_STREAMS=1 CWBL_BIG_STREAMS=1,CWBL_BIG_SUB=40000" CFG=c4 REPS=2 STEPS=2 timeout -k 10 400 bash scripts/ab_env.sh 2>&1 | tee $O/ab_c4_streams.txt
