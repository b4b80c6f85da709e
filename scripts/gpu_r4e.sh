#!/bin/bash
# r4e: search fix: GPU tests, search A/B (C2, C5), bench N=1, r4b profiles
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
LIBS="_ab/oldsearch _ab/new" REPS=2 STEPS=4 WARMUP=1 BENCH_ARGS="--no-transposes" timeout -k 10 300 bash scripts/ab_libs.sh 2>&1 | tee $O/ab_c2.txt
LIBS="_ab/oldsearch _ab/new" REPS=2 STEPS=2 WARMUP=1 BENCH_ARGS="--config c5 --no-transposes" timeout -k 10 400 bash scripts/ab_libs.sh 2>&1 | tee $O/ab_c5.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench1.log 2>&1 || { tail -20 $O/bench1.log; exit 4; }
TAG=r4b bash scripts/profile_r4.sh > $O/profile.log 2>&1 || { tail -30 $O/profile.log; exit 5; }
grep -E "^== |\"value\"" $O/profile.log | cut -c1-200
