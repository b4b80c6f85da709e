#!/bin/bash
# r4g: per-lane search restored + XCD-aware block order; bin-side sweep; GPU tests
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
LIBS="_ab/oldsearch _ab/xcd" REPS=2 STEPS=4 WARMUP=1 BENCH_ARGS="--no-transposes" timeout -k 10 300 bash scripts/ab_libs.sh 2>&1 | tee $O/ab_c2.txt
LIBS="_ab/oldsearch _ab/xcd" REPS=2 STEPS=2 WARMUP=1 BENCH_ARGS="--config c5 --no-transposes" timeout -k 10 400 bash scripts/ab_libs.sh 2>&1 | tee $O/ab_c5.txt
ENVS="CWBL_BIN_DIV=2 CWBL_BIN_DIV=3 CWBL_BIN_DIV=4" CFG=c5 REPS=1 STEPS=2 timeout -k 10 400 bash scripts/ab_env.sh 2>&1 | tee $O/bindiv_c5.txt
ENVS="CWBL_BIN_DIV=2 CWBL_BIN_DIV=3 CWBL_BIN_DIV=4" CFG=c2 REPS=1 STEPS=4 timeout -k 10 300 bash scripts/ab_env.sh 2>&1 | tee $O/bindiv_c2.txt
for T in 16 8 4; do OMP_NUM_THREADS=$T timeout -k 10 200 python3 scripts/host_memory_ab.py 3 2>&1 | tee -a $O/host_ab.txt; done
CWBL_PAGEABLE=register timeout -k 10 200 python3 scripts/host_memory_ab.py 3 2>&1 | sed 's/^/register: /' | tee -a $O/host_ab.txt
