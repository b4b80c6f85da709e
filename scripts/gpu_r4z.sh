#!/bin/bash
# r4z: what the per-kernel HIP-event timing costs the C2 step (CWBL_BENCH_KT=0: no kernel events)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/abenv
ENVS="CWBL_BENCH_KT=1 CWBL_BENCH_KT=0" CFG=c2 REPS=3 STEPS=10 timeout -k 10 400 bash scripts/ab_env.sh || exit 5
