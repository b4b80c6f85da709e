#!/bin/bash
# r4x: per-kernel profiles (kernel statistics, HBM traffic, executed FP64 work) of C2/C4/C5 after the search diet
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r4x timeout -k 10 900 bash scripts/profile_r4.sh > gpurun_out/r4x_profile.log 2>&1 || { tail -5 gpurun_out/r4x_profile.log; exit 3; }
grep "^==" -A1 gpurun_out/r4x_profile.log | cut -c1-200
