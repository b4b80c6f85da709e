#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
echo rc=$?
grep -c . gpurun_out/counters_list.txt
