#!/bin/bash
# GPU suite with the in-tree library, then an interleaved A/B of prebuilt libraries
# (_ab/*.so, untracked) on the C2 bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^FAILED|^E  " gpurun_out/pytest_gpu.log | head -30; exit $rc; }
bash scripts/gpu_ab.sh
