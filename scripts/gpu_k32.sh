#!/bin/bash
# k = 25..32 on the KP = 40 record path: parity tests, then the C2 grid at k = 25, 32, 40
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "split_kp40 or ragged or error" > gpurun_out/pytest_k32.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_k32.log
[ $rc -eq 0 ] || { grep -E "^FAILED|^E  " gpurun_out/pytest_k32.log | head -20; exit $rc; }
timeout -k 10 400 python scripts/k_sweep.py 25 32 40
