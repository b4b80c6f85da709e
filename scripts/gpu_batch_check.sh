cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "batch_plan or ragged or split_kp40" 2>&1 | tail -2
bash scripts/gpu_batch_sweep8.sh
