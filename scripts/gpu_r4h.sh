#!/bin/bash
# r4h: final r4 build: GPU tests, smoke, full bench (CPU baseline included), profiles, gloo N=2
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 4; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $O/bench1.log 2>&1 || { tail -20 $O/bench1.log; exit 5; }
TAG=r4c bash scripts/profile_r4.sh > $O/profile.log 2>&1 || { tail -30 $O/profile.log; exit 6; }
grep -E "^== " -A1 $O/profile.log | cut -c1-200
CWBL_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --no-detail-configs > $O/bench2.log 2>&1 || { tail -20 $O/bench2.log; exit 7; }
echo done
