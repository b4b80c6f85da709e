#!/bin/bash
# GPU run: parity tests + bench (+ optional sweep ablations)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "stop: pytest rc=$rc"; exit $rc; fi
timeout -k 10 600 python bench.py --steps 3 --warmup 1 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || exit 4
tail -1 gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'], d['detail'], 'mean_p', d['config']['mean_p'], 'TF', d['roofline']['achieved'], d['roofline']['kernel'], d.get('cpu_baseline'))"
