#!/bin/bash
# GPU run: parity tests, bench, sweep ablation, rocprofv3 kernel trace of the bench
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: pytest rc=$rc"; exit $rc; fi
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1 || exit 4
CWBL_DEBUG_MAX_SWEEPS=0 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_sw0.log 2>&1 || exit 5
CWBL_DEBUG_MAX_SWEEPS=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_sw1.log 2>&1 || exit 6
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit 7
tail -3 gpurun_out/pytest_gpu.log
for f in bench bench_sw0 bench_sw1; do echo $f; tail -1 gpurun_out/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['detail'], d['config']['mean_p'], d['roofline']['achieved'], d.get('cpu_baseline'))"; done
find gpurun_out/prof -name "*stats*"
