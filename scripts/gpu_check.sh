#!/bin/bash
# first GPU run: parity tests, smoke, short bench
cd "$GRAFT_REPO_ROOT"
ls /opt/conda/lib/libmkl_rt.so > gpurun_out/env.txt 2>&1; nproc >> gpurun_out/env.txt; lscpu | grep "Model name" >> gpurun_out/env.txt; rocminfo | grep -m2 gfx >> gpurun_out/env.txt
timeout -k 10 900 python -m pytest tests -m gpu -q -rA > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 3; }
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/bench1.log 2>&1
echo "bench rc=$?"
tail -5 gpurun_out/pytest_gpu.log
cat gpurun_out/smoke.log
tail -3 gpurun_out/bench1.log
