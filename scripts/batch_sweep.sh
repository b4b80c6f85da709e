#!/bin/bash
# C2 rate against the batch cap (CWBL_MAX_BATCH) and the record path's stream count
# (CWBL_TQ40_STREAMS), interleaved in one run: BATCHES="..." STREAMS="..." REPS=n
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/batch_sweep
for rep in $(seq 1 ${REPS:-2}); do
  for B in ${BATCHES:-160000 40000}; do
    for S in ${STREAMS:-1 0}; do
      CWBL_MAX_BATCH=$B CWBL_TQ40_STREAMS=$S timeout -k 10 120 python3 bench.py --steps 6 --warmup 2 \
        --no-cpu-baseline --no-cycle --no-detail-configs > gpurun_out/batch_sweep/b$B.s$S.$rep.log 2>&1 || exit 5
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('batch', sys.argv[2], 'streams', sys.argv[3], 'rep', sys.argv[4], round(d['value']/1e6,2), 'M', round(d['ms_per_step'],2), 'ms')" gpurun_out/batch_sweep/b$B.s$S.$rep.log $B $S $rep
    done
  done
done
