#!/bin/bash
# LDS conflict / instruction counters of solve_tq_kernel per ablation stage
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/tqconf_${TAG:-r1}
mkdir -p $OUT
for S in ${STAGES:-1 2 3 0}; do
  CWBL_DEBUG_TQ_STOP=$S timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-include-regex solve_tq -d $OUT/s$S -o s$S --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/s$S.log 2>&1
  rc=$?; echo "stage $S rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
