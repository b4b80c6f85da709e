#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/mfma_${TAG:-r1}
mkdir -p $OUT
for S in ${STAGES:-0 1}; do
  CWBL_DEBUG_TQ_STOP=$S timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAVES --kernel-include-regex solve_tq -d $OUT/s$S -o s$S --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/s$S.log 2>&1
  rc=$?; echo "stage $S rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
