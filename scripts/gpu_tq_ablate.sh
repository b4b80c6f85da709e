#!/bin/bash
# Phase ablation of solve_tq_kernel (CWBL_DEBUG_TQ_STOP) + SQ counters of the full kernel
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/tqab_${TAG:-r1}
mkdir -p $OUT
for S in ${STAGES:-0 1 2 3}; do
  CWBL_DEBUG_TQ_STOP=$S timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/stop$S.log 2>&1 || exit 4
  echo "stop=$S $(tail -1 $OUT/stop$S.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['detail']['ms_solve_per_step'])")"
done
[ -z "$PMC" ] && exit 0
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
         "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex solve_tq -d $OUT/p$i -o p$i --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
