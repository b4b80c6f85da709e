#!/bin/bash
# SQ counters of the solve kernels at CWBL_DEBUG_TQ_STOP = 1 (staging + assembly) and 0 (full)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for st in ${STOPS:-1 0}; do
  CWBL_DEBUG_TQ_STOP=$st TAG=${TAG:-x}_s$st KRE=${KRE:-solve_tq} scripts/gpu_sq_kernels.sh || exit $?
done
