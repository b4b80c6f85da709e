#!/bin/bash
# solve_tq40_kernel ablation instantiations (CWBL_DEBUG_TQ_STOP 4/2/3/0), then the split-path
# parity test and one bench line
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
CWBL_DEBUG_SERIAL=1 STOPS="${STOPS:-4 2 3 0}" bash scripts/gpu_ablate_c2.sh | grep -E "stop=|tq40|assemble" || exit 1
bash scripts/gpu_tq40.sh
