#!/bin/bash
# r4k: quad search vs lane search x stream priorities (C2), then C5
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
summ() {
  for f in gpurun_out/abenv/*.log; do
    python3 - "$f" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d.get('detail',{}).get('kernels_rank0',{})
print(sys.argv[1].split('/')[-1], {n: round(v['avg_launch_ms'],4) for n,v in k.items() if 'search_binned' in n or 'assemble' in n or 'tq40' in n})
PY
  done
}
timeout -k 10 60 python3 -c "import ctypes; l=ctypes.CDLL('/opt/rocm/lib/libamdhip64.so'); a=ctypes.c_int(); b=ctypes.c_int(); print('prio range', l.hipDeviceGetStreamPriorityRange(ctypes.byref(a), ctypes.byref(b)), a.value, b.value)"
ENVS="CWBL_SEARCH_LANE=1 CWBL_SEARCH_LANE=0 CWBL_SEARCH_LANE=0,CWBL_SSTREAM_PRIO=1 CWBL_SEARCH_LANE=0,CWBL_SSTREAM_PRIO=2 CWBL_SEARCH_LANE=1,CWBL_SSTREAM_PRIO=1" CFG=c2 REPS=2 STEPS=6 timeout -k 10 500 bash scripts/ab_env.sh || exit 5
summ
mkdir -p gpurun_out/abenv_k2 && mv gpurun_out/abenv/*.log gpurun_out/abenv_k2/
ENVS="CWBL_SEARCH_LANE=1 CWBL_SEARCH_LANE=0 CWBL_SEARCH_LANE=0,CWBL_SSTREAM_PRIO=1" CFG=c5 REPS=1 STEPS=2 timeout -k 10 400 bash scripts/ab_env.sh || exit 6
summ
