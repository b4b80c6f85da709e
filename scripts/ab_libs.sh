#!/bin/bash
# A/B of library builds on the C2 bench, interleaved in one run: LIBS="dir1 dir2 ..." (each
# holding a libcwbl.so), REPS rounds; extra bench flags in BENCH_ARGS
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${REPS:-3}); do
  for L in $LIBS; do
    tag=$(basename $L)
    CWBL_LIBRARY=$PWD/$L/libcwbl.so timeout -k 10 120 python3 bench.py --steps ${STEPS:-6} --warmup ${WARMUP:-2} \
      --no-cpu-baseline --no-cycle --no-detail-configs $BENCH_ARGS > gpurun_out/ab/$tag.$rep.log 2>&1 || { tail -5 gpurun_out/ab/$tag.$rep.log; exit 5; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['detail']['kernels_rank0']; print(sys.argv[2], 'rep', sys.argv[3], round(d['value']/1e6,2), 'M', round(d['ms_per_step'],2), 'ms', ' '.join(n.split('<')[0]+'='+str(round(e['avg_launch_ms'],4)) for n,e in k.items() if e['avg_launch_ms']>0.1))" gpurun_out/ab/$tag.$rep.log $tag $rep
  done
done
