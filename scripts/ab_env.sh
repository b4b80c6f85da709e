#!/bin/bash
# A/B of environment settings on one bench configuration, interleaved in one run:
# ENVS="CWBL_TILE=0 CWBL_TILE=2" (one setting, or several joined by commas, per variant),
# CFG (c2), REPS, STEPS
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abenv
for rep in $(seq 1 ${REPS:-2}); do
  for E in $ENVS; do
    tag=$(echo "$E" | tr ',=' '__')
    env $(echo "$E" | tr ',' ' ') timeout -k 10 200 python3 bench.py --config ${CFG:-c2} --steps ${STEPS:-4} --warmup 1 \
      --no-cpu-baseline --no-cycle --no-detail-configs > gpurun_out/abenv/$tag.$rep.log 2>&1 || { tail -5 gpurun_out/abenv/$tag.$rep.log; exit 5; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'rep', sys.argv[3], round(d['value']/1e6,3), 'M', round(d['ms_per_step'],2), 'ms')" gpurun_out/abenv/$tag.$rep.log "$E" $rep
  done
done
