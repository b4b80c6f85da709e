#!/usr/bin/env python3
"""C2 bench timing under several batch plans, interleaved in one process:
python scripts/batch_ab.py [reps] [steps].  Each plan sets cwbl options (CWBL_OPT_MAX_BATCH,
CWBL_OPT_LEAD_DIV) for bench.time_config("c2"); one line per plan and repetition."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
PLANS = [("default", {}),
         ("max 230k", {"max_batch": 230000}),
         ("max 320k", {"max_batch": 320000}),
         ("max 128k", {"max_batch": 128000}),
         ("max 100k", {"max_batch": 100000}),
         ("max 64k", {"max_batch": 64000}),
         ("max 160k lead 16", {"max_batch": 160000, "lead_div": 16}),
         ("max 80k", {"max_batch": 80000}),
         ("rec 78k", {"split40_batch": 78000}),
         ("rec 52k", {"split40_batch": 52000}),
         ("rec 39k", {"split40_batch": 39000})]
if os.environ.get("PLANS"):  # a subset by index, e.g. PLANS=0,3,4
    PLANS = [PLANS[int(i)] for i in os.environ["PLANS"].split(",")]
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
for rep in range(reps):
    for name, opts in PLANS:
        bench.CORE_OPTIONS.clear()
        bench.CORE_OPTIONS.update(opts)
        r = bench.time_config("c2", 0, 1, 0, dev, steps, 1)
        k = r["kernels_rank0"]
        launches = {n.split("<")[0]: e["launches"] for n, e in k.items() if e["launches"]}
        print(f"{name:18s} rep {rep}: {r['value'] / 1e6:6.2f} M  {r['ms_per_step']:6.2f} ms/step"
              f"  launches {launches.get('assemble_record_kernel', 0) // steps} per step", flush=True)
