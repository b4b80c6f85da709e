#!/usr/bin/env python3
"""Rank 0's share of the C2 grid at world size W (default 8), timed alone on one GPU under
several batch plans: per call the wall time around cwbl_analyze_var and the call's own
ms_total, so the host-side gap between calls shows.  python scripts/share_ab.py [W] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "cwbnwp-letkf_amd"))
import torch  # noqa: E402

from cwbl import abi, synth  # noqa: E402
from cwbl import dist as cdist  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
PLANS = [("default", {}), ("lead 8", {"lead_div": 8}), ("lead 16", {"lead_div": 16}),
         ("max 70k", {"max_batch": 70000}), ("max 141k", {"max_batch": 141000})]
if os.environ.get("PLANS"):  # a subset by index, e.g. PLANS=0
    PLANS = [PLANS[int(i)] for i in os.environ["PLANS"].split(",")]
dev = torch.device("cuda", 0)
w = synth.make("c2", shard=(0, world) if world > 1 else None)
types = [dict(family=1, type_id=w.radar_type, xyz=w.obs_xyz, obs=w.obs, hdxb=w.hdxb)]
_, types = cdist.unpack_obs_set(torch.from_numpy(cdist.pack_obs_set(types, w.k)).to(dev))
x, y, alt = (torch.from_numpy(a).to(dev) for a in (w.x, w.y, w.alt))
var = torch.from_numpy(w.var).to(dev)
slab = abi.make_slab(x, y, alt, var, memory=abi.MEM_DEVICE)
for rep in range(reps):
    for name, opts in PLANS:
        core = abi.Core(w.k, device=0, options=opts)
        core.set_obs(cdist.builder_from(types, abi.MEM_DEVICE).build())
        core.analyze_var(w.vp, slab)
        torch.cuda.synchronize()
        walls, tots = [], []
        t0 = time.perf_counter()
        for _ in range(5):
            a = time.perf_counter()
            st = core.analyze_var(w.vp, slab)
            walls.append((time.perf_counter() - a) * 1e3)
            tots.append(st.ms_total)
        torch.cuda.synchronize()
        step = (time.perf_counter() - t0) / 5 * 1e3
        core.finalize()
        print(f"W={world} {name:9s} rep {rep}: {step:6.2f} ms/step  call wall "
              f"{sum(walls) / 5:6.2f}  ms_total {sum(tots) / 5:6.2f}  solve {st.ms_solve:6.2f}",
              flush=True)
