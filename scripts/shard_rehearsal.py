# Rank 0's share of the C2 grid at world sizes 1, 2, 4, 8 (the reference's cyclic column
# grid), timed alone on one
# GPU: the per-rank step time the strong-scaling bench will see, without the collectives.
import sys, time
sys.path.insert(0, "cwbnwp-letkf_amd")
import numpy as np
import torch
from cwbl import abi, synth
from cwbl import dist as cdist

dev = torch.device("cuda", 0)
base = None
for world in [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]:
    w = synth.make("c2", shard=(0, world) if world > 1 else None)
    types = [dict(family=1, type_id=w.radar_type, xyz=w.obs_xyz, obs=w.obs, hdxb=w.hdxb)]
    _, types = cdist.unpack_obs_set(torch.from_numpy(cdist.pack_obs_set(types, w.k)).to(dev))
    x, y, alt = (torch.from_numpy(a).to(dev) for a in (w.x, w.y, w.alt))
    var = torch.from_numpy(w.var).to(dev)
    core = abi.Core(w.k, device=0)
    core.set_obs(cdist.builder_from(types, abi.MEM_DEVICE).build())
    slab = abi.make_slab(x, y, alt, var, memory=abi.MEM_DEVICE)
    core.analyze_var(w.vp, slab)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sts = [core.analyze_var(w.vp, slab) for _ in range(3)]
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 3 * 1e3
    if base is None:
        base = ms * world
    st = sts[-1]
    print(f"world {world}: rank-0 share {st.points} points, {ms:.1f} ms/step "
          f"(ideal {base / world:.1f}), efficiency {base / world / ms:.2f}; "
          f"solve {st.ms_solve:.1f} search {st.ms_search:.1f} prep {st.ms_prep:.1f} total {st.ms_total:.1f}",
          flush=True)
    del core, var, x, y, alt, slab
    torch.cuda.empty_cache()
