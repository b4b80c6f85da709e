# debug: NaN census + run-to-run determinism of the 256-thread kernel on the c4 block case
import sys, os
sys.path.insert(0, "cwbnwp-letkf_amd"); sys.path.insert(0, "tests")
import numpy as np
from cwbl import abi, synth
for k in [int(a) for a in sys.argv[1:]]:
    w = synth.make("c4", scale=0.1, k=k)
    c = abi.Core(w.k, device=0)
    c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
    outs = []
    for rep in range(3):
        var = w.var.copy()
        st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
        outs.append(var)
        bad = ~np.isfinite(var)
        pts = np.argwhere(bad.any(axis=0))
        print(k, rep, "nan points", len(pts), pts[:4].tolist(), flush=True)
    for rep in (1, 2):
        d = (outs[rep].view(np.uint32) != outs[0].view(np.uint32)).any(axis=0)
        print(k, "points differing run 0 vs", rep, int(d.sum()), flush=True)
