# C2 grid at other ensemble sizes: ms per variable on one GPU (device-resident slab)
import sys
import time
sys.path.insert(0, "cwbnwp-letkf_amd")
import torch
from cwbl import abi, synth

dev = torch.device("cuda", 0)
for k in [int(a) for a in sys.argv[1:]] or [24, 32, 40, 48, 64]:
    w = synth.make("c2", k=k)
    x, y, alt = (torch.from_numpy(a).to(dev) for a in (w.x, w.y, w.alt))
    var = torch.from_numpy(w.var).to(dev)
    core = abi.Core(k, device=0)
    core.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
    slab = abi.make_slab(x, y, alt, var, memory=abi.MEM_DEVICE)
    core.analyze_var(w.vp, slab)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        st = core.analyze_var(w.vp, slab)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 3 * 1e3
    print(f"k={k}: {ms:.1f} ms per variable, {w.points / ms / 1e3:.2f} M pts/s, solved {st.solved}", flush=True)
    core.finalize()
    del var, x, y, alt, slab
    torch.cuda.empty_cache()
