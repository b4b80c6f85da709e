# Per-call host overhead of cwbl_analyze_var at the 8-rank share (rank 0's columns of C2):
# wall time of each call against the library's own ms_total (which starts after the
# ordering synchronisation), and the cost of an idle hipDeviceSynchronize.
import ctypes as C
import sys
import time
sys.path.insert(0, "cwbnwp-letkf_amd")
import torch
from cwbl import abi, synth
from cwbl import dist as cdist

dev = torch.device("cuda", 0)
w = synth.make("c2", shard=(0, 8))
types = [dict(family=1, type_id=w.radar_type, xyz=w.obs_xyz, obs=w.obs, hdxb=w.hdxb)]
_, types = cdist.unpack_obs_set(torch.from_numpy(cdist.pack_obs_set(types, w.k)).to(dev))
x, y, alt = (torch.from_numpy(a).to(dev) for a in (w.x, w.y, w.alt))
var = torch.from_numpy(w.var).to(dev)
core = abi.Core(w.k, device=0)
core.set_obs(cdist.builder_from(types, abi.MEM_DEVICE).build())
slab = abi.make_slab(x, y, alt, var, memory=abi.MEM_DEVICE)
core.analyze_var(w.vp, slab)
torch.cuda.synchronize()
hip = C.CDLL("libamdhip64.so")
t0 = time.perf_counter()
for _ in range(100):
    hip.hipDeviceSynchronize()
print("idle hipDeviceSynchronize: %.1f us" % ((time.perf_counter() - t0) / 100 * 1e6))
for _ in range(5):
    t0 = time.perf_counter()
    st = core.analyze_var(w.vp, slab)
    wall = (time.perf_counter() - t0) * 1e3
    print("wall %.2f ms  ms_total %.2f  solve %.2f  search %.2f  prep %.2f" %
          (wall, st.ms_total, st.ms_solve, st.ms_search, st.ms_prep))
