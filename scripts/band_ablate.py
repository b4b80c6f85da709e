"""Timing ablations of the two-stage k = 128 band path on C4: per-kernel ms per launch at each
CWBL_DEBUG_TQ_STOP (head: 1 assembly only, 5 without the panel QRs, 6 the QRs without the
trailing updates; tail: 2 the chase only, 3 chase + quadrature).  Needs a library built with
`make DEBUG_KNOBS=1` (the release library ignores the variable), e.g. built in a copy of the
tree and passed as CWBL_LIBRARY=<copy>/cwbnwp-letkf_amd/lib/libcwbl.so.

Usage: python scripts/band_ablate.py [stops...]"""
import json
import os
import sys
import time

sys.path.insert(0, "cwbnwp-letkf_amd")
import torch  # noqa: E402

from cwbl import abi, dist as cdist, synth  # noqa: E402

stops = [int(a) for a in sys.argv[1:]] or [0, 1, 5, 6, 2, 3]
w = synth.make("c4", local_noise=True)
dev = torch.device("cuda:0")
types = [dict(family=1, type_id=w.radar_type, xyz=w.obs_xyz, obs=w.obs, hdxb=w.hdxb)]
_, types = cdist.unpack_obs_set(torch.from_numpy(cdist.pack_obs_set(types, w.k)).to(dev))
x, y, alt = (torch.from_numpy(a).to(dev) for a in (w.x, w.y, w.alt))
var0 = torch.from_numpy(w.var).to(dev)
core = abi.Core(w.k, device=0, options={"big_path": 2})
core.set_obs(cdist.builder_from(types, abi.MEM_DEVICE).build())
var = var0.clone()
slab = abi.make_slab(x, y, alt, var, memory=abi.MEM_DEVICE)
for stop in stops:
    os.environ["CWBL_DEBUG_TQ_STOP"] = str(stop)
    var.copy_(var0)
    core.analyze_var(w.vp, slab)
    core.set_kernel_timing(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    var.copy_(var0)
    core.analyze_var(w.vp, slab)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kt = core.kernel_times()
    core.set_kernel_timing(False)
    print(stop, json.dumps({"ms_per_var": round(el * 1e3, 1),
                            "kernels": {k: round(v["ms"] / max(v["launches"], 1), 3)
                                        for k, v in kt.items() if "band" in k}}), flush=True)
core.finalize()
