"""Timing ablations of the k = 128 paths on C4: per-kernel ms per launch at each
CWBL_DEBUG_TQ_STOP[:CWBL_DEBUG_TQ_STEPS] setting.  Needs the DEBUG_KNOBS library (`make -C
cwbnwp-letkf_amd debuglib`, loaded with CWBL_LIBRARY=cwbnwp-letkf_amd/lib_dbg/libcwbl.so); the
release library ignores the variables.

  --path 1 (hand-off path; hand-off kernel: 12 column staging only, 1 assembly only, 0:S the
            first S of its 64 steps; tail kernel: 2 its steps only, 3 steps + quadrature,
            2:64+S all hand-off steps and only the tail's first S steps)

  --config c2 (the record path: assembly kernel 11 = staging only (no MFMA groups), 13 =
            without the gathers, 1 = no record write; solve_tq40_kernel 5 = record loads
            only, 4 = + phase 1, 2 = + phase 2, 3 = + quadrature)

Usage: python scripts/c4_ablate.py [--config c2|c4] [--path N] [stop[:steps] ...]"""
import json
import os
import sys
import time

sys.path.insert(0, "cwbnwp-letkf_amd")
import torch  # noqa: E402

from cwbl import abi, dist as cdist, synth  # noqa: E402

args = sys.argv[1:]
path, config = 1, "c4"
while args[:1] in (["--path"], ["--config"]):
    if args[0] == "--path":
        path = int(args[1])
    else:
        config = args[1]
    args = args[2:]
specs = args or (["0", "12", "1", "0:16", "0:32", "0:48", "2", "3"] if config == "c4" else
                 ["0", "11", "13", "1", "5", "4", "2", "3"])
w = synth.make(config, local_noise=True)
dev = torch.device("cuda:0")
types = [dict(family=1, type_id=w.radar_type, xyz=w.obs_xyz, obs=w.obs, hdxb=w.hdxb)]
_, types = cdist.unpack_obs_set(torch.from_numpy(cdist.pack_obs_set(types, w.k)).to(dev))
x, y, alt = (torch.from_numpy(a).to(dev) for a in (w.x, w.y, w.alt))
var0 = torch.from_numpy(w.var).to(dev)
core = abi.Core(w.k, device=0, options={"big_path": path} if w.k > 64 else {})
core.set_obs(cdist.builder_from(types, abi.MEM_DEVICE).build())
var = var0.clone()
slab = abi.make_slab(x, y, alt, var, memory=abi.MEM_DEVICE)
for spec in specs:
    stop, _, steps = spec.partition(":")
    os.environ["CWBL_DEBUG_TQ_STOP"] = stop
    os.environ["CWBL_DEBUG_TQ_STEPS"] = steps or "0"
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
    print(spec, json.dumps({"ms_per_var": round(el * 1e3, 1),
                            "kernels": {k: round(v["ms"] / max(v["launches"], 1), 3)
                                        for k, v in kt.items() if "search" not in k}}), flush=True)
core.finalize()
