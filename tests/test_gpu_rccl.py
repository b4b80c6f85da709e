"""RCCL on the one-GPU lease: a world-1 "nccl" process group running the multi-GPU code paths.

RCCL refuses two ranks on one device, so the multi-rank tests carry their messages over gloo.
A world-1 nccl group is legal and executes the same RCCL calls the 8-GPU run makes
(cwbl/dist.py, cwbl/transpose.py):
  - init with device_id (eager communicator creation, as bench.py does);
  - the obs-set exchange as ONE broadcast of a device buffer (the counts every rank knows,
    wire_layout), handed to cwbl_set_obs(MEM_DEVICE) and cwbl_analyze_var with no
    synchronisation in between: the library must order itself after the collective's stream
    work (cwbl_set_stream / null-stream semantics, include/cwb_letkf_core.h:36-41);
  - the member <-> column transposes with loopback=True: every chunk, the rank's own
    included, goes through batch_isend_irecv (grouped ncclSend/ncclRecv to itself);
  - write_mean's reduce, scatter_vcoord / scatter_hcoord through the same transport.
Replaces module_gts_omboma.f90:532-605 (ibcast chain), module_mpi_util.f90:262,325
(alltoallv), module_grid.f90:744-821 (mpi_reduce per field).

Every result must equal the single-process analysis of the same case (host-memory slab, no
process group) bit for bit, and the transposes the oracle's (oracle/mpi_util_oracle.py).
The RCCL work runs in a child process (torch.multiprocessing spawn) so the test process
never holds a process group.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cwbl import abi, synth
from cwbl import dist as cdist
from cwbl import transpose as tr
from test_transpose import check_plan, run_plan

pytestmark = pytest.mark.gpu

CASE = dict(name="c2", seed=23, scale=0.1, nz=10)  # 30 x 30 x 10, k = 40


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rccl_worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    res = {}

    # ---- the obs set: one broadcast of the wire buffer, counted --------------------------
    c = dict(CASE)
    w = synth.make(c.pop("name"), **c)
    types = [dict(family=1, type_id=w.radar_type, xyz=w.obs_xyz, obs=w.obs, hdxb=w.hdxb)]
    calls = []
    real_bcast = dist.broadcast

    def counting(*a, **kw):
        calls.append(a[0].numel())
        return real_bcast(*a, **kw)

    dist.broadcast = counting
    try:
        k, got = cdist.broadcast_obs_set(types, w.k, dev, src=0,
                                         layout=cdist.wire_layout(types))
    finally:
        dist.broadcast = real_bcast
    res["bcast_calls"] = np.array(calls, np.int64)
    assert k == w.k and got[0]["xyz"].is_cuda
    core = abi.Core(k, device=0)
    # no synchronize: the broadcast is queued on RCCL's stream, set_obs must wait for it
    core.set_obs(cdist.builder_from(got, abi.MEM_DEVICE).build())
    x, y, alt = (torch.from_numpy(a).to(dev) for a in (w.x, w.y, w.alt))

    # ---- member fields -> column slab over RCCL self-sends -> analysis -> back ------------
    t = tr.Transposer(core, k, w.nx, w.ny, device=dev, loopback=True)
    assert t.world == 1 and t.backend == "nccl"
    members = {m: torch.from_numpy(np.ascontiguousarray(w.var[m])).to(dev) for m in range(k)}
    var = t.scatter_grid(members, w.nz)
    assert all(var.data_ptr() != f.data_ptr() for f in members.values())
    res["scattered"] = var.cpu().numpy()
    st = core.analyze_var(w.vp, abi.make_slab(x, y, alt, var, memory=abi.MEM_DEVICE))
    res["stats"] = np.array([st.points, st.solved, st.nobs_sum, st.nonconverged], np.int64)
    out = {m: torch.full_like(members[m], float("nan")) for m in range(k)}
    t.gather_grid(var, out=out)
    res["gathered"] = torch.stack([out[m] for m in range(k)]).cpu().numpy()

    # ---- write_mean: member sums on the device, one RCCL reduce, the root's scale ---------
    mean = t.write_mean({m: [out[m], out[m][0]] for m in range(k)})
    res["mean3d"], res["mean2d"] = mean[0].cpu().numpy(), mean[1].cpu().numpy()

    core.finalize()  # (the library state is per process: one Core at a time)

    # ---- the whole transpose plan (U/V staggers, vcoord, hcoord) against the oracle -------
    t8 = tr.Transposer(abi.Core(8, device=0), 8, 7, 5, device=dev, loopback=True)
    run_plan(t8, 8, 7, 5, 3, out_dir, 0)
    t8.core.finalize()
    np.savez(os.path.join(out_dir, "rccl.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_world1_broadcast_transposes_reduce(tmp_path):
    mp.spawn(_rccl_worker, args=(_free_port(), str(tmp_path)), nprocs=1, join=True)
    got = dict(np.load(tmp_path / "rccl.npz"))
    c = dict(CASE)
    w = synth.make(c.pop("name"), **c)
    types = [dict(family=1, type_id=w.radar_type, xyz=w.obs_xyz, obs=w.obs, hdxb=w.hdxb)]
    # one collective for the whole set, of the wire buffer's size
    assert got["bcast_calls"].tolist() == [cdist.wire_words(cdist.wire_layout(types), w.k)]
    # one rank owns every column: the slab is the stacked member fields
    np.testing.assert_array_equal(got["scattered"].view(np.uint32), w.var.view(np.uint32))
    # the single-process analysis of the same case from host memory, no process group
    core = abi.Core(w.k, device=0)
    core.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
    one = w.var.copy()
    st = core.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, one))
    core.finalize()
    assert got["stats"].tolist() == [st.points, st.solved, st.nobs_sum, 0] and st.solved > 0
    np.testing.assert_array_equal(got["gathered"].view(np.uint32), one.view(np.uint32))
    inv = np.float32(1.0) / np.float32(w.k)
    acc = np.zeros_like(one[0])
    for m in range(w.k):
        acc = acc + one[m]
    np.testing.assert_array_equal(got["mean3d"].view(np.uint32), (inv * acc).view(np.uint32))
    np.testing.assert_array_equal(got["mean2d"].view(np.uint32), (inv * acc[0]).view(np.uint32))
    check_plan(str(tmp_path), 1, 8, 7, 5, 3)
