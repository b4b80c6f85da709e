"""The sharded path with the HIP core in every rank (world size 2, one GPU, gloo transport).

What bench.py --gpus N and the reference's flat-MPI layout do (module_mpi_util.f90:38-56,
73-188): grid columns dealt over a px x py cyclic block-1 rank grid, the obs set packed on
rank 0 and broadcast once (cwbl/dist.py broadcast_obs_set, the device buffer of the wire
format) and handed to the core as DEVICE memory (builder_from(MEM_DEVICE)), each rank
analysing its own columns with cwbl_analyze_var.  Both ranks share cuda:0 (RCCL refuses two
ranks per device; gloo carries the broadcast of the device buffer).  The reassembled output
must equal the single-process HIP analysis of the whole grid bit for bit, and the oracle
within the north_star tolerance.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cwbl import abi, synth
from cwbl import dist as cdist
from helpers import increment_rel_rms, oracle

pytestmark = pytest.mark.gpu

INCR_TOL = 1e-6
CASE = dict(name="c2", seed=23, scale=0.1, nz=10)  # 30 x 30 x 10, k = 40


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir, case=CASE, workspace=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    c = dict(case)
    w = synth.make(c.pop("name"), shard=(rank, world), **c)
    types = None
    if rank == 0:
        types = [dict(family=1, type_id=w.radar_type, xyz=w.obs_xyz, obs=w.obs, hdxb=w.hdxb)]
    k, got = cdist.broadcast_obs_set(types, w.k, dev, src=0)
    assert k == w.k and got[0]["xyz"].is_cuda
    core = abi.Core(k, device=0, workspace_bytes=workspace)
    core.set_obs(cdist.builder_from(got, abi.MEM_DEVICE).build())
    x, y, alt, var = (torch.from_numpy(a).to(dev) for a in (w.x, w.y, w.alt, w.var))
    st = core.analyze_var(w.vp, abi.make_slab(x, y, alt, var, memory=abi.MEM_DEVICE))
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), var.cpu().numpy())
    np.save(os.path.join(out_dir, f"stats{rank}.npy"),
            np.array([st.points, st.solved, st.nobs_sum, st.nonconverged], np.int64))
    core.finalize()
    dist.barrier()
    dist.destroy_process_group()


def _sharded_run_equals_single_process_and_oracle(tmp_path, world, case, workspace=0,
                                                  block=None):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), case, workspace), nprocs=world,
             join=True)
    c = dict(case)
    full = synth.make(c.pop("name"), **c)
    # the single-process HIP analysis of the whole grid (host-memory slab)
    core = abi.Core(full.k, device=0)
    core.set_obs(abi.ObsSetBuilder().add_radar(full.radar_type, full.obs_xyz, full.obs,
                                               full.hdxb).build())
    one = full.var.copy()
    st1 = core.analyze_var(full.vp, abi.make_slab(full.x, full.y, full.alt, one))
    core.finalize()
    got = np.empty_like(one)
    seen = np.zeros(one.shape[2:], np.int32)
    tot = np.zeros(4, np.int64)
    for r in range(world):
        xs, ys = cdist.shard_columns(full.nx, full.ny, r, world)
        got[:, :, ys[:, None], xs[None, :]] = np.load(tmp_path / f"rank{r}.npy")
        seen[ys[:, None], xs[None, :]] += 1
        tot += np.load(tmp_path / f"stats{r}.npy")
    assert (seen == 1).all()
    assert tot[0] == st1.points and tot[1] == st1.solved and tot[2] == st1.nobs_sum
    assert tot[3] == 0 and st1.solved > 0
    np.testing.assert_array_equal(got.view(np.uint32), one.view(np.uint32))
    # the oracle on the whole grid, or on a block of whole columns (ny0, nx0, nb) of it
    j0, i0, nb = block if block else (0, 0, None)
    cut = (lambda a: np.ascontiguousarray(a[..., j0:j0 + nb, i0:i0 + nb])) if nb else \
        (lambda a: a)  # noqa: E731
    ref = cut(full.var).copy()
    ob = abi.ObsSetBuilder().add_radar(full.radar_type, full.obs_xyz, full.obs, full.hdxb).build()
    rc = oracle().orc_analyze_var(full.k, 0, -5.0, 0, C.byref(ob), C.byref(full.vp),
                                  C.byref(abi.make_slab(cut(full.x), cut(full.y), cut(full.alt),
                                                        ref)), 16, C.byref(abi.Stats()))
    assert rc == 0
    rel = increment_rel_rms(cut(got), ref, cut(full.var))
    assert rel <= INCR_TOL, rel


def test_two_ranks_hip_core_equals_single_process_and_oracle(tmp_path):
    _sharded_run_equals_single_process_and_oracle(tmp_path, 2, CASE)


def test_c3_eight_ranks_full_c2_grid(tmp_path):
    """configs[2] (C3): the full 300 x 300 x 50 C2 grid (k = 40, 22 500 obs) dealt over 8
    ranks (px x py = 4 x 2, 75 x 150 columns each), the obs set broadcast once from rank 0
    and each rank's HIP core analysing its 562 500 points.  All 8 ranks share cuda:0 over
    gloo here (RCCL refuses two ranks per device; the driver's 8-GPU bench runs the same code
    over RCCL), each with a 512 MiB list workspace.  The reassembled grid must equal the
    single-process analysis bit for bit, and the oracle on a 12 x 12-column block within
    1e-6."""
    _sharded_run_equals_single_process_and_oracle(
        tmp_path, 8, dict(name="c2"), workspace=512 << 20, block=(144, 144, 12))


@pytest.mark.timeout(900)
def test_bench_two_ranks_end_to_end():
    """`bench.py --gpus 2` end to end, as the driver's scaling run starts it (the script launches
    its own ranks under torch.distributed.run), with both ranks on this GPU over gloo: the
    obs-set broadcast, the sharded analysis, the member<->column transposes and the 16-variable
    cycle with write_mean, ending in one JSON line whose n_gpus counts distinct devices."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CWBL_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--no-cpu-baseline", "--no-detail-configs"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=850)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["n_gpus"] == 1 and d["config"]["ranks"] == 2 and d["value"] > 0
    t = d["detail"]["transposes"]
    assert t["scatter_ms"] > 0 and t["gather_ms"] > 0
    cy = d["detail"]["cycle"]
    assert cy["transposes"] is True and cy["variables"] == 16 and cy["write_mean_ms"] > 0
