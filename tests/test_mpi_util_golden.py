"""The member <-> column transposes pinned against the reference's own module_mpi_util.

tests/golden/mpi_util_n<nproc>_k<k>.npz hold what the reference's letkf_local_info,
letkf_scatter_grid, letkf_gather_grid, letkf_scatter_vcoord and letkf_scatter_hcoord
(module_mpi_util.f90:71-580, compiled from /root/reference with amdflang and run under MPICH's
mpirun by oracle/gen_mpi_util_goldens.py) produced on every rank.  Checked bit for bit:
  - the oracle restatement (oracle/mpi_util_oracle.py), which the GPU kernels are tested
    against, on every array of every rank;
  - the whole Transposer (cwbl/transpose.py) over nproc gloo ranks with the oracle's packing
    (the GPU packing kernels against the same fixtures: tests/test_gpu_transpose.py).
"""
import glob
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cwbl import transpose as tr

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import mpi_util_oracle as mo  # noqa: E402
from test_transpose import OracleCore, _free_port  # noqa: E402

FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "mpi_util_n*_k*.npz")))


def load(path):
    g = dict(np.load(path))
    nproc, k, nx, ny, nz = (int(v) for v in g["meta"])
    return g, nproc, k, nx, ny, nz


def test_fixtures_present():
    assert len(FIXTURES) >= 4


@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_oracle_matches_reference_mpi_util(path):
    g, nproc, k, nx, ny, nz = load(path)
    assert tr.dims_create(nproc) == mo.dims_create(nproc)
    info = mo.local_info(nx, ny, nproc)
    for r in range(nproc):
        for key in ("xloc", "yloc", "xloc_u", "yloc_v"):
            np.testing.assert_array_equal(info[r][key] + 1, g[f"r{r}_{key}"])
        # the Transposer's Decomposition deals the same columns
        d = tr.Decomposition(nx, ny, nproc)
        for st in (0, 1, 2):
            xs, ys = d.columns(r, st)
            lx, ly = d.local_shape(r, st)
            xk = "xloc_u" if st == 1 else "xloc"
            yk = "yloc_v" if st == 2 else "yloc"
            np.testing.assert_array_equal(xs + 1, g[f"r{r}_{xk}"])
            np.testing.assert_array_equal(ys + 1, g[f"r{r}_{yk}"])
            assert (lx, ly) == (len(xs), len(ys))
    for st in (0, 1, 2):
        members = [g[f"r{m}_s{st}_in"] for m in range(k)]     # member m is read by rank m
        want = mo.scatter_grid(members, nproc, st)
        for r in range(nproc):
            np.testing.assert_array_equal(want[r].view(np.uint32),
                                          g[f"r{r}_s{st}_local"].view(np.uint32))
        back = mo.gather_grid([np.float32(2.0) * g[f"r{r}_s{st}_local"] for r in range(nproc)],
                              nx, ny, st)
        for m in range(k):
            np.testing.assert_array_equal(back[m].view(np.uint32),
                                          g[f"r{m}_s{st}_back"].view(np.uint32))
        # the packed layout of one member is the ranks' chunks in rank order (sdispls)
        px, py = mo.dims_create(nproc)
        for m in range(k):
            chunks = np.concatenate([g[f"r{r}_s{st}_local"][m].ravel() for r in range(nproc)])
            np.testing.assert_array_equal(mo.pack_columns(members[m], px, py), chunks)
    for tag, stagger, nzp in (("v0", 0, nz + 1), ("v1", 1, nz)):
        ph = [g[f"r{m}_{tag}_in"] for m in range(k)]
        tmp4d = mo.scatter_grid(ph, nproc, 0)
        for r in range(nproc):
            want = g[f"r{r}_{tag}_out"]
            mkl = mo.mkl_sgemv_mean(tmp4d[r], stagger)
            if mkl is not None:   # the reference's sgemv is MKL's here
                np.testing.assert_array_equal(mkl.view(np.uint32), want.view(np.uint32))
            np.testing.assert_array_equal(mo.vcoord_mean(tmp4d[r], stagger).view(np.uint32),
                                          want.view(np.uint32))
    hgt = mo.scatter_grid([g["r0_vm1_in"]], nproc, 0)    # root's HGT
    for r in range(nproc):
        np.testing.assert_array_equal(hgt[r][0], g[f"r{r}_vm1_out"])
    for st in (0, 1, 2):
        for key, lkey in (("lat", "llat"), ("lon", "llon")):
            loc = mo.scatter_grid([g[f"r0_h{st}_{key}"][None]], nproc, st)   # root's field
            for r in range(nproc):
                np.testing.assert_array_equal(loc[r][0, 0], g[f"r{r}_h{st}_{lkey}"])


def _worker(rank, world, port, path, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g, nproc, k, nx, ny, nz = load(path)
    t = tr.Transposer(OracleCore(), k, nx, ny, device=torch.device("cpu"))
    res = {}
    for st in (0, 1, 2):
        own = {m: torch.from_numpy(g[f"r{m}_s{st}_in"].copy()) for m in t.owned()}
        var = t.scatter_grid(own, nz, st)
        res[f"s{st}_local"] = var.numpy().copy()
        back = t.gather_grid(var * 2.0, st)
        for m in t.owned():
            res[f"s{st}_back{m}"] = back[m].numpy().copy()
    for tag, stagger in (("v0", 0), ("v1", 1)):
        own = {m: torch.from_numpy(g[f"r{m}_{tag}_in"].copy()) for m in t.owned()}
        res[f"{tag}_out"] = t.scatter_vcoord(own, nz, stagger).numpy().copy()
    hgt = torch.from_numpy(g["r0_vm1_in"].copy()) if rank == 0 else None
    res["vm1_out"] = t.scatter_vcoord(hgt, 1, -1).numpy().copy()
    for st in (0, 1, 2):
        lat = torch.from_numpy(g[f"r0_h{st}_lat"].copy()) if rank == 0 else None
        lon = torch.from_numpy(g[f"r0_h{st}_lon"].copy()) if rank == 0 else None
        la, lo = t.scatter_hcoord(lat, lon, st)
        res[f"h{st}_llat"], res[f"h{st}_llon"] = la.numpy().copy(), lo.numpy().copy()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("path", [p for p in FIXTURES if "n8_k8" not in p], ids=os.path.basename)
def test_transposer_over_gloo_matches_reference(tmp_path, path):
    """The Transposer at world = nproc (member m on rank m, as the reference reads member
    files): every rank's slab, gathered members, vertical coordinate and lat/lon equal the
    reference's.  The vcoord mean is the oracle's reference-BLAS order, equal to MKL's sgemv
    on these fixtures (checked above)."""
    g, nproc, k, nx, ny, nz = load(path)
    mp.spawn(_worker, args=(nproc, _free_port(), path, str(tmp_path)), nprocs=nproc, join=True)
    for r in range(nproc):
        got = dict(np.load(tmp_path / f"rank{r}.npz"))
        for st in (0, 1, 2):
            np.testing.assert_array_equal(got[f"s{st}_local"], g[f"r{r}_s{st}_local"])
            if r < k:
                np.testing.assert_array_equal(got[f"s{st}_back{r}"], g[f"r{r}_s{st}_back"])
        for tag in ("v0", "v1", "vm1"):
            np.testing.assert_array_equal(got[f"{tag}_out"], g[f"r{r}_{tag}_out"])
        for st in (0, 1, 2):
            for key in ("llat", "llon"):
                np.testing.assert_array_equal(got[f"h{st}_{key}"], g[f"r{r}_h{st}_{key}"])
