"""CPU checks of the member <-> column transposes (cwbl/transpose.py):
the decomposition against MPICH's MPI_Dims_create (G6) and the reference's letkf_local_info
loops (oracle/mpi_util_oracle.py), and the exchange plan over gloo with world sizes 2 and 3.

On CPU the HIP packing kernels are unavailable, so the gloo tests hand the Transposer a
stand-in `core` whose pack/unpack/mean are the oracle's (test-only injection; the product
Transposer takes the real cwbl.abi.Core, whose init fails without a GPU).  The same plan with
the real kernels runs in tests/test_gpu_transpose.py."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cwbl import transpose as tr

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import mpi_util_oracle as mo  # noqa: E402


def test_dims_create_matches_mpich():
    with open(os.path.join(HERE, "golden", "dims_create.json")) as f:
        g = json.load(f)["dims"]
    for n, d in g.items():
        assert list(tr.dims_create(int(n))) == d, n
        assert list(mo.dims_create(int(n))) == d, n


@pytest.mark.parametrize("nx,ny,world", [(10, 7, 1), (10, 7, 2), (9, 11, 4), (5, 3, 8),
                                         (300, 300, 8), (2, 2, 6)])
def test_decomposition_matches_local_info(nx, ny, world):
    dec = tr.Decomposition(nx, ny, world)
    for r, info in enumerate(mo.local_info(nx, ny, world)):
        for st, (xk, yk) in ((0, ("xloc", "yloc")), (1, ("xloc_u", "yloc")),
                             (2, ("xloc", "yloc_v"))):
            xl, yl = dec.columns(r, st)
            np.testing.assert_array_equal(xl, info[xk])
            np.testing.assert_array_equal(yl, info[yk])
            assert dec.local_shape(r, st) == (len(info[xk]), len(info[yk]))
    # every column exactly once
    for st in (0, 1, 2):
        gx, gy = dec.grid(st)
        assert sum(a * b for a, b in (dec.local_shape(r, st) for r in range(world))) == gx * gy
        offs = dec.chunks(3, st)
        assert offs[-1][0] + offs[-1][1] == gx * gy * 3


def test_oracle_pack_is_scatter_order():
    rng = np.random.default_rng(3)
    nz, ny, nx, world = 3, 7, 10, 6
    f = rng.normal(size=(nz, ny, nx)).astype(np.float32)
    px, py = mo.dims_create(world)
    packed = mo.pack_columns(f, px, py)
    per_rank = mo.scatter_grid([f], world)
    np.testing.assert_array_equal(packed, np.concatenate([v[0].ravel() for v in per_rank]))
    np.testing.assert_array_equal(mo.unpack_columns(packed, nz, ny, nx, px, py), f)


class OracleCore:
    """Test stand-in for cwbl.abi.Core's transpose entry points (CPU tensors)."""

    def pack_columns(self, g, nx, ny, nz, px, py, send):
        send.copy_(torch.from_numpy(mo.pack_columns(g.numpy().reshape(nz, ny, nx), px, py)))

    def unpack_columns(self, recv, nx, ny, nz, px, py, g):
        g.copy_(torch.from_numpy(mo.unpack_columns(recv.numpy(), nz, ny, nx, px, py)))

    def pack_members(self, g, gstride, nm, nx, ny, nz, px, py, send, sstride):
        n = nx * ny * nz
        src = torch.as_strided(g, (nm, n), (gstride, 1))
        dst = torch.as_strided(send, (nm, n), (sstride, 1))
        for i in range(nm):
            dst[i].copy_(torch.from_numpy(mo.pack_columns(src[i].numpy().reshape(nz, ny, nx), px, py)))

    def unpack_members(self, recv, rstride, nm, nx, ny, nz, px, py, g, gstride):
        n = nx * ny * nz
        src = torch.as_strided(recv, (nm, n), (rstride, 1))
        dst = torch.as_strided(g, (nm, n), (gstride, 1))
        for i in range(nm):
            dst[i].copy_(torch.from_numpy(mo.unpack_columns(src[i].numpy(), nz, ny, nx, px, py).ravel()))

    def vcoord_mean(self, ph, n2d, nz_ph, k, stagger, gconst, alt):
        alt.copy_(torch.from_numpy(mo.vcoord_mean(ph.numpy(), stagger, np.float32(gconst))))

    def member_sum(self, fields, n, nm, out):
        acc = np.zeros(n, np.float32)
        for m in range(nm):  # fp32, member order (cwbl_member_sum)
            acc = acc + fields[m].numpy()
        out.copy_(torch.from_numpy(acc))

    def scale(self, x, n, alpha):
        x.copy_(torch.from_numpy(np.float32(alpha) * x.numpy()))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def fields_for(k, nz, gy, gx, seed):
    rng = np.random.default_rng(seed)
    return [rng.normal(size=(nz, gy, gx)).astype(np.float32) for _ in range(k)]


def run_plan(t, k, nx, ny, nz, out_dir, rank):
    """Scatter (mass, U, V grids), gather, vcoord (0, 1, -1) and hcoord; save per rank."""
    res = {}
    for st in (0, 1, 2):
        gx, gy = t.dec.grid(st)
        members = fields_for(k, nz, gy, gx, 10 + st)
        if st == 0:  # the owned members as views of one stacked tensor (one-launch packing)
            stk = torch.from_numpy(np.stack([members[m] for m in t.owned()])).to(t.device)
            own = {m: stk[i] for i, m in enumerate(t.owned())}
        else:
            own = {m: torch.from_numpy(members[m]).to(t.device) for m in t.owned()}
        var = t.scatter_grid(own, nz, st)
        res[f"var{st}"] = var.cpu().numpy()
        back = t.gather_grid(var * 2.0, st)
        for m in t.owned():
            res[f"back{st}_{m}"] = back[m].cpu().numpy()
    ph = fields_for(k, nz + 1, ny, nx, 30)
    own = {m: torch.from_numpy(ph[m]).to(t.device) for m in t.owned()}
    res["alt0"] = t.scatter_vcoord(own, nz, 0).cpu().numpy()
    own1 = {m: torch.from_numpy(ph[m][:nz].copy()).to(t.device) for m in t.owned()}
    res["alt1"] = t.scatter_vcoord(own1, nz, 1).cpu().numpy()
    hgt = torch.from_numpy(ph[0][:1].copy()).to(t.device) if rank == 0 else None
    res["altm1"] = t.scatter_vcoord(hgt, 1, -1).cpu().numpy()
    ll = fields_for(2, 1, ny, nx + 1, 40)   # U-grid lat/lon (stagger 1)
    lat = torch.from_numpy(ll[0][0].copy()).to(t.device) if rank == 0 else None
    lon = torch.from_numpy(ll[1][0].copy()).to(t.device) if rank == 0 else None
    la, lo = t.scatter_hcoord(lat, lon, 1)
    res["lat"], res["lon"] = la.cpu().numpy(), lo.cpu().numpy()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)


def check_plan(out_dir, world, k, nx, ny, nz):
    res = [dict(np.load(os.path.join(out_dir, f"rank{r}.npz"))) for r in range(world)]
    for st in (0, 1, 2):
        gx, gy = nx + (st == 1), ny + (st == 2)
        members = fields_for(k, nz, gy, gx, 10 + st)
        want = mo.scatter_grid(members, world, st)
        for r in range(world):
            np.testing.assert_array_equal(res[r][f"var{st}"], want[r])
            for m in range(r, k, world):
                np.testing.assert_array_equal(res[r][f"back{st}_{m}"], members[m] * 2.0)
    ph = fields_for(k, nz + 1, ny, nx, 30)
    tmp0 = mo.scatter_grid(ph, world, 0)
    tmp1 = mo.scatter_grid([p[:nz] for p in ph], world, 0)
    hg = mo.scatter_grid([ph[0][:1]], world, 0)
    ll = fields_for(2, 1, ny, nx + 1, 40)
    lat = mo.scatter_grid([ll[0]], world, 1)
    lon = mo.scatter_grid([ll[1]], world, 1)
    for r in range(world):
        np.testing.assert_array_equal(res[r]["alt0"], mo.vcoord_mean(tmp0[r], 0))
        np.testing.assert_array_equal(res[r]["alt1"], mo.vcoord_mean(tmp1[r], 1))
        np.testing.assert_array_equal(res[r]["altm1"], hg[r][0])
        np.testing.assert_array_equal(res[r]["lat"], lat[r][0, 0])
        np.testing.assert_array_equal(res[r]["lon"], lon[r][0, 0])


def _worker(rank, world, port, out_dir, k, nx, ny, nz, loopback=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = tr.Transposer(OracleCore(), k, nx, ny, device=torch.device("cpu"), loopback=loopback)
    run_plan(t, k, nx, ny, nz, out_dir, rank)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,k,loopback", [(2, 5, False), (3, 4, False), (1, 3, True),
                                              (2, 5, True)])
def test_transposes_gloo(tmp_path, world, k, loopback):
    """The whole plan over gloo ranks against the oracle.  loopback: a rank's own chunk goes
    through the transport too (the one-GPU RCCL exercise, tests/test_gpu_rccl.py)."""
    nx, ny, nz = 7, 5, 3
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), k, nx, ny, nz, loopback),
             nprocs=world, join=True)
    check_plan(str(tmp_path), world, k, nx, ny, nz)


@pytest.mark.parametrize("k,stagger", [(3, 0), (17, 1), (40, 0), (64, 1)])
def test_oracle_vcoord_mean_matches_mkl_sgemv(k, stagger):
    """Pins the oracle's mean: the reference's sgemv call itself, through MKL in its
    conditional-numerical-reproducibility COMPATIBLE mode, gives the same bits as the
    reference-BLAS order the oracle (and the HIP kernel) evaluates."""
    rng = np.random.default_rng(k)
    shape = (k, 9, 12, 11)
    ph = (np.arange(9, dtype=np.float32)[None, :, None, None] * 3000.0 +
          rng.normal(0, 50, shape)).astype(np.float32)
    mkl = mo.mkl_sgemv_mean(ph, stagger)
    if mkl is None:
        pytest.skip("MKL not available")
    np.testing.assert_array_equal(mo.vcoord_mean(ph, stagger), mkl)


def _mean_fields(k, seed=8):
    """Per member the write_mean field list: 2-D (psfc-like), staggered U-like, 3-D."""
    rng = np.random.default_rng(seed)
    return {m: [rng.normal(size=(7, 10)).astype(np.float32),
                rng.normal(size=(3, 7, 11)).astype(np.float32),
                rng.normal(size=(3, 7, 10)).astype(np.float32) + 280.0] for m in range(k)}


def _mean_worker(rank, world, port, out_dir, k):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = tr.Transposer(OracleCore(), k, 10, 7, device=torch.device("cpu"))
    allf = _mean_fields(k)
    mine = {m: [torch.from_numpy(a.copy()) for a in allf[m]] for m in t.owned()}
    out = t.write_mean(mine, root=0)
    if rank == 0:
        np.savez(os.path.join(out_dir, "mean.npz"), *[o.numpy() for o in out])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,k", [(2, 5), (3, 8)])
def test_write_mean_gloo(tmp_path, world, k):
    """write_mean's ensemble mean (module_grid.f90:700-840) through the Transposer: per-rank
    member sums, one reduce, the root's sscal by nmember_inv.  At 2 ranks the cross-rank sum
    is a single (commutative) add, so the result is bit-exact against the same order in
    numpy; at 3 ranks gloo's reduction order is its own, so the check is fp32 rounding."""
    mp.spawn(_mean_worker, args=(world, _free_port(), str(tmp_path), k), nprocs=world,
             join=True)
    got = np.load(tmp_path / "mean.npz")
    allf = _mean_fields(k)
    inv = np.float32(1.0) / np.float32(k)
    for i in range(3):
        parts = []
        for r in range(world):
            acc = np.zeros_like(allf[0][i])
            for m in range(r, k, world):
                acc = acc + allf[m][i]
            parts.append(acc)
        tot = parts[0]
        for p in parts[1:]:
            tot = tot + p
        exp = inv * tot
        g = got[f"arr_{i}"]
        if world == 2:
            np.testing.assert_array_equal(g.view(np.uint32), exp.view(np.uint32))
        else:
            np.testing.assert_allclose(g, exp, rtol=2e-6, atol=1e-6)
        # and the reference's definition up to fp32 rounding
        ref = np.mean(np.stack([allf[m][i] for m in range(k)]).astype(np.float64), axis=0)
        np.testing.assert_allclose(g, ref, rtol=1e-5, atol=1e-5)


def test_one_rank_transposes_alias_the_stacked_fields():
    """On one rank the column layout is the member layout: scatter_grid returns the stacked
    member tensor itself (no copy) and gather_grid's result is views of var; fields that are
    not one stacked tensor (or an explicit `out`) go through the packing, with the same
    values."""
    k, nx, ny, nz = 3, 6, 5, 4
    t = tr.Transposer(OracleCore(), k, nx, ny, device=torch.device("cpu"))
    assert t.world == 1
    members = fields_for(k, nz, ny, nx, 3)
    stk = torch.from_numpy(np.stack(members))
    own = {m: stk[m] for m in range(k)}
    var = t.scatter_grid(own, nz)
    assert var.data_ptr() == stk.data_ptr() and tuple(var.shape) == (k, nz, ny, nx)
    back = t.gather_grid(var, out=own)
    assert all(back[m].data_ptr() == stk[m].data_ptr() for m in range(k))
    sep = {m: torch.from_numpy(members[m].copy()) for m in range(k)}
    var2 = t.scatter_grid(sep, nz)
    assert var2.data_ptr() not in [f.data_ptr() for f in sep.values()]
    np.testing.assert_array_equal(var2.numpy(), np.stack(members))
    out = {m: torch.zeros((nz, ny, nx)) for m in range(k)}
    t.gather_grid(var2 * 3.0, out=out)
    for m in range(k):
        np.testing.assert_array_equal(out[m].numpy(), members[m] * 3.0)
    views = t.gather_grid(var2)
    assert views[1].data_ptr() == var2[1].data_ptr()
