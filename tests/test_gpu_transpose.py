"""GPU checks of the member <-> column transposes: the HIP packing
kernels and the ensemble-mean kernel against the oracle (oracle/mpi_util_oracle.py), and
the whole Transposer with the real kernels over 2 processes on one GPU (gloo transport)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cwbl import abi
from cwbl import transpose as tr

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import mpi_util_oracle as mo  # noqa: E402
from test_transpose import check_plan, run_plan  # noqa: E402

pytestmark = pytest.mark.gpu

_core = {}


def core(k=8):
    if _core.get("k") != k:
        if "c" in _core:
            _core["c"].finalize()
        _core["c"] = abi.Core(k, device=0)
        _core["k"] = k
    return _core["c"]


@pytest.mark.parametrize("nz,ny,nx,world", [(3, 7, 10, 1), (3, 7, 10, 6), (5, 11, 9, 8),
                                            (2, 3, 5, 8), (4, 33, 65, 12), (50, 300, 301, 8)])
def test_pack_unpack_vs_oracle(nz, ny, nx, world):
    c = core()
    px, py = tr.dims_create(world)
    f = torch.randn((nz, ny, nx), device="cuda", dtype=torch.float32)
    send = torch.full((nz * ny * nx,), float("nan"), device="cuda")
    c.pack_columns(f, nx, ny, nz, px, py, send)
    want = mo.pack_columns(f.cpu().numpy(), px, py)
    np.testing.assert_array_equal(send.cpu().numpy(), want)
    back = torch.full_like(f, float("nan"))
    c.unpack_columns(send, nx, ny, nz, px, py, back)
    assert torch.equal(back, f)


@pytest.mark.parametrize("nz,ny,nx,world,nm,pad", [(3, 7, 12, 6, 5, 0), (5, 11, 9, 8, 3, 7),
                                                     (4, 33, 64, 12, 8, 4), (50, 30, 301, 8, 5, 1),
                                                     (50, 300, 300, 1, 4, 0), (1, 70000, 3, 2, 2, 0),
                                                     (10, 20, 40, 2, 3, 0), (8, 12, 16, 4, 2, 4),
                                                     (6, 9, 20, 1, 3, 2)])
def test_pack_unpack_members_vs_oracle(nz, ny, nx, world, nm, pad):
    """cwbl_pack_members / cwbl_unpack_members: nm member fields in one launch at a member
    stride of n + pad elements (16-B global accesses where nx % 4 == 0 and every member is
    aligned, 4-B otherwise), the rows of a line folded into the grid (ny or nz past 65535),
    against the oracle member by member; lanes never write past a member's n elements."""
    c = core()
    px, py = tr.dims_create(world)
    n = nz * ny * nx
    st = n + pad
    f = torch.randn((nm * st,), device="cuda", dtype=torch.float32)
    send = torch.full((nm * st,), float("nan"), device="cuda")
    c.pack_members(f, st, nm, nx, ny, nz, px, py, send, st)
    got = send.cpu().numpy().reshape(nm, st)
    fh = f.cpu().numpy().reshape(nm, st)
    for i in range(nm):
        np.testing.assert_array_equal(got[i, :n], mo.pack_columns(fh[i, :n].reshape(nz, ny, nx), px, py))
        assert np.isnan(got[i, n:]).all()
    back = torch.full_like(f, float("nan"))
    c.unpack_members(send, st, nm, nx, ny, nz, px, py, back, st)
    b = back.cpu().numpy().reshape(nm, st)
    np.testing.assert_array_equal(b[:, :n], fh[:, :n])
    assert np.isnan(b[:, n:]).all()


@pytest.mark.parametrize("side_stream", [False, True])
def test_device_inputs_only_need_to_be_queued(side_stream):
    """The library's streams are non-blocking; every device-pointer entry point must wait for
    work the caller has merely queued on its stream (a NaN fill queued on torch's
    stream landed after unpack_columns had written its output).  The producer here is held
    back by a GPU spin, on torch's current stream or on a side stream named by
    cwbl_set_stream, and the library is called at once."""
    c = core()
    nz, ny, nx, world = 4, 33, 65, 12
    px, py = tr.dims_create(world)
    g = torch.randn((nz, ny, nx), device="cuda", dtype=torch.float32)
    f = torch.zeros_like(g)
    send = torch.zeros((nz * ny * nx,), device="cuda")
    torch.cuda.synchronize()
    s = torch.cuda.Stream() if side_stream else torch.cuda.current_stream()
    c.set_stream(s)
    with torch.cuda.stream(s):
        torch.cuda._sleep(20_000_000)  # ~10 ms of GPU spin before the input is written
        f.copy_(g)
    c.pack_columns(f, nx, ny, nz, px, py, send)  # no synchronize in between
    np.testing.assert_array_equal(send.cpu().numpy(), mo.pack_columns(g.cpu().numpy(), px, py))
    back = torch.full_like(g, float("nan"))  # queued on torch's stream, after the call above
    with torch.cuda.stream(s):
        torch.cuda._sleep(20_000_000)
        back.fill_(float("nan"))
    c.unpack_columns(send, nx, ny, nz, px, py, back)
    torch.cuda.synchronize()
    c.set_stream(None)
    assert torch.equal(back, g)


@pytest.mark.parametrize("k,stagger", [(8, 0), (40, 0), (40, 1), (128, 0)])
def test_vcoord_mean_vs_oracle(k, stagger):
    c = core()
    rng = np.random.default_rng(k + stagger)
    nz_ph, ly, lx = 11, 9, 13
    # geopotential-like magnitudes: level * 3000 m^2/s^2 plus member spread
    ph = (np.arange(nz_ph, dtype=np.float32)[None, :, None, None] * 3000.0 +
          rng.normal(0, 50, (k, nz_ph, ly, lx))).astype(np.float32)
    nz_out = nz_ph if stagger == 1 else nz_ph - 1
    alt = torch.empty((nz_out, ly, lx), device="cuda")
    c.vcoord_mean(torch.from_numpy(ph).cuda(), lx * ly, nz_ph, k, stagger, tr.G, alt)
    got = alt.cpu().numpy()
    np.testing.assert_array_equal(got, mo.vcoord_mean(ph, stagger))   # reference BLAS order
    mkl = mo.mkl_sgemv_mean(ph, stagger)
    if mkl is not None:   # the reference's own sgemv call (MKL_CBWR=COMPATIBLE)
        np.testing.assert_array_equal(got, mkl)


def test_transposer_local_world1():
    """world 1: separate member tensors go through the packing kernels (one launch), a stacked
    member tensor is var itself (no copy)."""
    c = core(5)
    t = tr.Transposer(c, 5, 7, 6)
    nz = 4
    members = [torch.randn((nz, 6, 7), device="cuda") for _ in range(5)]
    var = t.scatter_grid({m: members[m] for m in range(5)}, nz)
    assert torch.equal(var, torch.stack(members))   # one rank owns every column
    back = t.gather_grid(var)
    for m in range(5):
        assert torch.equal(back[m], members[m])
    stk = torch.stack(members)
    var = t.scatter_grid({m: stk[m] for m in range(5)}, nz)
    assert var.data_ptr() == stk.data_ptr()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir, k, nx, ny, nz):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    c = abi.Core(k, device=0)
    t = tr.Transposer(c, k, nx, ny)
    run_plan(t, k, nx, ny, nz, out_dir, rank)
    dist.barrier()
    c.finalize()
    dist.destroy_process_group()


def test_transposer_two_processes_real_kernels(tmp_path):
    world, k, nx, ny, nz = 2, 5, 7, 5, 3
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), k, nx, ny, nz), nprocs=world,
             join=True)
    check_plan(str(tmp_path), world, k, nx, ny, nz)


@pytest.mark.parametrize("nm,n", [(1, 1000), (5, 100_003), (40, 2_000_000)])
def test_member_sum_and_scale_kernels(nm, n):
    """cwbl_member_sum (fp32, member order) and cwbl_scale (sscal) bit for bit against the
    same operations in numpy."""
    c = core()
    rng = np.random.default_rng(nm)
    f = rng.normal(size=(nm, n)).astype(np.float32)
    dev = torch.device("cuda:0")
    fd = torch.from_numpy(f).to(dev)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    c.member_sum(fd, n, nm, out)
    acc = np.zeros(n, np.float32)
    for m in range(nm):
        acc = acc + f[m]
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), acc.view(np.uint32))
    inv = np.float32(1.0) / np.float32(nm)
    c.scale(out, n, float(inv))
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), (inv * acc).view(np.uint32))


def test_write_mean_single_rank():
    """write_mean through the Transposer with the real kernels, one rank holding all k
    members: the member-order sum times nmember_inv, bit for bit."""
    k = 8
    c = core(k)
    t = tr.Transposer(c, k, 10, 7, device=torch.device("cuda:0"))
    rng = np.random.default_rng(2)
    allf = {m: [rng.normal(size=(7, 10)).astype(np.float32),
                rng.normal(size=(4, 7, 11)).astype(np.float32)] for m in range(k)}
    fields = {m: [torch.from_numpy(a).cuda() for a in allf[m]] for m in range(k)}
    out = t.write_mean(fields)
    inv = np.float32(1.0) / np.float32(k)
    for i in range(2):
        acc = np.zeros_like(allf[0][i])
        for m in range(k):
            acc = acc + allf[m][i]
        np.testing.assert_array_equal(out[i].cpu().numpy().view(np.uint32),
                                      (inv * acc).view(np.uint32))


# ---- the kernels against the reference's own module_mpi_util (tests/golden/mpi_util_*.npz) --
from test_mpi_util_golden import FIXTURES, load  # noqa: E402


@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_pack_unpack_vcoord_kernels_vs_reference_fixtures(path):
    """cwbl_pack_members / cwbl_unpack_members / cwbl_vcoord_mean on the inputs the compiled
    reference's letkf_scatter_grid / letkf_gather_grid / letkf_scatter_vcoord saw under
    mpirun: a member's packed buffer is the ranks' slabs in rank order (the alltoallv
    sdispls), unpacking the ranks' 2 * var gives the reference's gathered members, and the
    vertical coordinate of every rank equals its sgemv mean (MKL) bit for bit."""
    g, nproc, k, nx, ny, nz = load(path)
    c = core(max(k, 2))
    px, py = tr.dims_create(nproc)
    for st in (0, 1, 2):
        gx, gy = nx + (st == 1), ny + (st == 2)
        n = gx * gy * nz
        members = torch.from_numpy(np.stack([g[f"r{m}_s{st}_in"] for m in range(k)])).cuda()
        send = torch.full((k * n,), float("nan"), device="cuda")
        c.pack_members(members, n, k, gx, gy, nz, px, py, send, n)
        want = np.stack([np.concatenate([g[f"r{r}_s{st}_local"][m].ravel() for r in range(nproc)])
                         for m in range(k)])
        np.testing.assert_array_equal(send.cpu().numpy().reshape(k, n), want)
        recv = torch.from_numpy(np.float32(2.0) * want).cuda()
        out = torch.full((k, nz, gy, gx), float("nan"), device="cuda")
        c.unpack_members(recv, n, k, gx, gy, nz, px, py, out, n)
        got = out.cpu().numpy()
        for m in range(k):
            np.testing.assert_array_equal(got[m], g[f"r{m}_s{st}_back"])
    for tag, stagger, nzp in (("v0", 0, nz + 1), ("v1", 1, nz)):
        tmp4d = mo.scatter_grid([g[f"r{m}_{tag}_in"] for m in range(k)], nproc, 0)
        for r in range(nproc):
            lx, ly = int(g[f"r{r}_info"][0]), int(g[f"r{r}_info"][1])
            alt = torch.empty((nz, ly, lx), device="cuda")
            c.vcoord_mean(torch.from_numpy(tmp4d[r]).cuda(), lx * ly, nzp, k, stagger, tr.G, alt)
            np.testing.assert_array_equal(alt.cpu().numpy().view(np.uint32),
                                          g[f"r{r}_{tag}_out"].view(np.uint32))
