"""TEST INFRASTRUCTURE ONLY: numpy restatement of the reference's member <-> column
transposes (module_mpi_util.f90), the checker for cwbl/transpose.py and the
cwbl_pack_columns / cwbl_unpack_columns / cwbl_vcoord_mean kernels.

  dims_create        MPI_Dims_create(nproc, 2, dims) as called by letkf_init (:48-49);
                     pinned against MPICH's own answers (tests/golden/dims_create.json)
  local_info         letkf_local_info (:71-188): cyclic block-1 xloc/yloc (+ _u/_v)
  scatter_grid       letkf_scatter_grid (:190-262) for every rank at once
  gather_grid        letkf_gather_grid (:264-358)
  vcoord_mean        letkf_scatter_vcoord's sgemv mean + destagger (:491-505): the reference
                     BLAS order in fp32 (y = 0; y += (alpha*1)*A(:,j)), and the same call
                     through MKL's sgemv_ (what an MKL-linked reference computes)

Pinned bit for bit against the reference itself: oracle/ref/build_mpi_util.sh compiles
module_mpi_util.f90 from /root/reference (MPICH's mpif.h behind a `module mpi` wrapper, the
image's mpi.mod being gfortran's), oracle/gen_mpi_util_goldens.py runs it under mpirun at
2, 6 and 8 ranks, and tests/test_mpi_util_golden.py checks every function below against
every rank's output (tests/golden/mpi_util_n*_k*.npz).
Arrays: a global field is global(nx,ny,nz) Fortran order = numpy (nz,ny,nx) C order; a local
slab var(loc_nx,loc_ny,nz,0:k-1) = numpy (k,nz,loc_ny,loc_nx).
"""
import ctypes as C
import math
import os

import numpy as np


def dims_create(nproc):
    """(nproc_x, nproc_y): the most balanced factorisation, nproc_x >= nproc_y."""
    d = next(d for d in range(math.isqrt(nproc), nproc + 1) if d * d >= nproc and nproc % d == 0)
    return d, nproc // d


def _split(n, start, stride):
    # do i = start, n, stride; do j = i, min(n, i+nxb-1) with nxb = 1 (0-based here)
    return np.arange(start, n, stride, dtype=np.int64)


def local_info(nx, ny, nproc):
    """Per rank: dict(id_x, id_y, xloc, yloc, xloc_u, yloc_v) with 0-based indices."""
    px, py = dims_create(nproc)
    out = []
    for rank in range(nproc):
        id_x, id_y = rank % px, rank // px
        out.append(dict(id_x=id_x, id_y=id_y,
                        xloc=_split(nx, id_x, px), yloc=_split(ny, id_y, py),
                        xloc_u=_split(nx + 1, id_x, px), yloc_v=_split(ny + 1, id_y, py)))
    return out


def _locs(info, stagger):
    return (info["xloc_u"] if stagger == 1 else info["xloc"],
            info["yloc_v"] if stagger == 2 else info["yloc"])


def scatter_grid(globals_by_member, nproc, stagger=0):
    """Member m's field (nz,ny,nx) -> every rank's var (k,nz,loc_ny,loc_nx)."""
    k = len(globals_by_member)
    nz, gy, gx = globals_by_member[0].shape
    nx, ny = gx - (stagger == 1), gy - (stagger == 2)
    out = []
    for info in local_info(nx, ny, nproc):
        xl, yl = _locs(info, stagger)
        var = np.empty((k, nz, len(yl), len(xl)), np.float32)
        for m in range(k):
            var[m] = globals_by_member[m][:, yl][:, :, xl]   # global(idxx, idxy, :)
        out.append(var)
    return out


def gather_grid(locals_by_rank, nx, ny, stagger=0):
    """Every rank's var (k,nz,loc_ny,loc_nx) -> member fields (nz,ny',nx')."""
    nproc = len(locals_by_rank)
    k, nz = locals_by_rank[0].shape[:2]
    gx, gy = nx + (stagger == 1), ny + (stagger == 2)
    g = [np.zeros((nz, gy, gx), np.float32) for _ in range(k)]
    for info, var in zip(local_info(nx, ny, nproc), locals_by_rank):
        xl, yl = _locs(info, stagger)
        for m in range(k):
            g[m][np.ix_(np.arange(nz), yl, xl)] = var[m]
    return g


def pack_columns(global_field, px, py):
    """cwbl_pack_columns restated: rank-major concatenation of the ranks' column chunks."""
    nz, ny, nx = global_field.shape
    parts = []
    for rank in range(px * py):
        xl, yl = _split(nx, rank % px, px), _split(ny, rank // px, py)
        parts.append(global_field[:, yl][:, :, xl].ravel())
    return np.concatenate(parts).astype(np.float32)


def unpack_columns(packed, nz, ny, nx, px, py):
    """cwbl_unpack_columns restated: the inverse of pack_columns -> (nz, ny, nx)."""
    g = np.zeros((nz, ny, nx), np.float32)
    off = 0
    for rank in range(px * py):
        xl, yl = _split(nx, rank % px, px), _split(ny, rank // px, py)
        n = len(xl) * len(yl) * nz
        g[np.ix_(np.arange(nz), yl, xl)] = packed[off:off + n].reshape(nz, len(yl), len(xl))
        off += n
    return g


def vcoord_mean(ph_local, stagger, g=np.float32(9.81)):
    """ph_local (k, nz_ph, loc_ny, loc_nx) -> alt: reference BLAS sgemv order, fp32."""
    k = ph_local.shape[0]
    alpha = np.float32(1.0) / (np.float32(g) * np.float32(k))
    y = np.zeros(ph_local.shape[1:], np.float32)
    for m in range(k):
        y = (y + (alpha * ph_local[m]).astype(np.float32)).astype(np.float32)
    if stagger == 1:
        return y
    return ((y[1:] + y[:-1]).astype(np.float32) * np.float32(0.5)).astype(np.float32)


_mkl = None


def mkl_sgemv_mean(ph_local, stagger, g=np.float32(9.81)):
    """The reference's call itself, sgemv('n', n, k, 1.0/(g*k), tmp4d, n, x=1, 1, 0.0, y, 1),
    through MKL (MKL_CBWR=COMPATIBLE), then the same destagger.  None without MKL."""
    global _mkl
    if _mkl is None:
        os.environ.setdefault("MKL_CBWR", "COMPATIBLE")
        for p in ("/opt/conda/lib/libmkl_rt.so", "libmkl_rt.so"):
            try:
                _mkl = C.CDLL(p)
                break
            except OSError:
                _mkl = False
    if not _mkl:
        return None
    k = ph_local.shape[0]
    a = np.ascontiguousarray(ph_local, np.float32)       # column j = member j (Fortran)
    n = a[0].size
    alpha = np.float32(1.0) / (np.float32(g) * np.float32(k))
    x = np.ones(k, np.float32)
    y = np.zeros(n, np.float32)
    ci = lambda v: C.byref(C.c_int(v))                    # noqa: E731
    cf = lambda v: C.byref(C.c_float(v))                  # noqa: E731
    _mkl.sgemv_(C.c_char_p(b"N"), ci(n), ci(k), cf(float(alpha)), a.ctypes.data_as(C.c_void_p),
                ci(n), x.ctypes.data_as(C.c_void_p), ci(1), cf(0.0),
                y.ctypes.data_as(C.c_void_p), ci(1))
    y = y.reshape(ph_local.shape[1:])
    if stagger == 1:
        return y
    return ((y[1:] + y[:-1]).astype(np.float32) * np.float32(0.5)).astype(np.float32)
