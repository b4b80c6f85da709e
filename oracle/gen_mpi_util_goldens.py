#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY: golden vectors of the reference's member <-> column transposes.

Runs oracle/_ref/mpi_util_harness (built from /root/reference's module_mpi_util.f90 by
oracle/ref/build_mpi_util.sh) under MPICH's mpirun (oversubscribed on this container's cores)
for each (nproc, k, nx, ny, nz) below and writes tests/golden/mpi_util_n<nproc>_k<k>.npz:
  meta                  [nproc, k, nx, ny, nz]
  r<r>_info             [loc_nx, loc_ny, loc_nx_u, loc_ny_v]
  r<r>_xloc ... _yloc_v 1-based index lists of letkf_local_info
  r<r>_s<st>_in         rank r's global(gx,gy,nz) of stagger st (member r when r < k)
  r<r>_s<st>_local      var(lx,ly,nz,0:k-1) after letkf_scatter_grid
  r<r>_s<st>_back       global after letkf_gather_grid of 2 * var (ranks < k)
  r<r>_v<0|1|m1>_in     letkf_scatter_vcoord input (PH of nz+1 / nz levels; HGT, root's used)
  r<r>_v<0|1|m1>_out    its local(loc_nx,loc_ny,nz) (MKL sgemv mean / g, destaggered for 0)
  r<r>_h<st>_lat/_lon   letkf_scatter_hcoord inputs (root's used); _llat/_llon its output
Arrays are numpy C order with the Fortran axes reversed: global(gx,gy,nz) -> (nz, gy, gx),
var(lx,ly,nz,0:k-1) -> (k, nz, ly, lx).

Usage: python3 oracle/gen_mpi_util_goldens.py  (MKL_NUM_THREADS=1 MKL_CBWR=COMPATIBLE)
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
EXE = os.path.join(HERE, "_ref", "mpi_util_harness")
MPIRUN = os.environ.get("MPIRUN", "/opt/conda/bin/mpirun")
CASES = [(2, 2, 11, 9, 3), (6, 4, 11, 9, 3), (8, 5, 11, 9, 3), (8, 8, 13, 10, 2)]


def _parse(path, k, nx, ny, nz):
    raw = open(path, "rb").read()
    off = 0

    def take(n, dt):
        nonlocal off
        a = np.frombuffer(raw, dt, n, off)
        off += a.nbytes
        return a

    rank, lnx, lny, lnxu, lnyv = (int(v) for v in take(5, np.int32))
    d = {"info": np.array([lnx, lny, lnxu, lnyv], np.int32),
         "xloc": take(lnx, np.int32).copy(), "yloc": take(lny, np.int32).copy(),
         "xloc_u": take(lnxu, np.int32).copy(), "yloc_v": take(lnyv, np.int32).copy()}
    f4 = np.float32
    for st in range(3):
        gx, gy = nx + (st == 1), ny + (st == 2)
        lx, ly = (lnxu if st == 1 else lnx), (lnyv if st == 2 else lny)
        d[f"s{st}_in"] = take(gx * gy * nz, f4).reshape(nz, gy, gx)
        d[f"s{st}_local"] = take(lx * ly * nz * k, f4).reshape(k, nz, ly, lx)
        d[f"s{st}_back"] = take(gx * gy * nz, f4).reshape(nz, gy, gx)
    for tag, nzp, nzo in (("v0", nz + 1, nz), ("v1", nz, nz), ("vm1", 1, 1)):
        d[f"{tag}_in"] = take(nx * ny * nzp, f4).reshape(nzp, ny, nx)
        d[f"{tag}_out"] = take(lnx * lny * nzo, f4).reshape(nzo, lny, lnx)
    for st in range(3):
        gx, gy = nx + (st == 1), ny + (st == 2)
        lx, ly = (lnxu if st == 1 else lnx), (lnyv if st == 2 else lny)
        d[f"h{st}_lat"] = take(gx * gy, f4).reshape(gy, gx)
        d[f"h{st}_lon"] = take(gx * gy, f4).reshape(gy, gx)
        d[f"h{st}_llat"] = take(lx * ly, f4).reshape(ly, lx)
        d[f"h{st}_llon"] = take(lx * ly, f4).reshape(ly, lx)
    if off != len(raw):
        raise RuntimeError(f"{path}: {len(raw) - off} trailing bytes")
    return rank, d


def main():
    if not os.path.exists(EXE):
        subprocess.check_call([os.path.join(HERE, "ref", "build_mpi_util.sh")])
    env = dict(os.environ, MKL_NUM_THREADS="1", MKL_CBWR="COMPATIBLE", OMP_NUM_THREADS="1")
    out_dir = os.path.join(REPO, "tests", "golden")
    for nproc, k, nx, ny, nz in CASES:
        with tempfile.TemporaryDirectory() as tmp:
            cmd = [MPIRUN, "-n", str(nproc), EXE, tmp, str(nx), str(ny), str(nz), str(k)]
            subprocess.run(cmd, cwd=tmp, env=env, check=True, timeout=300)
            res = {"meta": np.array([nproc, k, nx, ny, nz], np.int32)}
            for r in range(nproc):
                rank, d = _parse(os.path.join(tmp, f"r{r}.bin"), k, nx, ny, nz)
                assert rank == r
                res.update({f"r{r}_{key}": v for key, v in d.items()})
        path = os.path.join(out_dir, f"mpi_util_n{nproc}_k{k}.npz")
        np.savez_compressed(path, **res)
        print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    sys.exit(main())
