"""Member <-> column transposes on the device.

The reference moves every analysed variable between two layouts with host-packed MPI
collectives (module_mpi_util.f90):
  member layout  rank m holds member m's whole field, global(nx,ny,nz)
  column layout  each rank holds its columns for all members, var(loc_nx,loc_ny,nz,0:k-1)
  letkf_scatter_grid   (:190-262)  member -> column  (mpi_alltoallv)
  letkf_gather_grid    (:264-358)  column -> member  (mpi_alltoallv)
  letkf_scatter_hcoord (:360-443)  root's lat/lon -> columns (mpi_scatterv)
  letkf_scatter_vcoord (:445-580)  member PH -> column ensemble mean / g, destaggered
                                   (mpi_alltoallv + sgemv), or root's HGT (mpi_scatterv)
Columns are dealt cyclically with block 1 over a px x py rank grid (letkf_local_info,
:71-188, px >= py from mpi_dims_create).

Here the packing, unpacking and the ensemble mean are HIP kernels behind the C ABI
(cwbl_pack_columns / cwbl_unpack_columns / cwbl_vcoord_mean) working on device memory, and
the exchange is torch.distributed point-to-point: with backend "nccl" (RCCL on ROCm) one
group of ncclSend/ncclRecv over xGMI per transpose, messages going straight from the packed
buffer into their final place in `var` (member-slowest, so each member's chunk is
contiguous: no unpack on the column side).  Backend "gloo" stages each message through host
memory; it is the transport of the CPU/one-GPU multi-process tests, not a compute path.

Member m lives on rank m % world: the reference's rank m when world >= k, and k/world
members per rank on an 8-GPU node at k = 40.
Tensors: a global field is torch (nz, ny', nx') for Fortran global(nx',ny',nz); a column slab
is (k, nz, loc_ny, loc_nx) for var(loc_nx,loc_ny,nz,0:k-1).
"""
import math

import numpy as np

G = 9.81  # module_param.f90:109


def dims_create(nproc):
    """MPI_Dims_create(nproc, 2): the most balanced (px, py), px >= py (letkf_init :48-52)."""
    d = next(d for d in range(math.isqrt(nproc), nproc + 1) if d * d >= nproc and nproc % d == 0)
    return d, nproc // d


def _cyc(n, i, p):
    return (n - i + p - 1) // p if i < n else 0


class Decomposition:
    """letkf_local_info (:71-188) for an nx x ny mass grid over `world` ranks."""

    def __init__(self, nx, ny, world):
        self.nx, self.ny, self.world = nx, ny, world
        self.px, self.py = dims_create(world)

    def grid(self, stagger):
        """(nx', ny') of the field: U is staggered in x (stagger 1), V in y (stagger 2)."""
        return self.nx + (stagger == 1), self.ny + (stagger == 2)

    def coords(self, rank):
        return rank % self.px, rank // self.px

    def local_shape(self, rank, stagger=0):
        """(loc_nx, loc_ny), or (loc_nx_u, loc_ny) / (loc_nx, loc_ny_v) when staggered."""
        gx, gy = self.grid(stagger)
        ix, iy = self.coords(rank)
        return _cyc(gx, ix, self.px), _cyc(gy, iy, self.py)

    def columns(self, rank, stagger=0):
        """0-based xloc, yloc of `rank` (cpu(rank)%xloc - 1, ...)."""
        gx, gy = self.grid(stagger)
        ix, iy = self.coords(rank)
        return np.arange(ix, gx, self.px), np.arange(iy, gy, self.py)

    def chunks(self, nz, stagger=0):
        """(offset, count) of every rank's chunk in a packed buffer (sdispls/sendcnts)."""
        out, off = [], 0
        for r in range(self.world):
            lx, ly = self.local_shape(r, stagger)
            out.append((off, lx * ly * nz))
            off += lx * ly * nz
        return out


class Transposer:
    """One rank's side of the transposes.  `core` is the cwbl.abi.Core of this process.

    `loopback`: every chunk goes through the transport, a rank's own chunk included (a send
    to itself), and write_mean's reduce runs at world 1 too.  Off, a rank copies its own
    chunk and a one-rank job never communicates; on, a one-GPU RCCL job executes every
    collective and point-to-point call of the multi-GPU path (tests/test_gpu_rccl.py)."""

    def __init__(self, core, k, nx, ny, group=None, device=None, loopback=False):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.core, self.k, self.group, self.loopback = core, k, group, bool(loopback)
        if dist.is_available() and dist.is_initialized():
            self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
            self.backend = dist.get_backend(group)
        else:
            self.rank, self.world, self.backend = 0, 1, None
        self.dec = Decomposition(nx, ny, self.world)
        self.device = device or torch.device("cuda", torch.cuda.current_device())

    # ---- ownership -------------------------------------------------------------------------
    def owner(self, m):
        return m % self.world

    def owned(self):
        return list(range(self.rank, self.k, self.world))

    def local_shape(self, stagger=0):
        return self.dec.local_shape(self.rank, stagger)

    # ---- transport -------------------------------------------------------------------------
    def _peer(self, r):
        return r if self.group is None else self.dist.get_global_rank(self.group, r)

    def _exchange(self, sends, recvs):
        """sends / recvs: lists of (peer rank, tag, contiguous device tensor); posted in the
        same (peer, tag) order on both sides."""
        dist, torch = self.dist, self.torch
        if not sends and not recvs:
            return
        if self.backend == "nccl":
            ops = [dist.P2POp(dist.isend, t, self._peer(p), self.group) for p, _, t in sends]
            ops += [dist.P2POp(dist.irecv, t, self._peer(p), self.group) for p, _, t in recvs]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            return
        # gloo (tests): host staging, one tag per message; gloo has no pair to the rank
        # itself, so loopback messages are matched in posting order and copied
        own_s = [t for p, _, t in sends if p == self.rank]
        own_r = [t for p, _, t in recvs if p == self.rank]
        if len(own_s) != len(own_r):
            raise RuntimeError("transpose: unmatched loopback messages")
        for a, b in zip(own_s, own_r):
            b.copy_(a)
        sends = [x for x in sends if x[0] != self.rank]
        recvs = [x for x in recvs if x[0] != self.rank]
        reqs, landing = [], []
        for p, tag, t in sends:
            h = t.cpu()
            reqs.append((dist.isend(h, self._peer(p), group=self.group, tag=tag), h))
        for p, tag, t in recvs:
            h = torch.empty(t.shape, dtype=t.dtype)
            reqs.append((dist.irecv(h, self._peer(p), group=self.group, tag=tag), h))
            landing.append((h, t))
        for w, _ in reqs:
            w.wait()
        for h, t in landing:
            t.copy_(h)

    def _sync(self):
        # the library runs on its own stream: torch's producers must have finished
        if self.device.type == "cuda":
            self.torch.cuda.synchronize(self.device)

    # ---- write_mean's ensemble mean (module_grid.f90:700-840) -------
    def write_mean(self, fields, root=0):
        """fields: {m: [device tensors]} — the same list of analysed fields (psfc, mu, u, ...,
        any shapes) for every member this rank owns.  Returns, on `root`, the list of the
        ensemble means (sum over members * nmember_inv), None elsewhere.

        The reference reduces each field separately over the member ranks (one mpi_reduce
        per field, :744-822, 14-20 of them) and scales on the root with sscal (:827-...).
        Here the fields are packed into one buffer per member, the members a rank holds are
        summed on the device in member order (cwbl_member_sum), ONE reduce (RCCL over xGMI
        with backend nccl) combines the ranks, and the root scales (cwbl_scale).  The sum
        order across ranks is the collective's, as it is MPI's in the reference, so the
        means agree with the reference to fp32 rounding of the sums, not bit for bit."""
        torch, dist = self.torch, self.dist
        mine = self.owned()
        shapes = [tuple(t.shape) for t in fields[mine[0]]] if mine else []
        if self.world > 1:  # every rank needs the layout (a rank may own no member)
            shapes = self._bcast_shapes(shapes, self.owner(0))
        sizes = [int(np.prod(sh)) for sh in shapes]
        n = int(sum(sizes))
        packed = torch.empty((max(len(mine), 1), n), dtype=torch.float32, device=self.device)
        for i, m in enumerate(mine):
            off = 0
            for t, sz in zip(fields[m], sizes):
                packed[i, off:off + sz].copy_(t.reshape(-1))
                off += sz
        total = torch.empty(n, dtype=torch.float32, device=self.device)
        self._sync()
        if mine:
            self._member_sum(packed, n, len(mine), total)
        else:
            total.zero_()
        if self.world > 1 or (self.loopback and self.backend is not None):
            if self.backend == "nccl":
                dist.reduce(total, dst=self._peer(root), op=dist.ReduceOp.SUM, group=self.group)
            else:  # gloo (tests): host staging
                h = total.cpu()
                dist.reduce(h, dst=self._peer(root), op=dist.ReduceOp.SUM, group=self.group)
                total.copy_(h)
        if self.rank != root:
            return None
        self._sync()
        self._scale(total, n, float(np.float32(1.0) / np.float32(self.k)))  # nmember_inv
        out, off = [], 0
        for sh, sz in zip(shapes, sizes):
            out.append(total[off:off + sz].reshape(sh))
            off += sz
        return out

    MAX_FIELDS, MAX_DIMS = 64, 4

    def _bcast_shapes(self, shapes, src):
        """The field shapes of rank `src` to every rank as one fixed-size int64 tensor
        (count, then per field ndim and up to MAX_DIMS extents): no pickled object on the data
        path."""
        torch, dist = self.torch, self.dist
        w = 1 + self.MAX_DIMS
        buf = torch.zeros(1 + self.MAX_FIELDS * w, dtype=torch.int64)
        if self.rank == src:
            if len(shapes) > self.MAX_FIELDS or any(len(sh) > self.MAX_DIMS for sh in shapes):
                raise ValueError(f"write_mean: at most {self.MAX_FIELDS} fields of <= "
                                 f"{self.MAX_DIMS} dimensions")
            buf[0] = len(shapes)
            for i, sh in enumerate(shapes):
                buf[1 + i * w] = len(sh)
                for d, e in enumerate(sh):
                    buf[2 + i * w + d] = int(e)
        t = buf.to(self.device) if self.backend == "nccl" else buf
        dist.broadcast(t, src=self._peer(src), group=self.group)
        v = t.cpu().tolist()
        return [tuple(v[2 + i * w: 2 + i * w + v[1 + i * w]]) for i in range(v[0])]

    def _member_sum(self, packed, n, nm, out):
        self.core.member_sum(packed, n, nm, out)

    def _scale(self, x, n, alpha):
        self.core.scale(x, n, alpha)

    # ---- member fields as one stacked tensor ----------------------------------------------------
    @staticmethod
    def _stacked(tensors, shape):
        """(first tensor, stride in elements) when `tensors` are contiguous fields of `shape`
        laid out at one constant stride (views of a stacked tensor: one launch packs them
        all), else None."""
        if not tensors or any(not t.is_contiguous() or tuple(t.shape) != tuple(shape)
                              for t in tensors):
            return None
        n = int(np.prod(shape))
        if len(tensors) == 1:
            return tensors[0], n
        base = tensors[0].untyped_storage().data_ptr()
        if any(t.untyped_storage().data_ptr() != base for t in tensors):
            return None
        d = tensors[1].data_ptr() - tensors[0].data_ptr()
        if d % 4 or d // 4 < n:
            return None
        if any(tensors[i].data_ptr() - tensors[0].data_ptr() != i * d for i in range(len(tensors))):
            return None
        return tensors[0], d // 4

    def _pack(self, fields, gx, gy, nz, dst, dstride):
        """pack_columns of every field in `fields` (a list) into dst + i * dstride: one launch
        when the fields are a stacked tensor, else one per field."""
        st = self._stacked(fields, (nz, gy, gx))
        px, py = self.dec.px, self.dec.py
        if st is not None:
            self.core.pack_members(st[0], st[1], len(fields), gx, gy, nz, px, py, dst, dstride)
        else:
            for i, f in enumerate(fields):
                assert f.is_contiguous() and tuple(f.shape) == (nz, gy, gx), tuple(f.shape)
                n = gx * gy * nz
                self.core.pack_columns(f, gx, gy, nz, px, py, dst.view(-1)[i * dstride:i * dstride + n])

    def _unpack(self, src, sstride, outs, gx, gy, nz):
        st = self._stacked(outs, (nz, gy, gx))
        px, py = self.dec.px, self.dec.py
        if st is not None:
            self.core.unpack_members(src, sstride, len(outs), gx, gy, nz, px, py, st[0], st[1])
        else:
            n = gx * gy * nz
            for i, g in enumerate(outs):
                self.core.unpack_columns(src.reshape(-1)[i * sstride:i * sstride + n], gx, gy, nz,
                                         px, py, g)

    # ---- letkf_scatter_grid (:190-262) ---------------------------------------------------------
    def scatter_grid(self, fields, nz, stagger=0, out=None):
        """fields: {m: (nz, ny', nx') device tensor} for the members this rank owns.
        Returns var (k, nz, loc_ny, loc_nx) with every member's columns of this rank.

        On one rank the column layout IS the member layout (px = py = 1): when the fields are
        the k views of one stacked (k, nz, ny', nx') tensor and no `out` is given, that tensor
        is returned as var (no copy; the analysis then updates the member fields in place, as
        gather_grid would).  Otherwise every owned member is packed in one launch."""
        torch = self.torch
        gx, gy = self.dec.grid(stagger)
        lx, ly = self.local_shape(stagger)
        mine = self.owned()
        n = gx * gy * nz
        if self.world == 1 and out is None and not self.loopback:
            st = self._stacked([fields[m] for m in mine], (nz, gy, gx))
            if st is not None and st[1] == n:
                base = st[0]
                return torch.as_strided(base, (self.k, nz, ly, lx), (n, ly * lx, lx, 1))
        var = out if out is not None else torch.empty((self.k, nz, ly, lx), dtype=torch.float32,
                                                       device=self.device)
        chunks = self.dec.chunks(nz, stagger)
        self._sync()
        if self.world == 1 and not self.loopback:  # the one chunk is this rank's slab
            self._pack([fields[m] for m in mine], gx, gy, nz, var, lx * ly * nz)
            self._sync()
            return var
        packed = torch.empty((max(len(mine), 1), n), dtype=torch.float32, device=self.device)
        if mine:
            self._pack([fields[m] for m in mine], gx, gy, nz, packed, n)
        sends, recvs = [], []
        for m in range(self.k):
            src = self.owner(m)
            if src == self.rank:
                i = mine.index(m)
                for d, (off, cnt) in enumerate(chunks):
                    if d == self.rank and not self.loopback:
                        var[m].view(-1).copy_(packed[i, off:off + cnt])
                    elif cnt:
                        sends.append((d, m, packed[i, off:off + cnt]))
            if (src != self.rank or self.loopback) and lx * ly * nz:
                recvs.append((src, m, var[m].view(-1)))
        self._sync()
        self._exchange(sends, recvs)
        self._sync()
        return var

    # ---- letkf_gather_grid (:264-358) ------------------------------------------------------------
    def gather_grid(self, var, stagger=0, out=None):
        """var (k, nz, loc_ny, loc_nx) -> {m: (nz, ny', nx')} for the members this rank owns.
        On one rank with no `out`, the result is views of var (no copy); a member field of
        `out` that already is var's member (scatter_grid's aliasing) is left as it is."""
        torch = self.torch
        k, nz = var.shape[:2]
        gx, gy = self.dec.grid(stagger)
        n = gx * gy * nz
        chunks = self.dec.chunks(nz, stagger)
        mine = self.owned()
        out = out if out is not None else {}
        if self.world == 1 and not self.loopback:
            if not var.is_contiguous() or var.dtype != torch.float32:
                raise ValueError("gather_grid: var must be a contiguous float32 slab")
            todo = [m for m in mine
                    if out.get(m) is not None and out[m].data_ptr() != var[m].data_ptr()]
            for m in mine:
                if out.get(m) is None:
                    out[m] = var[m].view(nz, gy, gx)
            if todo:
                self._sync()
                if len(todo) == len(mine):  # all k members: var is their stack at stride n
                    self._unpack(var, n, [out[m] for m in mine], gx, gy, nz)
                else:
                    for m in todo:
                        self._unpack(var[m], n, [out[m]], gx, gy, nz)
            return out
        self._sync()
        bufs = torch.empty((max(len(mine), 1), n), dtype=torch.float32, device=self.device)
        sends, recvs = [], []
        for m in range(k):
            dst = self.owner(m)
            if dst == self.rank:
                buf = bufs[mine.index(m)]
                for s, (off, cnt) in enumerate(chunks):
                    if s == self.rank and not self.loopback:
                        buf[off:off + cnt].copy_(var[m].reshape(-1))
                    elif cnt:
                        recvs.append((s, m, buf[off:off + cnt]))
            if (dst != self.rank or self.loopback) and var[m].numel():
                sends.append((dst, m, var[m].reshape(-1).contiguous()))
        self._exchange(sends, recvs)
        self._sync()
        missing = [m for m in mine if out.get(m) is None]
        if missing:  # one stacked tensor, so that the unpacking is one launch
            stk = torch.empty((len(missing), nz, gy, gx), dtype=torch.float32, device=self.device)
            for i, m in enumerate(missing):
                out[m] = stk[i]
        if mine:
            self._unpack(bufs, n, [out[m] for m in mine], gx, gy, nz)
        return out

    # ---- root -> columns (letkf_scatter_hcoord :360-443, vcoord stagger -1 :543-575) ----------
    def scatter_from_root(self, field, nz=1, stagger=0, root=0):
        """field (nz, ny', nx') on `root` (ignored elsewhere) -> (nz, loc_ny, loc_nx)."""
        torch = self.torch
        gx, gy = self.dec.grid(stagger)
        lx, ly = self.local_shape(stagger)
        local = torch.empty((nz, ly, lx), dtype=torch.float32, device=self.device)
        chunks = self.dec.chunks(nz, stagger)
        self._sync()
        sends, recvs, keep = [], [], []
        if self.rank == root:
            assert field.is_contiguous() and tuple(field.shape) == (nz, gy, gx)
            packed = torch.empty(gx * gy * nz, dtype=torch.float32, device=self.device)
            self.core.pack_columns(field, gx, gy, nz, self.dec.px, self.dec.py, packed)
            keep.append(packed)
            for d, (off, cnt) in enumerate(chunks):
                if d == root and not self.loopback:
                    local.view(-1).copy_(packed[off:off + cnt])
                elif cnt:
                    sends.append((d, 0, packed[off:off + cnt]))
        if (self.rank != root or self.loopback) and local.numel():
            recvs.append((root, 0, local.view(-1)))
        self._exchange(sends, recvs)
        self._sync()
        return local

    def scatter_hcoord(self, lat, lon, stagger=0, root=0):
        """letkf_scatter_hcoord: root's (ny', nx') lat/lon -> this rank's columns."""
        one = lambda f: None if f is None else f.reshape((1,) + tuple(f.shape[-2:]))  # noqa: E731
        return (self.scatter_from_root(one(lat), 1, stagger, root)[0],
                self.scatter_from_root(one(lon), 1, stagger, root)[0])

    # ---- letkf_scatter_vcoord (:445-580) ---------------------------------------------------------
    def scatter_vcoord(self, fields, nz, stagger, g=G, root=0):
        """alt (nz, loc_ny, loc_nx) on the mass-grid columns.
        stagger 0/1: fields = {m: PH (nz_ph, ny, nx)} of the owned members, nz_ph = nz + 1
        (0: destaggered to mass levels) or nz (1: W/PH levels); the ensemble mean over all
        k members divided by g.  stagger -1: fields = HGT (1, ny, nx) on `root`."""
        if stagger == -1:
            return self.scatter_from_root(fields, 1, 0, root)
        nz_ph = nz if stagger == 1 else nz + 1
        tmp4d = self.scatter_grid(fields, nz_ph, 0)
        lx, ly = self.local_shape(0)
        alt = self.torch.empty((nz, ly, lx), dtype=self.torch.float32, device=self.device)
        self.core.vcoord_mean(tmp4d, lx * ly, nz_ph, self.k, 1 if stagger == 1 else 0, g, alt)
        return alt
