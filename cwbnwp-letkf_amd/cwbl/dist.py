"""Multi-GPU plumbing (one process per GPU, torch.distributed).

The analysis shards embarrassingly: grid columns are dealt to ranks and points never
communicate.  The only exchange is ONE broadcast of the packed observation set from the
rank that read it (RCCL over xGMI on MI355X, backend "nccl"; gloo on CPU for tests).  It
replaces the reference's ibcast/iallgatherv chain (module_gts_omboma.f90:524-611,
module_radar.f90:143-180).  Columns are dealt as the reference deals them: cyclically with
block 1 over a px x py rank grid (letkf_local_info, module_mpi_util.f90:71-188, px >= py from
MPI_Dims_create; cwbl/transpose.py's Decomposition), which balances the uneven obs density
and gives every rank the same point count whenever px | nx and py | ny (300 x 300 over 1, 2,
4 or 8 ranks).
"""
import numpy as np


def shard_columns(nx, ny, rank, world):
    """(xs, ys): the 0-based grid columns x and rows y of `rank`'s columns (cpu(rank)%xloc,
    %yloc of letkf_local_info); the rank analyses the loc_nx x loc_ny block of their products."""
    from .transpose import Decomposition
    return Decomposition(nx, ny, world).columns(rank)


# ---- wire format of a whole observation set ------------------------
# One float32 buffer; integers travel as int32 bit patterns:
#   [0] WIRE_MAGIC  [1] ntypes  [2] k
#   [3 + 4t .. 6 + 4t]  family (0 GTS, 1 radar), type_id, nvar, nobs of type t
#   then, type by type in header order, the cwbl_obs_set arrays in the reference's layouts
#   (module_gts_omboma.f90:18-21, module_radar.f90:13-16):
#     GTS:   xyz (n,3) | obs (n,nvar) | error (n,nvar) | hdxb (k,n,nvar) | qc (k,n,nvar) int32
#     radar: xyz (n,3) | obs (n,) | hdxb (k,n)
# The reference sends these as ~8 ibcasts and 2 iallgatherv per GTS type and 5 ibcasts + 1
# iallgatherv per radar type, after an mpi_bcast of the counts; here the counts ride in the
# header and the whole set is one message (one broadcast when every rank knows the layout,
# else preceded by its length).
WIRE_MAGIC = 0x4C4B4631  # "LKF1"


def _type_words(family, nvar, n, k):
    return 3 * n + (2 * n * nvar + 2 * k * n * nvar if family == 0 else n + k * n)


def pack_obs_set(types, k):
    """types: dicts {family, type_id, xyz, obs, hdxb} (+ error, qc for GTS), numpy arrays in
    the layouts above (ObsSetBuilder's).  Returns the float32 wire buffer."""
    hdr = [WIRE_MAGIC, len(types), int(k)]
    parts = []
    for t in types:
        fam = int(t["family"])
        xyz = np.ascontiguousarray(t["xyz"], np.float32)
        n = int(xyz.shape[0])
        obs = np.ascontiguousarray(t["obs"], np.float32)
        nvar = int(obs.shape[1]) if fam == 0 else 1
        hdr += [fam, int(t["type_id"]), nvar, n]
        parts.append(xyz.ravel())
        if fam == 0:
            parts += [obs.ravel(), np.ascontiguousarray(t["error"], np.float32).ravel(),
                      np.ascontiguousarray(t["hdxb"], np.float32).ravel(),
                      np.ascontiguousarray(t["qc"], np.int32).view(np.float32).ravel()]
        else:
            parts += [obs.ravel(), np.ascontiguousarray(t["hdxb"], np.float32).ravel()]
    return np.concatenate([np.asarray(hdr, np.int32).view(np.float32)] + parts)


def unpack_obs_set(buf):
    """(k, types): per-type views into a wire buffer (numpy array or torch tensor, on any
    device); qc views are int32."""
    is_np = isinstance(buf, np.ndarray)

    def ints(a):
        if is_np:
            return a.view(np.int32)
        import torch
        return a.view(torch.int32)

    def host_ints(a):
        v = ints(a)
        return [int(x) for x in (v if is_np else v.cpu().numpy())]

    magic, ntypes, k = host_ints(buf[:3])
    if magic != WIRE_MAGIC:
        raise ValueError(f"not an obs-set wire buffer (magic {magic:#x})")
    hdr = host_ints(buf[3:3 + 4 * ntypes])
    off = 3 + 4 * ntypes
    types = []
    for t in range(ntypes):
        fam, tid, nvar, n = hdr[4 * t:4 * t + 4]

        def take(cnt, shape):
            nonlocal off
            a = buf[off:off + cnt].reshape(shape)
            off += cnt
            return a

        d = dict(family=fam, type_id=tid, nvar=nvar, nobs=n, xyz=take(3 * n, (n, 3)))
        if fam == 0:
            d["obs"] = take(n * nvar, (n, nvar))
            d["error"] = take(n * nvar, (n, nvar))
            d["hdxb"] = take(k * n * nvar, (k, n, nvar))
            d["qc"] = ints(take(k * n * nvar, (k, n, nvar)))
        else:
            d["obs"] = take(n, (n,))
            d["hdxb"] = take(k * n, (k, n))
        types.append(d)
    if off != buf.shape[0]:
        raise ValueError(f"wire buffer has {buf.shape[0]} words, header describes {off}")
    return k, types


def builder_from(types, memory):
    """An abi.ObsSetBuilder holding the (unpacked) types."""
    from . import abi
    b = abi.ObsSetBuilder(memory)
    for t in types:
        if t["family"] == 0:
            b.add_gts(t["type_id"], t["xyz"], t["obs"], t["error"], t["hdxb"], t["qc"])
        else:
            b.add_radar(t["type_id"], t["xyz"], t["obs"], t["hdxb"])
    return b


def wire_layout(types):
    """The header of a set as (family, type_id, nvar, nobs) per type: what every rank must know
    to size the receive buffer of a one-collective broadcast (the reference broadcasts the
    same counts ahead of the data, module_gts_omboma.f90:524-531)."""
    out = []
    for t in types:
        fam = int(t["family"])
        n = int(np.asarray(t["xyz"]).shape[0]) if "nobs" not in t else int(t["nobs"])
        nvar = (int(t["nvar"]) if "nvar" in t else int(np.asarray(t["obs"]).shape[1])) \
            if fam == 0 else 1
        out.append((fam, int(t["type_id"]), nvar, n))
    return out


def wire_words(layout, k):
    """Length in words of the wire buffer of a set with this layout."""
    return 3 + 4 * len(layout) + sum(_type_words(f, nv, n, k) for f, _, nv, n in layout)


def broadcast_obs_set(types, k, device, src=0, group=None, layout=None):
    """The obs-set exchange of a cycle: `src` packs its set (`types`, ignored elsewhere),
    every rank receives it into one buffer on `device`.  Returns (k, types) as views into the
    received buffer.

    With `layout` (wire_layout of the set, known to every rank: the counts the reference
    broadcasts ahead of its data) the exchange is ONE broadcast of the whole set, sized from
    the layout.  Without it the length goes first (one 8-byte broadcast), then the set."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    gsrc = src if group is None else dist.get_global_rank(group, src)
    if rank == src:
        buf = torch.from_numpy(pack_obs_set(types, k)).to(device)
        if layout is not None and (wire_layout(types) != [tuple(x) for x in layout]
                                   or buf.shape[0] != wire_words(layout, k)):
            raise ValueError("broadcast_obs_set: the set does not match the agreed layout")
    if layout is not None:
        if rank != src:
            buf = torch.empty(wire_words(layout, k), dtype=torch.float32, device=device)
    else:
        ln = torch.tensor([buf.shape[0] if rank == src else 0], dtype=torch.int64,
                          device=device)
        dist.broadcast(ln, src=gsrc, group=group)
        if rank != src:
            buf = torch.empty(int(ln.item()), dtype=torch.float32, device=device)
    dist.broadcast(buf, src=gsrc, group=group)
    return unpack_obs_set(buf)


# ---- single radar type (the bench's synthetic set) ---------------------------------------
def pack_radar(obs_xyz, obs, hdxb):
    """One float32 buffer: xyz (n,3) | obs (n,) | hdxb (k,n)."""
    return np.concatenate([np.asarray(obs_xyz, np.float32).ravel(),
                           np.asarray(obs, np.float32).ravel(),
                           np.asarray(hdxb, np.float32).ravel()])


def packed_len(n, k):
    return n * (4 + k)


def unpack_radar(buf, n, k):
    """Views into a packed buffer (numpy array or torch tensor)."""
    xyz = buf[:3 * n].reshape(n, 3) if hasattr(buf, "reshape") else None
    return xyz, buf[3 * n:4 * n], buf[4 * n:4 * n + k * n].reshape(k, n)


def broadcast_obs(buf, src=0, group=None):
    """Broadcast of a pre-sized packed buffer (torch tensor, any backend)."""
    import torch.distributed as dist
    dist.broadcast(buf, src=src, group=group)
    return buf
