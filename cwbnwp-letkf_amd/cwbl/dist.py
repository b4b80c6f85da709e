"""Multi-GPU plumbing (one process per GPU, torch.distributed).

The analysis shards embarrassingly: grid columns are dealt to ranks and points never
communicate.  The only exchange is ONE broadcast of the packed observation set from the
rank that read it (RCCL over xGMI on MI355X, backend "nccl"; gloo on CPU for tests).  It
replaces the reference's ibcast/iallgatherv chain (module_gts_omboma.f90:532-605,
module_radar.f90:143-180).  Row dealing is cyclic with block 1, as the reference's
decomposition (module_mpi_util.f90:73-188), which balances the uneven obs density.
"""
import numpy as np


def shard_rows(ny, rank, world):
    """Grid rows j owned by `rank` (cyclic, block size 1)."""
    return np.arange(rank, ny, world)


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
    """The single obs-set broadcast (torch tensor, any backend)."""
    import torch.distributed as dist
    dist.broadcast(buf, src=src, group=group)
    return buf
