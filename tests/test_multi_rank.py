"""Multi-process (world_size 2, gloo, CPU) check of the sharded path: columns dealt as the
reference deals them (cyclic px x py grid),
the obs set broadcast once from rank 0, each rank analysing its shard independently (with
the oracle standing in for the GPU core on CPU), results reassembled == single process."""
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


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _analyse_oracle(w, xyz, obs, hdxb):
    from helpers import oracle
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, xyz, obs, hdxb).build()
    var = w.var.copy()
    st = abi.Stats()
    rc = oracle().orc_analyze_var(w.k, 0, -5.0, 0, C.byref(ob), C.byref(w.vp),
                                  C.byref(abi.make_slab(w.x, w.y, w.alt, var)), 1, C.byref(st))
    assert rc == 0
    return var, st.solved


def _worker(rank, world, port, out_dir):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w = synth.make("c2", seed=5, scale=0.06, nz=6, shard=(rank, world))
    n, k = w.obs.shape[0], w.k
    buf = torch.zeros(cdist.packed_len(n, k), dtype=torch.float32)
    if rank == 0:
        buf.copy_(torch.from_numpy(cdist.pack_radar(w.obs_xyz, w.obs, w.hdxb)))
    cdist.broadcast_obs(buf, src=0)
    xyz, obs, hdxb = cdist.unpack_radar(buf.numpy(), n, k)
    var, solved = _analyse_oracle(w, xyz, obs, hdxb)
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), var)
    tot = torch.tensor([solved], dtype=torch.int64)
    dist.all_reduce(tot)
    if rank == 0:
        np.save(os.path.join(out_dir, "solved.npy"), tot.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_analysis_equals_single_process(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    full = synth.make("c2", seed=5, scale=0.06, nz=6)
    ref, solved_ref = _analyse_oracle(full, full.obs_xyz, full.obs, full.hdxb)
    got = np.empty_like(ref)
    for r in range(world):
        xs, ys = cdist.shard_columns(full.nx, full.ny, r, world)
        got[:, :, ys[:, None], xs[None, :]] = np.load(tmp_path / f"rank{r}.npy")
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert int(np.load(tmp_path / "solved.npy")[0]) == solved_ref


def _wire_types(case):
    """The G4 case's obs types in ObsSetBuilder layouts (radar: obs (n,), hdxb (k,n))."""
    out = []
    for t in case.types:
        d = dict(t)
        if t["family"] == 1:
            d["obs"], d["hdxb"] = t["obs"][:, 0], t["hdxb"][:, :, 0]
        out.append(d)
    return out


def _worker_obs_set(rank, world, port, out_dir, with_layout=False):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "tests"))
    from helpers import DriverCase, oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    case = DriverCase("driver_mixed.npz")
    types = _wire_types(case) if rank == 0 else None
    layout = cdist.wire_layout(_wire_types(case)) if with_layout else None
    calls = []
    real = dist.broadcast
    dist.broadcast = lambda *a, **kw: (calls.append(1), real(*a, **kw))[1]
    try:
        k, got = cdist.broadcast_obs_set(types, case.k, torch.device("cpu"), src=0,
                                         layout=layout)
    finally:
        dist.broadcast = real
    assert len(calls) == (1 if with_layout else 2), calls
    got = [{key: (v.numpy() if isinstance(v, torch.Tensor) else v) for key, v in t.items()}
           for t in got]
    ob = cdist.builder_from(got, abi.MEM_HOST).build()
    slab, var = case.slab()
    rc = oracle().orc_analyze_var(k, case.wf, case.norain, 0, C.byref(ob), C.byref(case.vp),
                                  C.byref(slab), 1, C.byref(abi.Stats()))
    assert rc == 0
    np.save(os.path.join(out_dir, f"obs_rank{rank}.npy"), var)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("with_layout", [False, True])
def test_obs_set_broadcast_carries_the_whole_set(tmp_path, with_layout):
    """The obs-set wire format (GTS sound/synop/metar with QC + radar dbz/vr) through the
    broadcast of a 2-rank gloo group: every rank's analysis of the received set equals the
    reference's output for the G4 mixed case bit for bit.  With the layout (the counts every
    rank knows) the exchange is ONE broadcast; without it the length goes first."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from helpers import DriverCase
    world = 2
    mp.spawn(_worker_obs_set, args=(world, _free_port(), str(tmp_path), with_layout),
             nprocs=world, join=True)
    ref = DriverCase("driver_mixed.npz").var_out
    for r in range(world):
        got = np.load(tmp_path / f"obs_rank{r}.npy")
        np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_obs_set_wire_roundtrip():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from helpers import DriverCase
    case = DriverCase("driver_mixed.npz")
    types = _wire_types(case)
    buf = cdist.pack_obs_set(types, case.k)
    k, got = cdist.unpack_obs_set(buf)
    assert k == case.k and len(got) == len(types)
    for a, b in zip(types, got):
        assert (a["family"], a["type_id"]) == (b["family"], b["type_id"])
        keys = ("xyz", "obs", "error", "hdxb", "qc") if a["family"] == 0 else ("xyz", "obs", "hdxb")
        for key in keys:
            np.testing.assert_array_equal(np.asarray(b[key]), np.asarray(a[key]))
        if a["family"] == 0:
            assert b["qc"].dtype == np.int32
    with pytest.raises(ValueError):
        cdist.unpack_obs_set(buf[:-1])
    bad = buf.copy()
    bad[0] = 0.0
    with pytest.raises(ValueError):
        cdist.unpack_obs_set(bad)


def test_wire_layout_sizes_the_buffer():
    """wire_words(wire_layout(set)) is the packed length, for raw and unpacked types; a set
    that does not match the agreed layout is refused before anything is sent."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from helpers import DriverCase
    case = DriverCase("driver_mixed.npz")
    types = _wire_types(case)
    buf = cdist.pack_obs_set(types, case.k)
    lay = cdist.wire_layout(types)
    assert cdist.wire_words(lay, case.k) == buf.shape[0]
    assert cdist.wire_layout(cdist.unpack_obs_set(buf)[1]) == lay
    assert {f for f, _, _, _ in lay} == {0, 1}


def test_shard_columns_partition():
    for nx, ny in ((1, 1), (7, 5), (300, 300), (301, 299)):
        for world in (1, 2, 3, 8):
            seen = np.zeros((ny, nx), np.int32)
            for r in range(world):
                xs, ys = cdist.shard_columns(nx, ny, r, world)
                seen[ys[:, None], xs[None, :]] += 1
            assert (seen == 1).all()


def test_pack_roundtrip():
    rng = np.random.default_rng(0)
    n, k = 17, 5
    xyz, obs, hdxb = rng.random((n, 3)), rng.random(n), rng.random((k, n))
    p = cdist.pack_radar(xyz, obs, hdxb)
    assert p.shape[0] == cdist.packed_len(n, k)
    a, b, c = cdist.unpack_radar(p, n, k)
    np.testing.assert_array_equal(a, xyz.astype(np.float32))
    np.testing.assert_array_equal(b, obs.astype(np.float32))
    np.testing.assert_array_equal(c, hdxb.astype(np.float32))
