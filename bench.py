#!/usr/bin/env python3
"""Benchmark of the MI355X LETKF analysis core on BASELINE.json's headline metric.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]

A "step" is one cwbl_analyze_var call on the configuration's full synthetic grid, i.e. one
pass of the reference's per-variable hot loop (module_letkf_core.f90:63-64 + 209-240):
k-d tree builds, QC columns, neighbour search and the per-point LETKF solve for every grid
point.  Inputs (obs set and slab) are resident in HBM before the timed region.

Multi-GPU (launched by torch.distributed.run, one process per GPU): grid columns are dealt
to ranks as the reference deals them (cyclic block-1 px x py grid, module_mpi_util.f90:71-188;
300 x 300 splits evenly over 1, 2, 4 and 8 ranks); the observation
set is generated on rank 0 and sent to every rank with ONE RCCL broadcast (backend "nccl")
before the timed region; there is no collective on the data path.  The grid is fixed as N
grows (configs[2]: the 300x300x50 grid sharded across GPUs), so scaling is "strong".

Rank 0 prints one JSON line.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "cwbnwp-letkf_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from cwbl import abi, synth  # noqa: E402
from cwbl import dist as cdist  # noqa: E402
from cwbl.transpose import dims_create as tr_dims  # noqa: E402

METRIC = "analysis grid-points/sec (+ wall-clock per cycle) at k=40, 1/2/4/8 MI355X"
FP64_PEAK_TFLOPS = 78.6   # MI355X dense FP64 (vector = matrix on gfx950), spec
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E (MI355X_MICROARCH.md)


def host_cores():
    """(logical CPUs this process may run on, physical cores among them, cgroup CPU quota or
    None).  The reference runs flat MPI, one single-threaded rank per core
    (cwb_letkf.f90:28): the CPU baselines use one process/thread per physical core of the
    affinity set, capped by the cgroup's CPU quota when one is set (processes beyond the
    quota would only be time-sliced)."""
    aff = sorted(os.sched_getaffinity(0))
    phys = set()
    for c in aff:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            phys.add((open(base + "physical_package_id").read().strip(),
                      open(base + "core_id").read().strip()))
        except OSError:
            phys.add(("?", str(c)))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return len(aff), len(phys), quota


def baseline_procs():
    n_aff, n_phys, quota = host_cores()
    procs = n_phys if quota is None else max(1, min(n_phys, int(quota)))
    note = (f"affinity {n_aff} logical CPUs, {n_phys} physical cores"
            + (f", cgroup quota {quota:g} CPUs" if quota is not None else ", no cgroup quota")
            + f"; {procs} used ({cpu_model()})")
    return procs, note


def cpu_baseline(w, target_s=12.0, threads=None):
    """Oracle (C restatement, OpenMP over host cores) on a bounded sample of the same
    workload: a block of whole columns cut out of the grid.  Rank 0, N=1 only."""
    from helpers import oracle
    lib = oracle()
    note = ""
    if threads is None:
        threads, note = baseline_procs()
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build()

    def run(nb):
        j0, i0 = w.ny // 2 - nb // 2, w.nx // 2 - nb // 2
        sub = lambda a: np.ascontiguousarray(a[..., j0:j0 + nb, i0:i0 + nb])  # noqa: E731
        var = sub(w.var).copy()
        slab = abi.make_slab(sub(w.x), sub(w.y), sub(w.alt), var)
        st = abi.Stats()
        t0 = time.perf_counter()
        rc = lib.orc_analyze_var(w.k, 0, -5.0, 0, C.byref(ob), C.byref(w.vp), C.byref(slab),
                                 threads, C.byref(st))
        dt = time.perf_counter() - t0
        assert rc == 0
        return dt, st, nb * nb * w.nz

    dt, st, pts = run(4)
    nb = 4
    for _ in range(2):  # size the block for ~target_s of CPU work (small blocks run faster)
        rate = pts / dt
        nb = int(max(4, min(w.nx, np.sqrt(target_s * rate / w.nz))))
        dt, st, pts = run(nb)
        if dt >= 0.8 * target_s or nb >= w.nx:
            break
    return {"value": pts / dt, "unit": "grid-points/s", "cores": threads, "kind": "port",
            "sample": f"{nb}x{nb} columns x {w.nz} levels = {pts} points of the {w.name} grid "
                      f"({dt:.1f} s), mean p={st.nobs_sum / max(st.solved, 1):.0f}, "
                      f"LAPACK={lib.orc_lapack_name().decode()}, {threads} OpenMP threads; "
                      f"{note}"}


REF_HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")


def _ref_driver_blob(w, i0, j0, nb):
    """Input of `ref_harness driver` (oracle/ref/ref_driver.inc:54-74) for the nb x nb columns
    at (i0, j0) of the workload: the slab in the reference's Fortran layouts and the one
    radar type with this variable's namelist parameters (radar error rides in err_muti(1),
    ref_driver.inc:477).  C-contiguous (.., ny, nx) arrays are Fortran (nx, ny, ..)."""
    sub = lambda a: np.ascontiguousarray(a[..., j0:j0 + nb, i0:i0 + nb])  # noqa: E731
    tp = w.vp.radar[w.radar_type - 1]
    i4 = lambda v: np.asarray(v, np.int32).tobytes()  # noqa: E731
    f4 = lambda v: np.asarray(v, np.float32).tobytes()  # noqa: E731
    n = w.obs.shape[0]
    return b"".join([
        i4([w.k, nb, nb, w.nz, nb, nb, 0, w.vp.use_rtpp, w.vp.use_rtps, 1]),
        f4([-5.0, w.vp.multi_infl, w.vp.rtpp_alpha, w.vp.rtps_alpha]),
        f4(sub(w.x)), f4(sub(w.y)), f4(sub(w.alt)), f4(sub(w.var)),
        i4([1, w.radar_type, 1, n, tp.use_it, tp.max_lz_pts] + list(tp.is_assim)),
        f4([tp.hclr, tp.vclr] + list(tp.err_muti) + list(tp.err_rej)),
        f4(w.obs_xyz), f4(w.obs), f4(w.hdxb)])


def cpu_baseline_reference(w, target_s=12.0, procs=None):
    """The reference's own compiled code (oracle/_ref/ref_harness: letkf_solve, kdtree2 and
    read_namelist built from /root/reference with amdflang + MKL dsyevd, the driver-loop glue
    restated line for line) timed on the host cores as the reference runs: flat, one
    single-threaded process per core (MPI ranks in the reference), each on its own block of
    whole columns of the same grid.  None when the harness was not built."""
    import subprocess
    import tempfile
    if not os.path.exists(REF_HARNESS):
        return None
    note = ""
    if procs is None:
        procs, note = baseline_procs()
    env = dict(os.environ, MKL_CBWR="COMPATIBLE", MKL_THREADING_LAYER="SEQUENTIAL",
               MKL_NUM_THREADS="1", OMP_NUM_THREADS="1")

    def run(nb, nproc):
        side = int(np.ceil(np.sqrt(nproc)))
        i00, j00 = w.nx // 2 - side * nb // 2, w.ny // 2 - side * nb // 2
        with tempfile.TemporaryDirectory() as td:
            jobs = []
            for p in range(nproc):
                d = os.path.join(td, str(p))
                os.mkdir(d)
                with open(os.path.join(d, "in.bin"), "wb") as f:
                    f.write(_ref_driver_blob(w, i00 + (p % side) * nb, j00 + (p // side) * nb, nb))
                jobs.append(d)
            t0 = time.perf_counter()
            ps = [subprocess.Popen([REF_HARNESS, "driver", "in.bin", "out.bin"], cwd=d, env=env,
                                   stdout=subprocess.DEVNULL) for d in jobs]
            rcs = [p.wait() for p in ps]
            dt = time.perf_counter() - t0
            if any(rcs):
                raise RuntimeError(f"ref_harness driver failed: {rcs}")
            out = np.fromfile(os.path.join(jobs[0], "out.bin"), np.float32)
            assert out.size == nb * nb * w.nz * w.k and np.isfinite(out).all()
        return dt, nproc * nb * nb * w.nz

    nb_max = w.nx // int(np.ceil(np.sqrt(procs)))
    run(2, 1)  # warm-up: the first launch on a fresh box pages in the runtime and MKL
    dt, pts = run(3, 1)  # one process, a 3x3-column block: the per-point time
    nb = 3
    for _ in range(2):  # size the blocks for ~target_s of work per process
        nb = int(max(2, min(nb_max, nb * np.sqrt(target_s / max(dt, 1e-3)))))
        dt, pts = run(nb, procs)
        if dt >= 0.7 * target_s or nb >= nb_max:
            break
    n_aff, n_phys, quota = host_cores()
    return {"value": pts / dt, "unit": "grid-points/s", "cores": procs, "kind": "reference",
            "per_core": pts / dt / procs,
            "physical_cores_in_affinity": n_phys,
            "extrapolated_all_physical_cores": pts / dt / procs * n_phys,
            "extrapolation_note": "per-core rate x the physical cores of the affinity set, for "
                                  "comparison only: the job's cgroup quota caps what can run "
                                  "at once" if quota is not None and quota < n_phys else
                                  "all physical cores were timed",
            "sample": f"{procs} single-threaded processes (the reference's flat MPI layout), "
                      f"each {nb}x{nb} columns x {w.nz} levels of the {w.name} grid: {pts} points "
                      f"in {dt:.1f} s; reference letkf_solve/kdtree2/read_namelist compiled with "
                      f"amdflang, MKL dsyevd (oracle/_ref/ref_harness driver); {note}"}


def time_transposes(core, w, k, rank, world, dev):
    """One letkf_scatter_grid + letkf_gather_grid of the whole variable (k members of
    nx x ny x nz fp32) through cwbl/transpose.py: HIP packing + RCCL point-to-point, the
    owned members held as one stacked tensor (one packing launch per transpose; on one rank
    the column layout is the member layout and var aliases the fields, no copy).  Members
    are dealt m % world; max over ranks of one timed pass after one warm-up.  The packing
    kernels alone are timed as well (pack_members / unpack_members of the owned members
    into a separate buffer, best of 5): their effective HBM rate, 2 x 4 B per element."""
    from cwbl import transpose as tr
    nx, ny, nz = w.extra["cfg"]["nx"], w.extra["cfg"]["ny"], w.nz
    t = tr.Transposer(core, k, nx, ny, device=dev)
    mine = t.owned()
    stk = torch.randn((len(mine), nz, ny, nx), device=dev)
    fields = {m: stk[i] for i, m in enumerate(mine)}
    ref = stk.clone()
    res = {}
    for it in range(2):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        var = t.scatter_grid(fields, nz)
        t1 = time.perf_counter()
        back = t.gather_grid(var, out=fields)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res = {"scatter_ms": (t1 - t0) * 1e3, "gather_ms": (t2 - t1) * 1e3}
    for i, m in enumerate(mine):
        assert torch.equal(back[m], ref[i]), "transpose round trip"
    n = nx * ny * nz
    buf = torch.empty((max(len(mine), 1), n), device=dev)
    px, py = t.dec.px, t.dec.py
    kern = {}
    for name, fn in (("pack", lambda: core.pack_members(stk, n, len(mine), nx, ny, nz, px, py, buf, n)),
                     ("unpack", lambda: core.unpack_members(buf, n, len(mine), nx, ny, nz, px, py, stk, n))):
        best = None
        for _ in range(5):
            torch.cuda.synchronize()
            a = time.perf_counter()
            fn()
            el = time.perf_counter() - a
            best = el if best is None else min(best, el)
        kern[f"{name}_ms"] = best * 1e3
        kern[f"{name}_gbs"] = 2 * 4 * n * len(mine) / best / 1e9
    if world > 1:
        v = torch.tensor([res["scatter_ms"], res["gather_ms"]], dtype=torch.float64, device=dev)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        res = {"scatter_ms": float(v[0]), "gather_ms": float(v[1])}
    gb = k * nx * ny * nz * 4 / 1e9
    res.update(variable_gb=gb, px_py=list(tr.dims_create(world)),
               scatter_gbs=gb / max(res["scatter_ms"] * 1e-3, 1e-9),
               gather_gbs=gb / max(res["gather_ms"] * 1e-3, 1e-9),
               kernels_rank0=dict(kern, members=len(mine),
                                  note="one launch over the owned members, host wall time of "
                                       "the synchronous call (launch + sync included)"),
               aliased=world == 1)
    return res


# input.nml's var_update (:7) and multi_infl (:162), with the slab each variable takes in
# letkf_driver (module_letkf_core.f90:70-81, 90-158): U has nx+1 columns and V ny+1 rows of
# which only the mass-grid ones are analysed (Q2, :209-210; mass-point altitude, :192-193);
# W and PH have nz+1 levels; MU one; QVAPOR and the hydrometeors get letkf_tune_q (:252-278).
CYCLE = (("U", 1.6, "u"), ("V", 1.6, "v"), ("W", 1.6, "w"), ("T", 1.6, "m"),
         ("QVAPOR", 1.6, "q"), ("QRAIN", 1.1, "q"), ("QSNOW", 1.1, "q"), ("QGRAUP", 1.1, "q"),
         ("QHAIL", 1.1, "q"), ("QNRAIN", 1.1, "q"), ("QNSNOW", 1.1, "q"),
         ("QNGRAUPEL", 1.1, "q"), ("QNHAIL", 1.1, "q"), ("MU", 1.1, "mu"), ("P", 1.1, "m"),
         ("PH", 1.1, "w"))
# (transpose stagger, levels above nz) of each slab kind (module_letkf_core.f90:70-81)
KINDS = {"u": (1, 0), "v": (2, 0), "w": (0, 1), "m": (0, 0), "q": (0, 0), "mu": (0, None)}


def _kind_slab(kind, x, y, alt, lx, ly):
    """(x, y, alt) of a variable's slab on this rank's columns: U/V take one more staggered
    column/row where the rank holds one (loc_nx_u / loc_ny_v), with mass-point altitude (Q2);
    W/PH one level above the top; MU the lowest level."""
    ny, nx = x.shape
    xs, ys, al = x, y, alt
    if kind == "u" and lx > nx:
        xs = torch.cat([x, x[:, -1:] + 2e3], 1).contiguous()
        ys = torch.cat([y, y[:, -1:]], 1).contiguous()
    elif kind == "v" and ly > ny:
        xs = torch.cat([x, x[-1:]], 0).contiguous()
        ys = torch.cat([y, y[-1:] + 2e3], 0).contiguous()
    elif kind == "w":
        al = torch.cat([alt, alt[-1:] + 400.0], 0).contiguous()
    elif kind == "mu":
        al = alt[:1].contiguous()
    return xs, ys, al


def time_cycle(core, w, rank, world, dev, x, y, alt, transposes=True):
    """Wall-clock of one analysis cycle on this rank: every var_update entry
    of input.nml, each as letkf_driver runs it (module_letkf_core.f90:59-297) —
    letkf_scatter_grid (member -> column transpose, module_mpi_util.f90:262), the analysis of
    this rank's columns, letkf_gather_grid (column -> member, :325) — and then write_mean's
    ensemble mean of the analysed fields (module_grid.f90:700-840, one RCCL reduce).  The
    members are dealt m % world (k/world per rank on an 8-GPU node); the transposes are the
    HIP packing kernels + RCCL point-to-point (cwbl/transpose.py).  One obs type, so the k-d
    trees are built once and shared (the tree cache, as for variables of equal localisation).
    Member fields are synthetic N(0,1) in HBM before the timed region (the cost does not
    depend on the values).  No file I/O.  Max over ranks."""
    from cwbl import transpose as tr
    cfg, k, nz = w.extra["cfg"], w.k, w.nz
    nxg, nyg = cfg["nx"], cfg["ny"]
    t = tr.Transposer(core, k, nxg, nyg, device=dev)
    lx0, ly0 = t.local_shape(0)
    assert (ly0, lx0) == tuple(x.shape), ((ly0, lx0), tuple(x.shape))
    fields, slabs, runs = {}, {}, []
    for kind, (stg, up) in KINDS.items():
        nzv = 1 if up is None else nz + up
        gx, gy = t.dec.grid(stg)
        if transposes:  # the owned members' fields as one stacked tensor
            stk = torch.randn((len(t.owned()), nzv, gy, gx), device=dev)
            fields[kind] = {m: stk[i] for i, m in enumerate(t.owned())}
        lx, ly = t.local_shape(stg)
        slabs[kind] = (nzv, stg, lx, ly, _kind_slab(kind, x, y, alt, lx, ly),
                       None if transposes else torch.randn((k, nzv, ly, lx), device=dev))
    for name, infl, kind in CYCLE:
        vp = synth.radar_var_params(cfg["hclr"], cfg["vclr"], cfg["max_lz"], cfg["err"],
                                    cfg["err_rej"], cfg["radar_type"], multi_infl=infl)
        vp.tune_q = 1 if kind == "q" else 0
        runs.append((name, kind, vp))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    per, ms_sc, ms_an, ms_ga = {}, 0.0, 0.0, 0.0
    t0 = time.perf_counter()
    for name, kind, vp in runs:
        nzv, stg, lx, ly, (xs, ys, al), var = slabs[kind]
        ta = time.perf_counter()
        if transposes:
            var = t.scatter_grid(fields[kind], nzv, stg)
        tb = time.perf_counter()
        core.analyze_var(vp, abi.make_slab(xs, ys, al, var, memory=abi.MEM_DEVICE,
                                           ix_lim=lx0, iy_lim=ly0))
        tc = time.perf_counter()
        if transposes:
            t.gather_grid(var, stg, out=fields[kind])
            torch.cuda.synchronize()
        td = time.perf_counter()
        ms_sc += (tb - ta) * 1e3
        ms_an += (tc - tb) * 1e3
        ms_ga += (td - tc) * 1e3
        per[name] = round((td - ta) * 1e3, 2)
    tm = time.perf_counter()
    if transposes:  # write_mean: every analysed field of the owned members, one reduce
        t.write_mean({m: [fields[kind][m] for _, kind, _ in runs] for m in t.owned()})
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    vals = _max_over_ranks([(t1 - t0) * 1e3, ms_sc, ms_an, ms_ga, (t1 - tm) * 1e3], world, dev)
    return {"cycle_ms": vals[0], "variables": len(CYCLE),
            "scatter_ms": vals[1], "analysis_ms": vals[2], "gather_ms": vals[3],
            "write_mean_ms": vals[4], "transposes": transposes,
            "per_variable_ms_rank0": per,
            "note": "input.nml var_update on this configuration's grid and obs set, per "
                    "variable letkf_scatter_grid (HIP pack + RCCL point-to-point) -> "
                    "cwbl_analyze_var -> letkf_gather_grid, then write_mean (member sums + "
                    "one reduce); U/V staggered (Q2), W/PH nz+1 levels, MU 1 level, tune_q on "
                    "the Q species; no file I/O; component times are max over ranks"
                    if transposes else
                    "analysis only (--no-transposes): no member<->column transposes"}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def _max_over_ranks(vals, world, dev, op=None):
    if world == 1:
        return vals
    t = torch.tensor(vals, dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=op or dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


def time_config(name, rank, world, local, dev, steps, warmup):
    """One of BASELINE.json's other configurations timed like the headline one (detail only):
    this rank's columns of the configuration's grid in HBM, the obs set broadcast once (RCCL
    at N > 1), `warmup` + `steps` cwbl_analyze_var calls, max over ranks.  configs[3] (C4,
    k = 128) and configs[4] (C5, dense radar on 600 x 600 x 60)."""
    w = synth.make(name, shard=(rank, world) if world > 1 else None, local_noise=True)
    types = [dict(family=1, type_id=w.radar_type, xyz=w.obs_xyz, obs=w.obs, hdxb=w.hdxb)]
    if world > 1:
        # one RCCL broadcast: every rank knows the set's layout (the counts)
        _, types = cdist.broadcast_obs_set(types if rank == 0 else None, w.k, dev, src=0,
                                           layout=cdist.wire_layout(types))
    else:
        _, types = cdist.unpack_obs_set(torch.from_numpy(cdist.pack_obs_set(types, w.k)).to(dev))
    x, y, alt, var = (torch.from_numpy(a).to(dev) for a in (w.x, w.y, w.alt, w.var))
    del w.var
    core = abi.Core(w.k, device=local, options=CORE_OPTIONS)
    core.set_obs(cdist.builder_from(types, abi.MEM_DEVICE).build())
    slab = abi.make_slab(x, y, alt, var, memory=abi.MEM_DEVICE)
    for _ in range(warmup):
        core.analyze_var(w.vp, slab)
    core.set_kernel_timing(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    stats = [core.analyze_var(w.vp, slab) for _ in range(steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    ktimes = core.kernel_times()
    solved = sum(s.solved for s in stats)
    nobs = sum(s.nobs_sum for s in stats)
    ms_solve = sum(s.ms_solve for s in stats)
    roof, per_kernel = roofline_block(ktimes, w.k, solved, nobs, ms_solve, name)
    if roof is not None:
        roof["hbm"] = hbm_block(name, w.k, float(sum(s.points for s in stats)) / steps,
                                el / steps * 1e3)
    el, pts, sol, nsum = _max_over_ranks([el], world, dev) + _max_over_ranks(
        [float(sum(s.points for s in stats)), float(solved), float(nobs)], world, dev,
        dist.ReduceOp.SUM if world > 1 else None)
    core.finalize()
    cfg = w.extra["cfg"]
    return {"workload": f"{name}: {cfg['nx']}x{cfg['ny']}x{cfg['nz']} grid, k={w.k}, "
                        f"{cfg['n_obs']} obs (hclr {cfg['hclr']} km, vclr {cfg['vclr']} km), "
                        f"max_lz_pts {cfg['max_lz']}",
            "value": pts / el, "unit": "grid-points/s", "ms_per_step": el / steps * 1e3,
            "steps": steps, "warmup": warmup, "ranks": world,
            "mean_p": nsum / max(sol, 1),
            "nonconverged": sum(s.nonconverged for s in stats),
            "roofline_rank0": roof, "kernels_rank0": per_kernel}


def time_host_memory(w, local, steps, warmup, pinned):
    """The headline configuration with the slab in HOST memory (MEM_HOST): every call copies
    x, y, alt and the 720 MB var in, analyses, and copies var back (BASELINE.md §4's
    PCIe-inclusive definition).  `pinned`: page-locked host arrays (torch pin_memory), else
    ordinary pageable numpy arrays as a Fortran host would pass them.  Detail only; never
    `value`."""
    if pinned:
        def host(a):
            t = torch.empty(a.shape, dtype=torch.float32, pin_memory=True)
            t.copy_(torch.from_numpy(a))
            return t.numpy()
    else:
        def host(a):
            return np.array(a, np.float32, copy=True)
    x, y, alt, var = (host(a) for a in (w.x, w.y, w.alt, w.var))
    core = abi.Core(w.k, device=local)
    core.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
    slab = abi.make_slab(x, y, alt, var)
    for _ in range(warmup):
        core.analyze_var(w.vp, slab)
    t0 = time.perf_counter()
    stats = [core.analyze_var(w.vp, slab) for _ in range(steps)]
    el = time.perf_counter() - t0
    core.finalize()
    return {"value": sum(s.points for s in stats) / el, "unit": "grid-points/s",
            "ms_per_step": el / steps * 1e3, "steps": steps,
            "ms_copy_per_step": sum(s.ms_copy for s in stats) / steps,
            "host_arrays": "pinned (page-locked)" if pinned else "pageable numpy",
            "bytes_per_step": int(x.nbytes + y.nbytes + alt.nbytes + 2 * var.nbytes)}


def self_launch(n):
    """Run this script as n ranks under torch.distributed.run (one process per GPU, rendezvous
    on 127.0.0.1) and return their exit status.  The caller has not initialised HIP: the
    ranks are fresh child processes, nothing is exec'd in place."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    return subprocess.call(cmd)


# ---- roofline accounting -----------------------------------------------------------------------
# Algorithmic FP64 flops of each solve kernel: the terms of SURVEY.md §8(d)'s F(k,p) that the
# kernel's part of the algorithm must execute, per solved point with p accepted obs:
#   syrk + Yb d        p k(k+1) + 2pk     (module_letkf_core.f90:649, 651)
#   tridiagonalisation sum over steps j of 4 n_j^2, n_j = k-1-j  (dsytd2: 4k^3/3 in all)
#   reflectors on b1, x' and back      3 x 2k^2
# (the eigendecomposition F prices at 13k^3 is never formed: the kernels apply A^-1 and
# A^-1/2 to two vectors through T = Q^T A Q and a quadrature)
def _tri_flops(k, j0, j1):
    return sum(4 * (k - 1 - j) ** 2 for j in range(j0, min(j1, k - 1)))


# cwbl_set_option values for every Core the bench makes (--big-path)
CORE_OPTIONS = {}


def kernel_algorithmic_flops(name, k, solved, nobs_sum):
    syrk = nobs_sum * (k * (k + 1) + 2 * k)
    vec = solved * 6 * k * k
    if name.startswith("assemble_record_kernel"):
        return syrk
    if name.startswith("solve_tq40_kernel"):
        return solved * _tri_flops(k, 0, k) + vec
    if name.startswith("solve_tq_big_kernel") and name.count(",") == 2:  # hand-off kernel
        j0 = int(name.split(",")[2].strip(" >"))
        return syrk + solved * _tri_flops(k, 0, j0)
    if name.startswith("solve_tq_rows_kernel"):  # half-row hand-off kernel <KP, J0>
        j0 = int(name.split(",")[1].strip(" >"))
        return syrk + solved * _tri_flops(k, 0, j0)
    if name.startswith("solve_tqb_tail_kernel"):
        j0 = int(name.split(",")[1].strip(" >"))
        return solved * _tri_flops(k, j0, k) + vec
    if name.startswith("solve_tq_kernel") or name.startswith("solve_tq_big_kernel"):
        return syrk + solved * _tri_flops(k, 0, k) + vec
    if name.startswith("solve_kernel"):  # Jacobi: the eigendecomposition itself
        return synth.flops_total(k, solved, nobs_sum)
    return None


def load_pmc(config):
    """Committed per-kernel PMC figures of `config` (profiles/pmc_kernels.json, written by
    scripts/pmc_kernels.py from rocprofv3 passes): HBM bytes and executed FP64 flops per
    launch, points per launch."""
    path = os.path.join(REPO, "profiles", "pmc_kernels.json")
    if not os.path.exists(path):
        return {}, None
    with open(path) as f:
        pm = json.load(f)
    return pm.get("configs", {}).get(config, {}), pm.get("tag")


def roofline_block(ktimes, k, solved, nobs_sum, ms_solve, config):
    """`roofline` of the dominant kernel (largest summed HIP-event time over the timed steps):
    its algorithmic FP64 flops / its summed launch time; plus the solve kernels together
    (algorithmic over the solve span), the reference-equivalent F rate and the PMC-executed
    rates as detail."""
    pmc, tag = load_pmc(config)
    per = {}
    for name, t in ktimes.items():
        alg = kernel_algorithmic_flops(name, k, solved, nobs_sum)
        e = {"launches": t["launches"], "points": t["points"], "ms": t["ms"],
             "avg_launch_ms": t["ms"] / max(t["launches"], 1)}
        if alg is not None and t["ms"] > 0:
            e["algorithmic_tflops"] = alg / (t["ms"] * 1e-3) / 1e12
            e["algorithmic_frac"] = e["algorithmic_tflops"] / FP64_PEAK_TFLOPS
        pk = pmc.get(name)
        if pk and t["ms"] > 0 and pk.get("fp64_flops_per_point"):
            ex = pk["fp64_flops_per_point"] * t["points"] / (t["ms"] * 1e-3) / 1e12
            e["executed_tflops"] = ex
            e["executed_frac"] = ex / FP64_PEAK_TFLOPS
        per[name] = e
    solve = {n: e for n, e in per.items() if "algorithmic_tflops" in e}
    if not solve:
        return None, per
    dom = max(solve, key=lambda n: solve[n]["ms"])
    d = solve[dom]
    alg_all = sum(kernel_algorithmic_flops(n, k, solved, nobs_sum) for n in solve)
    F = synth.flops_total(k, solved, nobs_sum)
    pk = pmc.get(dom, {})
    roof = {
        "bound": "mfma",
        "achieved": d["algorithmic_tflops"],
        "peak": FP64_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": d["algorithmic_frac"],
        "traffic": pk.get("hbm_bytes_per_launch"),
        "kernel": dom,
        "launches": d["launches"],
        "avg_launch_ms": d["avg_launch_ms"],
        "note": "dominant kernel (largest summed HIP-event time, events on its own stream): "
                "algorithmic FP64 flops of its part of letkf_solve (SURVEY.md 8(d) terms: "
                "syrk + Yb d for the assembly; 4k^3/3 tridiagonalisation + 6k^2 for the "
                "reflector solve) / its summed launch time; traffic = PMC HBM bytes per launch "
                f"(profiles/pmc_kernels.json, {tag})",
        "solve_kernels": {
            "kernels": sorted(solve),
            "algorithmic_tflops": alg_all / (ms_solve * 1e-3) / 1e12 if ms_solve > 0 else None,
            "note": "all solve kernels' algorithmic flops / the solve span (ms_solve)"},
        "reference_equivalent_F": {
            "tflops": F / (ms_solve * 1e-3) / 1e12 if ms_solve > 0 else None,
            "note": "F(k,p) of SURVEY.md 8(d) (13k^3 for dsyevd + the two k^3 products, never "
                    "executed here) / the solve span: not a hardware rate"},
    }
    ex = [(n, e) for n, e in solve.items() if "executed_tflops" in e]
    if len(ex) == len(solve) and ms_solve > 0:
        tot = sum(pmc[n]["fp64_flops_per_point"] * per[n]["points"] for n in solve)
        roof["executed"] = {"tflops": tot / (ms_solve * 1e-3) / 1e12,
                            "frac": tot / (ms_solve * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                            "note": f"PMC-counted FP64 work ({tag}) of the solve kernels per "
                                    "point x points / the solve span"}
    return roof, per


def hbm_block(config, k, points_per_step, ms_per_step):
    """The step's HBM fraction (north_star asks for the throughput "as fraction of the HBM
    roofline"; SURVEY.md 8(d) says to report it beside the FP64 one): the PMC HBM bytes of
    every kernel of one profiled step (profiles/pmc_kernels.json: FETCH_SIZE / WRITE_SIZE per
    launch x launches, gfx950-corrected) / the live ms_per_step / 8 TB/s, and the unique-bytes
    fraction 4 (2k + 3) B per point (xb in, xa out, coordinates) / ms_per_step / 8 TB/s."""
    pmc, tag = load_pmc(config)
    steps = max(int(pmc.get("_meta", {}).get("steps", 1)), 1)  # steps in the profiled run
    kern = {n: e for n, e in pmc.items() if isinstance(e, dict) and "hbm_bytes_per_launch" in e}
    if not kern or not ms_per_step:
        return None
    per_step = sum(e["hbm_bytes_per_launch"] * e.get("calls", 0) for e in kern.values()) / steps
    sec = ms_per_step * 1e-3
    uniq = 4.0 * (2 * k + 3) * points_per_step
    return {"pmc_bytes_per_step": per_step,
            "achieved_gbs": per_step / sec / 1e9,
            "peak_gbs": HBM_PEAK_GBS,
            "frac": per_step / sec / 1e9 / HBM_PEAK_GBS,
            "unique_bytes_per_step": uniq,
            "unique_gbs": uniq / sec / 1e9,
            "unique_frac": uniq / sec / 1e9 / HBM_PEAK_GBS,
            "by_kernel_bytes_per_step": {n: e["hbm_bytes_per_launch"] * e.get("calls", 0) / steps
                                         for n, e in sorted(kern.items())},
            "note": f"PMC bytes of every kernel of one profiled step ({tag}, "
                    "profiles/pmc_kernels.json) over the live ms_per_step; the path is FP64-bound "
                    "(SURVEY.md 8(d)), so neither fraction is the roofline it is held to"}


def distinct_devices(world, dev):
    """GPUs the ranks run on (under gloo several ranks may share one)."""
    if world == 1:
        return 1
    t = torch.tensor([dev.index], dtype=torch.int64, device=dev)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return len({int(v.item()) for v in out})


class Stage:
    """The part of the run in progress, for the error line a failure prints (CWBL_BENCH_FAIL_AT
    = <stage name> raises there: the tests' failure injection)."""

    def __init__(self):
        self.name = "setup"

    def __call__(self, name):
        self.name = name
        if os.environ.get("CWBL_BENCH_FAIL_AT") == name:
            raise RuntimeError(f"injected failure at stage {name!r} (CWBL_BENCH_FAIL_AT)")


def error_line(args, rank, world, stage, exc):
    """The JSON line of a run that failed: the contract's keys with value null, the exception
    and the stage it was raised in (a first RCCL run that fails still reports)."""
    return {"metric": METRIC, "value": None, "unit": "grid-points/s", "n_gpus": args.gpus,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": None,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic", "config": {"workload": args.config, "ranks": world},
            "roofline": None, "cpu_baseline": None,
            "error": repr(exc), "stage": stage.name, "rank": rank}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-transposes", action="store_true",
                    help="cycle without the member<->column transposes and write_mean")
    ap.add_argument("--no-cycle", action="store_true",
                    help="skip the wall-clock-per-cycle detail (16 var_update entries)")
    ap.add_argument("--no-detail-configs", action="store_true",
                    help="skip the C4 / C5 / host-memory detail legs")
    ap.add_argument("--big-path", type=int, choices=(0, 1), default=None,
                    help="CWBL_OPT_BIG_PATH for k > 64 (default: the library's, 1 = hand-off; "
                         "0 = one 256-thread kernel)")
    args = ap.parse_args()
    if args.big_path is not None:
        CORE_OPTIONS["big_path"] = args.big_path

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` without a launcher: start the N ranks ourselves, before
        # this process touches the GPU (it never initialises HIP; it only waits)
        sys.exit(self_launch(args.gpus))

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; refusing to time "
              f"{world} rank(s) as {args.gpus} GPU(s)", file=sys.stderr, flush=True)
        sys.exit(2)
    stage = Stage()
    try:
        run(args, rank, world, stage)
    except Exception as e:  # noqa: BLE001
        import traceback
        traceback.print_exc()
        print(f"bench.py rank {rank}: failed in stage {stage.name}: {e!r}", file=sys.stderr,
              flush=True)
        if rank == 0:
            print(json.dumps(error_line(args, rank, world, stage, e)), flush=True)
        sys.exit(1)


def run(args, rank, world, stage):
    stage("device")
    backend = os.environ.get("CWBL_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()  # (does not initialise HIP on this image)
    if world > 1 and backend == "nccl" and ndev < world:
        raise RuntimeError(f"{world} ranks need {world} distinct GPUs with RCCL, {ndev} visible "
                           f"(CWBL_DIST_BACKEND=gloo rehearses several ranks on one GPU)")
    # (gloo rehearsal only: ranks share the visible GPUs modulo their count)
    local = int(os.environ.get("LOCAL_RANK", 0)) % max(ndev, 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        stage("process_group")
        import datetime
        # RCCL over xGMI; CWBL_DIST_BACKEND=gloo rehearses the multi-rank path on one GPU.  A
        # bounded timeout: a rank that dies leaves the others an exception, not a hang
        tmo = datetime.timedelta(minutes=10)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
    n_dev = distinct_devices(world, dev)

    stage("synthesis")
    w = synth.make(args.config, shard=(rank, world) if world > 1 else None)
    k = w.k
    # ---- observation set: packed on rank 0 (obs-set wire format), broadcast over RCCL --------
    stage("obs_broadcast")
    n = w.obs.shape[0]
    types = [dict(family=1, type_id=w.radar_type, xyz=w.obs_xyz, obs=w.obs, hdxb=w.hdxb)]
    bcast_ms = 0.0
    if world > 1:
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        _, types = cdist.broadcast_obs_set(types if rank == 0 else None, k, dev, src=0,
                                           layout=cdist.wire_layout(types))
        torch.cuda.synchronize()
        bcast_ms = (time.perf_counter() - t0) * 1e3
    else:
        _, types = cdist.unpack_obs_set(torch.from_numpy(cdist.pack_obs_set(types, k)).to(dev))
    # ---- slab in HBM ---------------------------------------------------------------------------
    stage("core_init")
    x, y, alt = (torch.from_numpy(a).to(dev) for a in (w.x, w.y, w.alt))
    var = torch.from_numpy(w.var).to(dev)
    torch.cuda.synchronize()

    core = abi.Core(k, device=local, options=CORE_OPTIONS)
    core.set_obs(cdist.builder_from(types, abi.MEM_DEVICE).build())
    slab = abi.make_slab(x, y, alt, var, memory=abi.MEM_DEVICE)

    stage("warmup")
    for _ in range(args.warmup):
        core.analyze_var(w.vp, slab)
    core.set_kernel_timing(os.environ.get("CWBL_BENCH_KT", "1") != "0")
    stage("timed")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = []
    for _ in range(args.steps):
        stats.append(core.analyze_var(w.vp, slab))
    torch.cuda.synchronize()
    t_rank = time.perf_counter() - t0  # this rank's own analysis time (load balance)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ktimes = core.kernel_times()
    core.set_kernel_timing(False)

    stage("reduce")
    pts_local = sum(s.points for s in stats)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        p = torch.tensor([pts_local], dtype=torch.float64, device=dev)
        dist.all_reduce(p, op=dist.ReduceOp.SUM)
        elapsed, pts_total = float(t.item()), float(p.item())
        tr_ = torch.tensor([t_rank / args.steps * 1e3, float(pts_local) / args.steps],
                           dtype=torch.float64, device=dev)
        allr = [torch.zeros_like(tr_) for _ in range(world)]
        dist.all_gather(allr, tr_)
        rank_ms = [float(v[0]) for v in allr]
        rank_pts = [int(v[1]) for v in allr]
    else:
        pts_total = float(pts_local)
        rank_ms, rank_pts = [t_rank / args.steps * 1e3], [int(pts_local / args.steps)]
    per_rank = {"ms_per_step": rank_ms, "points_per_step": rank_pts,
                "min_ms": min(rank_ms), "max_ms": max(rank_ms),
                "imbalance": max(rank_ms) / min(rank_ms) if min(rank_ms) > 0 else None,
                "note": "each rank's own wall time of the timed steps (before the closing "
                        "barrier); `value` uses the max over ranks"}

    def guarded(fn, *a, **kw):
        # a detail leg that fails is reported in `detail`, never at the cost of the JSON line
        try:
            return fn(*a, **kw)
        except Exception as e:  # noqa: BLE001
            print(f"bench.py rank {rank}: {fn.__name__} failed: {e!r}", file=sys.stderr,
                  flush=True)
            return {"error": repr(e)}

    stage("detail")
    tr_detail = None if args.no_transposes else guarded(time_transposes, core, w, k, rank,
                                                        world, dev)
    cycle = None if args.no_cycle else guarded(time_cycle, core, w, rank, world, dev, x, y, alt,
                                               transposes=not args.no_transposes)
    legs = {}
    if not args.no_detail_configs and args.config == "c2":
        # the other configurations on the same clock (detail; the library is re-initialised
        # per leg, so the headline core is finished first)
        del slab, var
        core.finalize()
        torch.cuda.empty_cache()
        legs["c4"] = guarded(time_config, "c4", rank, world, local, dev, steps=2, warmup=1)
        torch.cuda.empty_cache()
        legs["c5"] = guarded(time_config, "c5", rank, world, local, dev, steps=2, warmup=1)
        torch.cuda.empty_cache()
        if world == 1:
            legs["host_memory"] = {
                "pageable": guarded(time_host_memory, w, local, steps=3, warmup=1, pinned=False),
                "pinned": guarded(time_host_memory, w, local, steps=3, warmup=1, pinned=True)}
        core = abi.Core(k, device=local)  # (finalised below)

    stage("report")
    if rank == 0:
        solved = sum(s.solved for s in stats)
        nobs_sum = sum(s.nobs_sum for s in stats)
        ms_solve = sum(s.ms_solve for s in stats)
        ms_search = sum(s.ms_search for s in stats)
        roof, per_kernel = roofline_block(ktimes, k, solved, nobs_sum, ms_solve, args.config)
        if roof is not None:
            roof["hbm"] = hbm_block(args.config, k, pts_total / args.steps,
                                    elapsed / args.steps * 1e3)
        hm = legs.get("host_memory") or {}
        pageable = hm.get("pageable") or {}
        out = {
            "metric": METRIC,
            "value": pts_total / elapsed,
            "unit": "grid-points/s",
            "n_gpus": n_dev,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": f"{args.config}: {w.extra['cfg']['nx']}x{w.extra['cfg']['ny']}x{w.nz} grid, k={k}, "
                            f"{n} {'radar-dbz' if w.radar_type == abi.RADAR_DBZ else 'radar-VR'}-like obs (hclr {w.extra['cfg']['hclr']} km, vclr "
                            f"{w.extra['cfg']['vclr']} km), RTPP+RTPS, Gaussian localisation",
                "grid_points": int(w.extra["cfg"]["nx"] * w.extra["cfg"]["ny"] * w.nz),
                "k": k,
                "n_obs": n,
                "mean_p": nobs_sum / max(solved, 1),
                "ranks": world,
                "slab": "device-resident: var(nx,ny,nz,0:k-1) in HBM before the timed region, as "
                        "the device member->column transposes (cwbl/transpose.py) leave it; the "
                        "PCIe-inclusive rate of a pageable host slab is value_host_pageable",
                "parallelism": f"column-sharded x{world} (px x py = "
                               f"{'x'.join(map(str, tr_dims(world)))})" + (
                    ", obs-set broadcast over " + ("RCCL" if dist.get_backend() == "nccl"
                                                  else dist.get_backend())
                    if world > 1 else ""),
            },
            "value_host_pageable": pageable.get("value"),
            "roofline": roof,
            "detail": {
                "solver": "householder+quadrature",
                "per_rank": per_rank,
                "kernels_rank0": per_kernel,
                "solved_per_step": solved / args.steps,
                "ms_solve_per_step": ms_solve / args.steps,
                "ms_search_per_step": ms_search / args.steps,
                "ms_prep_per_step": sum(s.ms_prep for s in stats) / args.steps,
                # decade of the quadrature rule's spectrum bound
                "max_quad_level": max(s.max_sweeps for s in stats),
                "mean_quad_level": sum(s.sweeps_sum for s in stats) / max(solved, 1),
                "nonconverged": sum(s.nonconverged for s in stats),
                "obs_bcast_ms": bcast_ms,
                "transposes": tr_detail,
                "cycle": cycle,
                **legs,
            },
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            # the reference's own compiled path when it travelled with the tree (built in
            # the container that has /root/reference), else the C restatement (port)
            ref = guarded(cpu_baseline_reference, w)
            port = guarded(cpu_baseline, w)
            ref = ref if ref and "error" not in ref else None
            out["cpu_baseline"] = ref or port
            if ref:
                out["detail"]["cpu_baseline_port"] = port
                # round 3's figure: 16 processes (the box's OMP_NUM_THREADS), for comparison
                if ref["cores"] != 16:
                    out["detail"]["cpu_baseline_16_procs"] = guarded(
                        cpu_baseline_reference, w, procs=16)
        print(json.dumps(out), flush=True)
    core.finalize()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
