#!/usr/bin/env python3
"""Generate tests/golden/* from the reference's own compiled code (oracle/_ref/ref_harness).

TEST INFRASTRUCTURE ONLY.  Run in the build container (where /root/reference and amdflang
exist):  python oracle/gen_goldens.py
Every fixture holds inputs AND the reference's outputs; the manifest records seeds, shapes
and provenance ("MKL dsyevd, amdflang -O2, x86-64 without FMA, glibc 2.35 expf(FMA)").

Fixtures
  G0 consts.npz            gc1999, gc1999**2 (module_param.f90:116, module_localization.f90:202)
  G1 solve_k{K}.npz        letkf_solve KATs (module_letkf_core.f90:598-700) + dsyevd eigenvalues
  G2 search_*.npz          build_tree/get_lz KATs on kdtree2 (module_localization.f90, module_kdtree2.f90)
  G3 gc.npz                Gaspari_Cohn_1999 (module_localization.f90:333-364)
  G4 driver_*.npz          one variable through the driver loop (module_letkf_core.f90:59-240)
  G5 tune_q.npz            letkf_tune_q KATs (module_letkf_core.f90:702-733), incl. Q3 columns
  G6 dims_create.json      MPI_Dims_create(n, 2) from the MPICH the reference links
                           (/opt/conda/lib/libmpi.so), as letkf_init calls it (module_mpi_util.f90:48-49)

`python oracle/gen_goldens.py tuneq` / `dims` regenerate only G5 / G6 (and their manifest entries).
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
HARNESS = os.path.join(HERE, "_ref", "ref_harness")
OUT = os.path.join(REPO, "tests", "golden")
ENV = dict(os.environ, MKL_CBWR="COMPATIBLE", MKL_THREADING_LAYER="SEQUENTIAL", MKL_NUM_THREADS="1")

i4 = np.int32
f4 = np.float32


def run(mode, blob):
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(fin, "wb") as f:
            f.write(blob)
        subprocess.run([HARNESS, mode, fin, fout], check=True, env=ENV, cwd=td)
        with open(fout, "rb") as f:
            return f.read()


def b(*arrs):
    return b"".join(np.ascontiguousarray(a).tobytes(order="F") if isinstance(a, np.ndarray)
                    else np.asarray(a).tobytes() for a in arrs)


# ------------------------------------------------------------------------------------- G1
def solve_cases(k, rng):
    ps = [1, k - 1, k, k + 1, 200, 2000]
    if k >= 64:
        ps = [1, k - 1, k, k + 1, 200]
    combos = [(1, 1), (0, 0), (1, 0), (0, 1)]
    out = []
    for p in ps:
        for rho in (1.1, 1.6):
            for (rp, rs) in combos:
                if p >= 2000 and (rp, rs) not in ((1, 1), (0, 0)):
                    continue
                if k >= 64 and (rp, rs) not in ((1, 1),):
                    continue
                npts = 1 if (p >= 2000 or k >= 64) else 2
                out.append((p, rho, rp, rs, npts))
    return out


def gen_solve(k, seed):
    rng = np.random.default_rng(seed)
    recs = dict(p=[], rho=[], rtpp=[], rtps=[], rtpp_a=[], rtps_a=[], xb=[], yo=[], yb=[],
                xa=[], lam=[])
    for (p, rho, rp, rs, npts) in solve_cases(k, rng):
        rtpp_a, rtps_a = f4(0.95), f4(0.85 if rp and rs else 0.95)
        pts = []
        for ip in range(npts):
            mu = 0.0 if ip % 2 == 0 else 285.0
            xb = (mu + rng.standard_normal(k) * 1.5).astype(f4)
            w = np.exp(-0.25 * rng.uniform(0, 13.3, p)).astype(f4)
            yb = (rng.standard_normal((k, p)) * 1.3 * w).astype(f4)
            yo = (rng.standard_normal(p) * 1.7 * w).astype(f4)
            pts.append((xb, yo, yb))
        blob = b(np.array([k, len(pts), rp, rs], i4), np.array([rho, rtpp_a, rtps_a], f4))
        for (xb, yo, yb) in pts:
            blob += b(np.array([p], i4), xb, yo, yb)
        raw = run("solve", blob)
        per = 4 * k + 8 * k
        assert len(raw) == per * len(pts)
        for ip, (xb, yo, yb) in enumerate(pts):
            chunk = raw[ip * per:(ip + 1) * per]
            recs["xa"].append(np.frombuffer(chunk[:4 * k], f4))
            recs["lam"].append(np.frombuffer(chunk[4 * k:], np.float64))
            recs["p"].append(p); recs["rho"].append(rho); recs["rtpp"].append(rp)
            recs["rtps"].append(rs); recs["rtpp_a"].append(rtpp_a); recs["rtps_a"].append(rtps_a)
            recs["xb"].append(xb); recs["yo"].append(yo); recs["yb"].append(yb.T.ravel())
    col_off = np.concatenate([[0], np.cumsum(recs["p"])]).astype(np.int64)
    return dict(
        k=np.int32(k), p=np.array(recs["p"], i4), col_off=col_off,
        multi_infl=np.array(recs["rho"], f4), use_rtpp=np.array(recs["rtpp"], i4),
        use_rtps=np.array(recs["rtps"], i4), rtpp_alpha=np.array(recs["rtpp_a"], f4),
        rtps_alpha=np.array(recs["rtps_a"], f4), xb=np.stack(recs["xb"]),
        yo=np.concatenate(recs["yo"]), yb=np.concatenate(recs["yb"]),  # (ncol, k) member fastest
        xa=np.stack(recs["xa"]), lam=np.stack(recs["lam"]))


# ------------------------------------------------------------------------------------- G2
def gen_search(name, seed, nobs, nq, hclr, vclr, max_lz, dup_frac=0.0, box_km=(120, 120, 15)):
    rng = np.random.default_rng(seed)
    xyz = np.empty((3, nobs), f4)
    xyz[0] = rng.uniform(0, box_km[0] * 1e3, nobs)
    xyz[1] = rng.uniform(0, box_km[1] * 1e3, nobs)
    xyz[2] = rng.uniform(0, box_km[2] * 1e3, nobs)
    ndup = int(dup_frac * nobs)
    if ndup:
        src = rng.integers(0, nobs, ndup)
        dst = rng.integers(0, nobs, ndup)
        xyz[:, dst] = xyz[:, src]
    q = np.empty((3, nq), f4)
    q[0] = rng.uniform(-10e3, (box_km[0] + 10) * 1e3, nq)
    q[1] = rng.uniform(-10e3, (box_km[1] + 10) * 1e3, nq)
    q[2] = rng.uniform(0, box_km[2] * 1e3, nq)
    q[:, :4] = xyz[:, :4]  # queries exactly on observations
    blob = b(np.array([nobs, nq, max_lz], i4), np.array([hclr, vclr], f4), xyz, q)
    raw = run("search", blob)
    rec = 4 + 8 * max_lz
    assert len(raw) == rec * nq
    nf = np.empty(nq, i4); idx = np.zeros((nq, max_lz), i4); r2 = np.zeros((nq, max_lz), f4)
    for iq in range(nq):
        c = raw[iq * rec:(iq + 1) * rec]
        nf[iq] = np.frombuffer(c[:4], i4)[0]
        idx[iq] = np.frombuffer(c[4:4 + 4 * max_lz], i4) - 1  # 0-based, -1 padding
        r2[iq] = np.frombuffer(c[4 + 4 * max_lz:], f4)
    for iq in range(nq):
        idx[iq, nf[iq]:] = -1
    return dict(obs_xyz=xyz.T.copy(), q_xyz=q.T.copy(), hclr=f4(hclr), vclr=f4(vclr),
                max_lz=np.int32(max_lz), nfound=nf, idx=idx, r2=r2)


# ------------------------------------------------------------------------------------- G4
GTS_NVAR = {1: 4, 2: 5, 8: 1, 10: 5, 11: 5}


def gen_driver(name, seed, k, nx, ny, nz, ix_lim, iy_lim, types, wf=0, norain=-5.0,
               multi_infl=1.6, rtpp=(1, 0.95), rtps=(1, 0.95), dx=2e3, ztop=12e3,
               xb_mu=0.0):
    """types: list of dicts(family, type_id, nobs, use_it, max_lz, hclr, vclr,
    err_muti[5], err_rej[5], is_assim[5], qc_bad_frac, norain_frac)"""
    rng = np.random.default_rng(seed)
    x = np.empty((nx, ny), f4); y = np.empty((nx, ny), f4)
    gx, gy = np.meshgrid(np.arange(nx) * dx, np.arange(ny) * dx, indexing="ij")
    x[:] = gx + rng.uniform(-50, 50, gx.shape); y[:] = gy + rng.uniform(-50, 50, gy.shape)
    alt = np.empty((nx, ny, nz), f4)
    lev = np.linspace(10.0, ztop, nz)
    alt[:] = lev[None, None, :] + rng.uniform(0, 30, (nx, ny, nz))
    var = (xb_mu + rng.standard_normal((nx, ny, nz, k)) * 1.2).astype(f4)
    blob = b(np.array([k, nx, ny, nz, ix_lim, iy_lim, wf, rtpp[0], rtps[0], len(types)], i4),
             np.array([norain, multi_infl, rtpp[1], rtps[1]], f4), x, y, alt, var)
    tstore = []
    ext = (nx * dx, ny * dx)
    for t in types:
        fam, tid, n = t["family"], t["type_id"], t["nobs"]
        nvar = GTS_NVAR[tid] if fam == 0 else 1
        xyz = np.empty((3, n), f4)
        xyz[0] = rng.uniform(-0.3 * ext[0], 1.3 * ext[0], n)
        xyz[1] = rng.uniform(-0.3 * ext[1], 1.3 * ext[1], n)
        xyz[2] = rng.uniform(0, ztop if t.get("upper", True) else 50.0, n)
        truth = rng.standard_normal((nvar, n)) * 2.0
        hdxb = (truth[:, :, None] + rng.standard_normal((nvar, n, k)) * 1.5).astype(f4)
        obs = (truth + rng.standard_normal((nvar, n)) * 1.0).astype(f4)
        gross = rng.uniform(0, 1, (nvar, n)) < t.get("gross_frac", 0.05)
        obs[gross] += f4(40.0)
        if fam == 1 and tid == 1:  # dbz: norain cases (module_letkf_core.f90:504-507)
            nr = rng.uniform(0, 1, n) < t.get("norain_frac", 0.2)
            obs[0, nr] = f4(norain)
            both = nr & (rng.uniform(0, 1, n) < 0.5)
            hdxb[0, both, :] = f4(norain)
        err = (0.5 + rng.uniform(0, 1.5, (nvar, n))).astype(f4)
        qc = np.zeros((nvar, n, k), i4)
        if fam == 0:
            bad = rng.uniform(0, 1, (nvar, n)) < t.get("qc_bad_frac", 0.1)
            qc[bad, :] = -1
            part = rng.uniform(0, 1, (nvar, n)) < 0.1
            qc[part, :] = np.where(rng.uniform(0, 1, (int(part.sum()), k)) < 0.5, -1, 0)
        hdr_i = np.array([fam, tid, nvar, n, t["use_it"], t["max_lz"]] + list(t["is_assim"]), i4)
        hdr_f = np.array([t["hclr"], t["vclr"]] + list(t["err_muti"]) + list(t["err_rej"]), f4)
        blob += b(hdr_i, hdr_f, xyz)
        if fam == 0:
            blob += b(obs, err, hdxb, qc)
        else:
            blob += b(obs[0], hdxb[0])
        tstore.append(dict(hdr_i=hdr_i, hdr_f=hdr_f, xyz=xyz.T.copy(), obs=obs.T.copy(),
                           error=err.T.copy(), hdxb=np.transpose(hdxb, (2, 1, 0)).copy(),
                           qc=np.transpose(qc, (2, 1, 0)).copy()))
    raw = run("driver", blob)
    var_out = np.frombuffer(raw, f4).reshape((nx, ny, nz, k), order="F")
    d = dict(k=np.int32(k), dims=np.array([nx, ny, nz, ix_lim, iy_lim], i4),
             ctl=np.array([wf, rtpp[0], rtps[0]], i4),
             ctl_f=np.array([norain, multi_infl, rtpp[1], rtps[1]], f4),
             x=x.T.copy(), y=y.T.copy(), alt=alt.T.copy(),          # C order (ny,nx) etc.
             var_in=np.transpose(var, (3, 2, 1, 0)).copy(),           # (k,nz,ny,nx)
             var_out=np.transpose(var_out, (3, 2, 1, 0)).copy(),
             ntypes=np.int32(len(types)))
    for it, t in enumerate(tstore):
        for key, v in t.items():
            d[f"t{it}_{key}"] = v
    return d


def T(family, type_id, nobs, hclr, vclr, max_lz, err_muti=1.0, err_rej=5.0, is_assim=1,
      use_it=1, **kw):
    em = err_muti if isinstance(err_muti, (list, tuple)) else [err_muti] * 5
    er = err_rej if isinstance(err_rej, (list, tuple)) else [err_rej] * 5
    ia = is_assim if isinstance(is_assim, (list, tuple)) else [is_assim] * 5
    d = dict(family=family, type_id=type_id, nobs=nobs, hclr=hclr, vclr=vclr, max_lz=max_lz,
             err_muti=em, err_rej=er, is_assim=ia, use_it=use_it)
    d.update(kw)
    return d


# ------------------------------------------------------------------------------------- G5
def gen_tuneq(seed):
    """q(nx,ny,nz,k) fields: mixed signs, all-zero columns (Q3: 0/0 -> NaN), all-negative
    columns (x/0 -> -inf, zeros -> NaN), all-positive columns, tiny and large magnitudes."""
    rng = np.random.default_rng(seed)
    cases = []
    for k, (nx, ny, nz) in ((8, (7, 5, 3)), (40, (6, 4, 2)), (128, (3, 3, 2))):
        q = rng.normal(0.0, 1.0, (nx, ny, nz, k)).astype(f4) * f4(1e-3)
        q[0, 0, 0, :] = 0.0                                   # Q3: all zero
        q[1, 0, 0, :] = -np.abs(q[1, 0, 0, :])                # no positive member
        q[1, 0, 0, 0] = 0.0
        q[2, 0, 0, :] = np.abs(q[2, 0, 0, :]) + f4(1e-4)      # all positive (ratio 1-ish)
        q[0, 1, 0, :] = q[0, 1, 0, :] * f4(1e-30)             # tiny
        q[1, 1, 0, :] = q[1, 1, 0, :] * f4(1e6)               # large
        q[2, 1, 0, ::3] = 0.0                                 # exact zeros mixed in
        if nz > 1:
            q[0, 0, 1, :] = np.where(np.arange(k) == k - 1, f4(5e-4), f4(-1e-4))  # one positive
        out = np.frombuffer(run("tuneq", b(np.array([k, nx, ny, nz], i4), q)), f4)
        cases.append((k, q, out.reshape((nx, ny, nz, k), order="F").copy()))
    d = {}
    for i, (k, q, o) in enumerate(cases):
        d[f"k{i}"] = np.int32(k)
        d[f"q_in{i}"] = q
        d[f"q_out{i}"] = o
    d["ncases"] = np.int32(len(cases))
    return d


def main_tuneq():
    d = gen_tuneq(501)
    np.savez_compressed(os.path.join(OUT, "tune_q.npz"), **d)
    mpath = os.path.join(OUT, "MANIFEST.json")
    with open(mpath) as f:
        manifest = json.load(f)
    manifest["files"]["tune_q.npz"] = {
        "what": "G5 letkf_tune_q KAT (source text of module_letkf_core.f90:702-733 with the "
                "cpu(myid)%loc_nx/loc_ny bounds replaced by size(q,1)/size(q,2))",
        "seed": 501, "ks": [int(d[f"k{i}"]) for i in range(int(d["ncases"]))],
        "nan_out": int(sum(np.isnan(d[f"q_out{i}"]).sum() for i in range(int(d["ncases"]))))}
    with open(mpath, "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(json.dumps(manifest["files"]["tune_q.npz"], indent=1))


def main_dims():
    """G6: MPICH's MPI_Dims_create(n, 2) for n = 1..128 (a singleton MPI_Init, no mpirun)."""
    import ctypes as C
    lib = C.CDLL(os.environ.get("MPI_LIB", "/opt/conda/lib/libmpi.so"), mode=C.RTLD_GLOBAL)
    assert lib.MPI_Init(None, None) == 0
    out = {}
    for n in range(1, 129):
        d = (C.c_int * 2)(0, 0)
        assert lib.MPI_Dims_create(n, 2, d) == 0
        out[str(n)] = [d[0], d[1]]
    lib.MPI_Finalize()
    with open(os.path.join(OUT, "dims_create.json"), "w") as f:
        json.dump({"source": "MPICH MPI_Dims_create(n, 2, dims) with dims = 0, "
                   "/opt/conda/lib/libmpi.so", "dims": out}, f, sort_keys=True)
    mpath = os.path.join(OUT, "MANIFEST.json")
    with open(mpath) as f:
        manifest = json.load(f)
    manifest["files"]["dims_create.json"] = {"what": "G6 MPI_Dims_create(n, 2), n = 1..128"}
    with open(mpath, "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


def driver_cases():
    gts5 = dict(err_muti=[0.5] * 5, err_rej=[5.0] * 5)
    return [
        # C1: 10x10x5, k=8, 50 synop obs at the surface (BASELINE.json configs[0])
        ("driver_c1.npz", 401, dict(k=8, nx=10, ny=10, nz=5, ix_lim=10, iy_lim=10,
          types=[T(0, 2, 50, 50.0, 3.0, 100, upper=False, **gts5)], ztop=6e3)),
        # mixed GTS + radar, truncation (max_lz small), QC/gross/norain rejects, Q2 bounds
        ("driver_mixed.npz", 402, dict(k=16, nx=12, ny=9, nz=6, ix_lim=11, iy_lim=9,
          types=[T(0, 1, 30, 75.0, 3.0, 12, err_muti=[0.5, 0.5, 0.7, 0.5, 0.5]),
                 T(0, 2, 40, 50.0, 3.0, 100, upper=False, is_assim=[1, 1, 0, 1, 1], **gts5),
                 T(0, 10, 25, 50.0, 3.0, 9, **gts5),
                 T(1, 1, 400, 8.0, 2.0, 30, err_muti=2.5, err_rej=20.0),
                 T(1, 2, 500, 12.0, 3.0, 300, err_muti=1.0, err_rej=8.0)])),
        # Gaspari-Cohn weighting, k = 40
        ("driver_gc_k40.npz", 403, dict(k=40, nx=8, ny=7, nz=5, ix_lim=8, iy_lim=6, wf=1,
          multi_infl=1.1, rtps=(0, 0.95),
          types=[T(0, 11, 30, 50.0, 3.0, 100, **gts5),
                 T(1, 2, 600, 12.0, 3.0, 300, err_muti=1.0, err_rej=8.0)])),
        # 2-D family (gpspw alone) + radar kdp in the other family
        ("driver_2d.npz", 404, dict(k=12, nx=9, ny=9, nz=4, ix_lim=9, iy_lim=9,
          rtpp=(0, 0.95),
          types=[T(0, 8, 40, 75.0, -1.0, 20, err_muti=0.5, upper=False),
                 T(1, 4, 200, 24.0, 3.0, 300, err_muti=1.0, err_rej=8.0)])),
        # Q1 defined case: last GTS type appended is 2-D (gpspw) -> 3-D types searched in 2-D
        ("driver_q1.npz", 405, dict(k=10, nx=7, ny=8, nz=4, ix_lim=7, iy_lim=8,
          types=[T(0, 2, 30, 50.0, 3.0, 100, **gts5),
                 T(0, 8, 20, 75.0, -1.0, 20, err_muti=0.5, upper=False)])),
        # offset state (xb ~ 285): fp32 rounding of the analysis at T-like magnitudes
        ("driver_offset.npz", 406, dict(k=40, nx=9, ny=8, nz=5, ix_lim=9, iy_lim=8,
          xb_mu=285.0, types=[T(1, 2, 700, 12.0, 3.0, 1000, err_muti=1.0, err_rej=8.0)])),
        # radar zdr (type 3, 'MD', module_radar.f90:70-79) beside dbz with its norain rules
        # and a sounding, k = 20, RTPS only
        ("driver_zdr.npz", 407, dict(k=20, nx=10, ny=9, nz=5, ix_lim=10, iy_lim=9,
          rtpp=(0, 0.95), multi_infl=1.3,
          types=[T(0, 1, 25, 75.0, 3.0, 40, err_muti=[0.5, 0.5, 0.7, 0.5, 0.5]),
                 T(1, 1, 300, 10.0, 2.0, 60, err_muti=2.5, err_rej=20.0),
                 T(1, 3, 400, 12.0, 3.0, 200, err_muti=1.0, err_rej=6.0)])),
    ]


def main_driver(name):
    """Regenerate one G4 case (and its manifest entry) without touching the others."""
    case = [c for c in driver_cases() if c[0] == name]
    if not case:
        sys.exit(f"no driver case {name}")
    fn, seed, kw = case[0]
    d = gen_driver(fn, seed, **kw)
    np.savez_compressed(os.path.join(OUT, fn), **d)
    mf = os.path.join(OUT, "MANIFEST.json")
    with open(mf) as f:
        manifest = json.load(f)
    manifest["files"][fn] = {"what": "G4 one variable through the driver loop", "seed": seed,
                             "k": kw["k"], "grid": [kw["nx"], kw["ny"], kw["nz"]],
                             "points_changed": int(np.any(d["var_out"] != d["var_in"], axis=0).sum())}
    with open(mf, "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(fn, manifest["files"][fn])


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build oracle/_ref/ref_harness first (make -C oracle ref)")
    os.makedirs(OUT, exist_ok=True)
    manifest = {"provenance": "reference modules param/config/eigen/kdtree2 (Q7: one array "
                "section of kdtree2_create made explicit) and localization (build_tree, get_lz, "
                "Gaspari_Cohn_1999) on type-only gts_omboma/simulated_radar modules cut from "
                "the reference, + source text of letkf_yoyb, letkf_solve and letkf_tune_q, "
                "compiled by oracle/ref/build_ref.sh with amdflang 22 -O2 (x86-64, no FMA), MKL "
                "libmkl_rt (sequential, MKL_CBWR=COMPATIBLE), glibc 2.35 expf (FMA IFUNC "
                "variant); only letkf_driver's point loop (module_letkf_core.f90:209-240) is "
                "written out, in oracle/ref/ref_driver.inc", "files": {}}

    raw = run("consts", b"")
    c = np.frombuffer(raw, f4)
    np.savez_compressed(os.path.join(OUT, "consts.npz"), gc1999=c[0], r2=c[1],
                        nmember_inv_k8=c[2], nmember_1_inv_k8=c[3])
    manifest["files"]["consts.npz"] = {"what": "G0 constants"}

    for k, seed in ((8, 101), (40, 140), (64, 164), (128, 228)):
        d = gen_solve(k, seed)
        fn = f"solve_k{k}.npz"
        np.savez_compressed(os.path.join(OUT, fn), **d)
        manifest["files"][fn] = {"what": "G1 letkf_solve KAT", "seed": seed, "k": k,
                                 "points": int(len(d["p"])), "p": sorted(set(map(int, d["p"])))}

    searches = [
        ("search_3d.npz", 201, 3000, 300, 12.0, 3.0, 1000, 0.0),
        ("search_3d_overflow.npz", 202, 3000, 300, 12.0, 3.0, 40, 0.0),
        ("search_2d.npz", 203, 600, 300, 50.0, -1.0, 200, 0.0),
        ("search_2d_overflow_dups.npz", 204, 600, 300, 50.0, -1.0, 17, 0.2),
        ("search_3d_small.npz", 205, 5, 50, 36.0, 3.0, 10, 0.0),
        ("search_3d_bucket.npz", 206, 13, 50, 36.0, 3.0, 20, 0.0),
    ]
    for (fn, seed, nobs, nq, h, v, mlz, dup) in searches:
        d = gen_search(fn, seed, nobs, nq, h, v, mlz, dup)
        np.savez_compressed(os.path.join(OUT, fn), **d)
        manifest["files"][fn] = {"what": "G2 kdtree2 fixed-ball search KAT", "seed": seed,
                                 "nobs": nobs, "nq": nq, "hclr": h, "vclr": v, "max_lz": mlz,
                                 "nfound_max": int(d["nfound"].max())}

    rng = np.random.default_rng(300)
    xs = np.concatenate([np.linspace(0, 4, 4001), rng.uniform(0, 4, 4000),
                         [1.8257418, 1.8257419, 3.6514835, 3.6514838, 3.651484]]).astype(f4)
    gy = np.frombuffer(run("gc", b(np.array([len(xs)], i4), xs)), f4)
    np.savez_compressed(os.path.join(OUT, "gc.npz"), x=xs, y=gy)
    manifest["files"]["gc.npz"] = {"what": "G3 Gaspari_Cohn_1999"}

    drivers = driver_cases()
    for (fn, seed, kw) in drivers:
        d = gen_driver(fn, seed, **kw)
        np.savez_compressed(os.path.join(OUT, fn), **d)
        changed = int(np.any(d["var_out"] != d["var_in"], axis=0).sum())
        manifest["files"][fn] = {"what": "G4 one variable through the driver loop",
                                 "seed": seed, "k": kw["k"],
                                 "grid": [kw["nx"], kw["ny"], kw["nz"]],
                                 "points_changed": changed}
    with open(os.path.join(OUT, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(json.dumps(manifest["files"], indent=1))


if __name__ == "__main__":
    if sys.argv[1:] == ["tuneq"]:
        main_tuneq()
    elif sys.argv[1:] == ["dims"]:
        main_dims()
    elif sys.argv[1:2] == ["driver"]:
        main_driver(sys.argv[2])
    else:
        main()
        main_tuneq()
        main_dims()
