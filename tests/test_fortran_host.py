"""The Fortran side of the boundary: the iso_c_binding module compiles, the glue that reads
the reference's namelist state compiles against the reference's own config/param modules,
and (GPU) a Fortran host program analyses a golden case through the C ABI."""
import os
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

from helpers import REPO, DriverCase, increment_rel_rms

PKG = os.path.join(REPO, "cwbnwp-letkf_amd")
FC = shutil.which("amdflang") or shutil.which("flang")
DRIVER = os.path.join(PKG, "lib", "abi_case_driver")
needs_fc = pytest.mark.skipif(FC is None, reason="no Fortran compiler")


@needs_fc
def test_fortran_binding_and_driver_build():
    subprocess.run(["make", "-C", PKG, "fortran"], check=True, capture_output=True)
    assert os.path.exists(DRIVER)


@needs_fc
@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="reference not present")
def test_namelist_glue_compiles_against_reference_config():
    cpp = ["cpp", "-C", "-P", "-traditional", "-Wno-invalid-pp-token", "-ffreestanding",
           "-DREAL64"]
    with tempfile.TemporaryDirectory() as td:
        for m in ("module_param", "module_config"):
            with open(os.path.join(td, m + ".F90"), "w") as f:
                subprocess.run(cpp + [f"/root/reference/{m}.f90"], stdout=f, check=True)
            subprocess.run([FC, "-c", m + ".F90"], cwd=td, check=True)
        subprocess.run([FC, "-c", os.path.join(PKG, "fortran", "letkf_core_gpu.f90")], cwd=td,
                       check=True)
        subprocess.run([FC, "-c", os.path.join(PKG, "fortran", "letkf_core_gpu_config.f90")],
                       cwd=td, check=True)


def write_case(case, path):
    i4 = lambda *v: np.array(v, np.int32).tobytes()  # noqa: E731
    with open(path, "wb") as f:
        f.write(i4(case.k, case.var_in.shape[3], case.var_in.shape[2], case.var_in.shape[1],
                   case.ix_lim, case.iy_lim, case.wf, len(case.types)))
        f.write(np.float32(case.norain).tobytes())
        f.write(bytes(case.vp))
        for a in (case.x, case.y, case.alt, case.var_in):
            f.write(np.ascontiguousarray(a, np.float32).tobytes())
        for t in case.types:
            f.write(i4(t["family"], t["type_id"], t["nvar"], t["nobs"]))
            f.write(np.ascontiguousarray(t["xyz"], np.float32).tobytes())
            if t["family"] == 0:
                for key in ("obs", "error", "hdxb"):
                    f.write(np.ascontiguousarray(t[key], np.float32).tobytes())
                f.write(np.ascontiguousarray(t["qc"], np.int32).tobytes())
            else:
                f.write(np.ascontiguousarray(t["obs"][:, 0], np.float32).tobytes())
                f.write(np.ascontiguousarray(t["hdxb"][:, :, 0], np.float32).tobytes())


@pytest.mark.gpu
@needs_fc
@pytest.mark.parametrize("name", ["driver_mixed.npz", "driver_gc_k40.npz"])
def test_fortran_host_analysis_matches_reference(name):
    if not os.path.exists(DRIVER):
        subprocess.run(["make", "-C", PKG, "fortran"], check=True, capture_output=True)
    case = DriverCase(name)
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "case.bin"), os.path.join(td, "out.bin")
        write_case(case, fin)
        r = subprocess.run([DRIVER, fin, fout], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "fortran host: solved=" in r.stdout
        var = np.fromfile(fout, np.float32).reshape(case.var_in.shape)
    assert increment_rel_rms(var, case.var_out, case.var_in) <= 1e-6


@needs_fc
def test_fortran_host_ingest_equals_the_python_binding(tmp_path):
    """A Fortran host reads the member obs files through the ingest interfaces of
    letkf_core_gpu.f90 (fortran/ingest_driver.f90) and packs the wire buffer that replaces
    gts_distribute / radar_distribute: the same bits as the ctypes binding's."""
    from cwbl import ingest
    drv = os.path.join(PKG, "lib", "ingest_driver")
    subprocess.run(["make", "-C", PKG, "fortran"], check=True, capture_output=True)
    d = os.path.join(REPO, "tests", "golden", "ingest")
    out = str(tmp_path / "wire.bin")
    r = subprocess.run([drv, d, "3", out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gts types=8 radar types=2" in r.stdout
    h = ingest.Ingest(3)
    for m in range(3):
        h.read_gts(os.path.join(d, f"gts_letkf_{m + 1:03d}"), os.path.join(d, "obs_gts"))
        h.read_radar(os.path.join(d, f"VR_letkf_{m + 1:03d}"), "VR")
        h.read_radar(os.path.join(d, f"MR_letkf_{m + 1:03d}"), "MR")
    np.testing.assert_array_equal(np.fromfile(out, np.uint32), h.wire().view(np.uint32))
