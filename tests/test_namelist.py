"""The host-side namelist reader (cwbl/namelist.py) against the reference's own read_namelist
(module_config.f90, compiled with amdflang from /root/reference) and the Fortran glue that
fills the ABI blocks (fortran/letkf_core_gpu_config.f90): the ABI bytes must be equal.

tests/golden/namelist/input.nml is the reference's input.nml (a data file).  amdflang's
namelist reader rejects its `radar_nml % dbz % use_it` lines (Q6), so the
Fortran side reads a copy with the blanks around `%` removed; the Python reader reads the
original."""
import ctypes as C
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from cwbl import abi, namelist
from helpers import GOLDEN, REPO

FC = shutil.which("amdflang") or shutil.which("flang")
NML = os.path.join(GOLDEN, "namelist", "input.nml")
FORT = os.path.join(REPO, "cwbnwp-letkf_amd", "fortran")
needs_ref = pytest.mark.skipif(FC is None or not os.path.isdir("/root/reference"),
                               reason="needs amdflang and the reference sources")

DUMP = r"""
program nml_dump
    use iso_c_binding
    use letkf_core_gpu
    use letkf_core_gpu_config
    use config
    implicit none
    character(len=512) :: fin, fout
    type(cwbl_var_params)  :: vp
    type(cwbl_init_params) :: ip
    integer :: ivar, u
    call get_command_argument(1, fin)
    call get_command_argument(2, fout)
    call read_namelist(trim(fin))
    open(newunit=u, file=trim(fout), access='stream', form='unformatted', status='replace')
    call init_params_from_namelist(3, ip)
    write(u) ip
    do ivar = 1, 16
        call var_params_from_namelist(ivar, vp)
        write(u) vp
    end do
    write(u) cen_lon, cen_lat, truelat1, truelat2, sta_lon, norain_value
    write(u) nmember, weight_function, wrf_mp_physics, wrf_mp_hail_opt
    write(u) var_update
    close(u)
end program nml_dump
"""


@pytest.fixture(scope="module")
def dumper(tmp_path_factory):
    if FC is None or not os.path.isdir("/root/reference"):
        pytest.skip("needs amdflang and the reference sources")
    td = str(tmp_path_factory.mktemp("nml"))
    cpp = ["cpp", "-C", "-P", "-traditional", "-Wno-invalid-pp-token", "-ffreestanding",
           "-DREAL64"]
    objs = []
    for m in ("module_param", "module_config"):
        with open(os.path.join(td, m + ".F90"), "w") as f:
            subprocess.run(cpp + [f"/root/reference/{m}.f90"], stdout=f, check=True)
        subprocess.run([FC, "-c", m + ".F90"], cwd=td, check=True)
        objs.append(m + ".o")
    for f in ("letkf_core_gpu.f90", "letkf_core_gpu_config.f90"):
        subprocess.run([FC, "-c", os.path.join(FORT, f)], cwd=td, check=True)
        objs.append(f.replace(".f90", ".o"))
    with open(os.path.join(td, "nml_dump.f90"), "w") as f:
        f.write(DUMP)
    lib = os.path.join(REPO, "cwbnwp-letkf_amd", "lib")  # (cwbl_error binds cwbl_last_error)
    subprocess.run([FC, "nml_dump.f90"] + objs + ["-o", "nml_dump", "-L" + lib, "-lcwbl",
                    "-Wl,-rpath," + lib], cwd=td, check=True)
    return os.path.join(td, "nml_dump")


def fortran_dump(dumper, text, tmp_path):
    fin, fout = tmp_path / "in.nml", tmp_path / "out.bin"
    fin.write_text(text)
    r = subprocess.run([dumper, str(fin), str(fout)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    return fout.read_bytes()


def python_dump(cfg):
    out = bytes(namelist.init_params(cfg, 3))
    for ivar in range(1, 17):
        out += bytes(namelist.var_params(cfg, ivar))
    p, c = cfg["projection"], cfg["control"]
    out += np.array([p["cen_lon"], p["cen_lat"], p["truelat1"], p["truelat2"], p["sta_lon"],
                     c["norain_value"]], np.float32).tobytes()
    out += np.array([c["nmember"], c["weight_function"], c["wrf_mp_physics"],
                     c["wrf_mp_hail_opt"]], np.int32).tobytes()
    out += "".join(v.ljust(10) for v in c["var_update"]).encode()
    return out


@needs_ref
def test_reference_input_nml_gives_the_fortran_glue_bytes(dumper, tmp_path):
    text = open(NML).read()
    assert re.search(r"\w\s+%\s+\w", text)                   # the file has Q6 lines
    fixed = re.sub(r"\s*%\s*", "%", text)                     # what amdflang accepts
    want = fortran_dump(dumper, fixed, tmp_path)
    cfg = namelist.read_namelist(NML)                         # the original, Q6 included
    assert python_dump(cfg) == want
    assert namelist.var_names(cfg)[:4] == ["U", "V", "W", "T"] and cfg["control"]["nmember"] == 96


EDGE = """! edge cases of the namelist syntax
&control
 nmember = 40, weight_function = 1
 var_update = 'U', "V", 2*'QRAIN', , 'P'
 norain_value = -7.5e0
/
&other
 ignored = 1
/
&projection
 sta_lon = 121.25, cen_lat = 22.5d0
/
&observations
 radar_nml%vr%use_it = .true.
 radar_nml%vr%hclr = 16*12.5
 radar_nml%vr%hclr(3:5) = 3*30.
 radar_nml%vr%vclr(2) = 4.
 radar_nml%kdp%use_it = .T., radar_nml%kdp%error = 0.3
 synop_nml%use_it = T
 synop_nml%hclr = 1., , 3., 2*
 synop_nml%u%is_assim = 4*T, F, .false., t
 synop_nml%q%err_muti = 0.7
 gpspw_nml%tpw%is_assim(16) = T
/
&inflation
 multi_infl = 16*1.3, use_RTPP = 8*T
 RTPP_Alpha(2:3) = 0.5 0.6
 use_rtps = T
/
"""


@needs_ref
def test_namelist_syntax_edge_cases_equal_the_reference_reader(dumper, tmp_path):
    want = fortran_dump(dumper, EDGE, tmp_path)
    assert python_dump(namelist.read_namelist(EDGE, is_text=True)) == want


def test_errors_carry_the_reference_messages(tmp_path):
    with pytest.raises(namelist.NamelistError, match="input.nml doesn't exist"):
        namelist.read_namelist(str(tmp_path / "missing.nml"))
    with pytest.raises(namelist.NamelistError, match="Please input ensemble size"):
        namelist.read_namelist("&control\n/\n&projection\n/\n&observations\n/\n&inflation\n/\n",
                               is_text=True)
    with pytest.raises(namelist.NamelistError, match="projection_nml fail"):
        namelist.read_namelist("&control\n nmember=4\n/\n&inflation\n/\n", is_text=True)
    with pytest.raises(namelist.NamelistError, match="control_nml fail"):
        namelist.read_namelist("&control\n nmembers=4\n/\n", is_text=True)
    with pytest.raises(namelist.NamelistError, match="inflation_nml fail"):
        namelist.read_namelist("&control\n nmember=4\n/\n&projection\n/\n&observations\n/\n"
                               "&inflation\n multi_infl = 17*1.0\n/\n", is_text=True)


def test_var_params_feed_the_core_types():
    cfg = namelist.read_namelist(NML)
    vp = namelist.var_params(cfg, 1)                       # U: multi_infl 1.6, RTPP/RTPS .95
    assert abs(vp.multi_infl - 1.6) < 1e-6 and vp.use_rtpp == 1 and vp.tune_q == 0
    vr = vp.radar[abi.RADAR_VR - 1]
    assert vr.use_it == 1 and vr.max_lz_pts == 300 and vr.hclr == 36.0 and vr.vclr == 3.0
    assert vr.err_muti[0] == 1.0 and vr.err_rej[0] == 8.0  # radar error rides in err_muti(1)
    q = namelist.var_params(cfg, 6)                        # QRAIN: tune_q
    assert q.tune_q == 1 and q.radar[abi.RADAR_DBZ - 1].hclr == 8.0
    p = namelist.projection(cfg)
    assert (p.sta_lon, p.truelat1, p.truelat2) == (120.0, 10.0, 40.0)


def test_var_names_stop_at_the_first_blank_entry():
    """letkf_driver exits its variable loop at the first blank var_update entry
    (module_letkf_core.f90:59-60): the EDGE namelist has a null value after 2*'QRAIN', so
    'P' is never analysed and ivar positions are not shifted."""
    cfg = namelist.read_namelist(EDGE, is_text=True)
    assert namelist.var_names(cfg) == ["U", "V", "QRAIN", "QRAIN"]
