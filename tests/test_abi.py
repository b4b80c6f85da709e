"""CPU checks of the C-ABI boundary: the built library loads and exports every symbol the
header declares, the ctypes structs match the C compiler's layout, and compute entry points
fail loudly (no CPU fallback) when there is no GPU."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

from cwbl import abi
from helpers import REPO

HEADER = os.path.join(REPO, "include", "cwb_letkf_core.h")
LIB = abi.default_library_path()


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(cwbl_[a-z_]+)\s*\(", src)))


def test_header_declares_the_python_export_list():
    assert header_functions() == sorted(abi.EXPORTS)


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(REPO, "cwbnwp-letkf_amd"), "-j4", "all"],
                       check=True, capture_output=True)
    return abi.load_library(LIB)


def test_library_exports_every_header_symbol(lib):
    """Every entry point declared in include/*.h (the core and the ingest header)."""
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (cwbl_\w+)", out))
    declared = set()
    inc = os.path.join(REPO, "include")
    for h in sorted(os.listdir(inc)):
        if h.endswith(".h"):
            declared |= set(re.findall(r"\b(cwbl_[a-z_]+)\s*\(", open(os.path.join(inc, h)).read()))
    assert {"cwbl_analyze_var", "cwbl_ingest_read_gts", "cwbl_lonlat_to_xy"} <= declared
    missing = declared - exported
    assert not missing, missing
    assert lib.cwbl_abi_version() == abi.ABI_VERSION


def test_library_has_gfx950_code_object():
    data = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


STRUCTS = {
    "cwbl_init_params": abi.InitParams, "cwbl_gts_obs": abi.GtsObs,
    "cwbl_radar_obs": abi.RadarObs, "cwbl_obs_set": abi.ObsSet,
    "cwbl_type_params": abi.TypeParams, "cwbl_var_params": abi.VarParams,
    "cwbl_slab": abi.Slab, "cwbl_stats": abi.Stats, "cwbl_kernel_time": abi.KernelTime,
}


def test_struct_layouts_match_c():
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(){"]
    for cname, py in STRUCTS.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as td:
        src, exe = os.path.join(td, "l.c"), os.path.join(td, "l")
        open(src, "w").write("\n".join(lines))
        subprocess.run(["gcc", src, "-o", exe], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    got = dict(line.split() for line in out if line)
    for cname, py in STRUCTS.items():
        assert int(got[cname]) == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got[f"{cname}.{fname}"]) == getattr(py, fname).offset, (cname, fname)


def test_compute_without_state_fails_loudly(lib):
    # no cwbl_init: every compute entry point reports a state error, nothing runs on the CPU
    assert lib.cwbl_set_obs(C.byref(abi.ObsSet())) == 2
    assert lib.cwbl_analyze_var(C.byref(abi.VarParams()), C.byref(abi.Slab()), None) == 2
    assert b"cwbl_init" in lib.cwbl_last_error()


def test_init_without_gpu_reports_no_device(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    rc = lib.cwbl_init(C.byref(abi.InitParams(8, 0, 0, -5.0, 0, 0, 0)))
    assert rc == 3, lib.cwbl_last_error()
