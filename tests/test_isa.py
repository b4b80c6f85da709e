"""ISA checks of hand-written inline asm (CPU: compiles the kernel source to gfx950 assembly).

solve_tq40_kernel fuses row broadcasts into `v_fmac_f64_dpp ... row_newbcast` through inline
asm (cwbl_tq40.hip fmac_row / fnmac_row).  gfx9 requires two wait states between a VALU
write of a VGPR and a DPP instruction reading it as its (DPP) source; the compiler's hazard
recognizer does not see inside the asm, so the kernel pins its sources behind an `s_nop 1`.
This scans the production instantiation's ISA for any such hazard and for spills."""
import os
import re
import shutil
import subprocess

import pytest

from helpers import REPO

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
SRC = os.path.join(REPO, "cwbnwp-letkf_amd", "csrc")
needs_hipcc = pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")


def regs(tok):
    m = re.match(r"-?v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"-?v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def dpp_hazards(lines):
    """(writer, reader) pairs where a VALU instruction writes the DPP source of a DPP
    instruction fewer than 2 wait states before it (s_nop N counts N + 1)."""
    out = []
    for i, l in enumerate(lines):
        if "row_newbcast" not in l and "quad_perm" not in l and "row_" not in l:
            continue
        ops = l.split(None, 1)[1].split(",") if " " in l else []
        if len(ops) < 2:
            continue
        src = regs(ops[1].strip().split()[0])
        ws, j = 0, i - 1
        while j >= 0 and ws < 2:
            t = lines[j]
            op = t.split()[0]
            if op.startswith("s_nop"):
                ws += int(t.split()[1]) + 1
            else:
                if op.startswith("v_") and " " in t and regs(t.split(None, 1)[1].split(",")[0].strip()) & src:
                    out.append((t, l))
                    break
                ws += 1
            j -= 1
    return out


@needs_hipcc
def test_tq40_dpp_fma_has_no_hazard_and_no_spill(tmp_path):
    text = open(os.path.join(SRC, "cwbl_tq40.hip")).read()
    # the production instantiation only (the timing-ablation ones take 3 more minutes)
    text = "\n".join(l for l in text.splitlines() if not re.match(r"\s*case [234]: hipLaunchKernelGGL", l))
    src = tmp_path / "tq40.hip"
    src.write_text(text)
    asm = tmp_path / "tq40.s"
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-munsafe-fp-atomics", "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-I", SRC,
                        "--offload-device-only", "-S", str(src), "-o", str(asm)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l.strip() for l in asm.read_text().splitlines()
             if l.startswith("\t") and not l.strip().startswith((".", ";"))]
    fused = [l for l in lines if l.startswith("v_fmac_f64_dpp")]
    assert len(fused) > 3000, len(fused)           # the broadcasts are fused
    assert dpp_hazards(lines) == []
    assert not [l for l in lines if l.startswith("scratch_")]  # no spills, nothing parked


def test_hazard_scan_finds_a_hazard():
    bad = ["v_mul_f64 v[2:3], v[4:5], v[6:7]",
           "v_fmac_f64_dpp v[0:1], v[2:3], v[8:9] row_newbcast:1 row_mask:0xf bank_mask:0xf"]
    assert len(dpp_hazards(bad)) == 1
    ok = [bad[0], "s_nop 1", bad[1]]
    assert dpp_hazards(ok) == []
    ok2 = [bad[0], "v_add_f64 v[10:11], v[12:13], v[14:15]", "s_nop 0", bad[1]]
    assert dpp_hazards(ok2) == []
