"""CPU tests of the host obs ingest and projection (include/cwb_letkf_ingest.h,
csrc/obs_ingest.cpp) against the reference's own readers.

tests/golden/ingest/ holds synthetic files in the reference's formats (obs_gts, three members'
gts_letkf_### / VR_ / MR_letkf_###) and tests/golden/ingest.npz what the reference's compiled
read_gts_omboma / read_alt_info / get_alt / read_radar and module_projection made of them
(oracle/gen_ingest.py -> oracle/_ref/ref_harness ingest).  Everything must agree bit for bit.
"""
import os
import shutil

import numpy as np
import pytest

from cwbl import abi
from cwbl import dist as cdist
from cwbl import ingest
from helpers import GOLDEN, golden

DIR = os.path.join(GOLDEN, "ingest")


def read_all(d=DIR, k=3, order=None):
    h = ingest.Ingest(k)
    for m in (order or range(k)):
        h.read_gts(os.path.join(d, f"gts_letkf_{m + 1:03d}"), os.path.join(d, "obs_gts"))
        h.read_radar(os.path.join(d, f"VR_letkf_{m + 1:03d}"), "VR")
        h.read_radar(os.path.join(d, f"MR_letkf_{m + 1:03d}"), "MR")
    return h


def bits(a):
    a = np.asarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


def test_projection_matches_the_reference():
    g = golden("ingest.npz")
    x, y = ingest.lonlat_to_xy(g["lonlat"][:, 0], g["lonlat"][:, 1])
    np.testing.assert_array_equal(bits(np.stack([x, y], 1)), bits(g["xy"]))
    # the map origin (sta_lon, cen_lat) is x = 0
    assert x[0] == 0.0


@pytest.mark.parametrize("order", [None, [2, 0, 1]])
def test_readers_match_the_reference_bit_for_bit(order):
    g = golden("ingest.npz")
    h = read_all(order=order)
    types = h.types()
    got_g = [t["type_id"] for t in types if t["family"] == 0]
    got_r = [t["type_id"] for t in types if t["family"] == 1]
    assert got_g == list(g["gts_types"]) and got_r == list(g["radar_types"])
    for t in types:
        p = f"{'g' if t['family'] == 0 else 'r'}{t['type_id']}_"
        keys = ("xyz", "obs", "error", "hdxb", "qc") if t["family"] == 0 else ("xyz", "obs", "hdxb")
        for key in keys:
            np.testing.assert_array_equal(bits(t[key]), bits(g[p + key]), err_msg=p + key)
        m = h.meta(t["family"], t["type_id"])
        for key in ("lat", "lon", "alt"):
            np.testing.assert_array_equal(bits(m[key]), bits(g[p + key]), err_msg=p + key)
        if t["family"] == 0:
            assert [s.encode() for s in m["ids"]] == list(g[p + "ids"])


def test_station_altitudes_follow_get_alt():
    """get_alt (module_gts_omboma.f90:1032-1049): the first station of an id wins, the 5
    characters of the omboma id must equal the obs_gts id up to trailing blanks, vertical
    reports take level k's height, gpspw / gpsref keep the file's own altitude."""
    h = read_all()
    syn = h.meta(0, abi.GTS_SYNOP)
    assert syn["ids"] == ["46692", "467A1", "C0A9 "]
    np.testing.assert_array_equal(syn["alt"], np.float32([9.0, 31.5, 14.25]))  # not 999
    snd = h.meta(0, abi.GTS_SOUND)
    np.testing.assert_array_equal(snd["alt"], np.float32([9.0, 1523.7, 5870.25, 25.0, 3102.125]))
    assert h.meta(0, abi.GTS_GPSPW)["alt"][0] == np.float32(212.75)


def test_fortran_field_conversions():
    """F17.7 without a decimal point takes 7 implied decimals, an exponent is read, a blank
    field is zero (the hdxb is then obs - 0), 123456.1234567 rounds to the nearest fp32."""
    h = read_all()
    t = {(d["family"], d["type_id"]): d for d in h.types()}
    syn = t[(0, abi.GTS_SYNOP)]
    g = golden("ingest.npz")
    np.testing.assert_array_equal(bits(syn["obs"]), bits(g["g2_obs"]))
    # synop report 2 var 1 has no decimal point: 7 implied decimals
    raw = open(os.path.join(DIR, "gts_letkf_001")).read().splitlines()
    field = [ln for ln in raw if ln.startswith("       2       1467A1")][0][56:73]
    assert "." not in field and syn["obs"][1, 0] == np.float32(int(field) * 1e-7)
    # metar report 1 var 3 has a blank omb in every member: hdxb = obs - 0
    met = t[(0, abi.GTS_METAR)]
    assert all(met["hdxb"][m, 0, 2] == met["obs"][0, 2] for m in range(3))
    assert met["obs"][1, 0] == np.float32(123456.1234567)


def test_wire_buffer_equals_the_python_packer_and_round_trips():
    h = read_all()
    types = h.types()
    wire = h.wire()
    ref = cdist.pack_obs_set(types, 3)
    np.testing.assert_array_equal(wire.view(np.uint32), ref.view(np.uint32))
    k, back = cdist.unpack_obs_set(wire)
    assert k == 3 and len(back) == len(types)
    for a, b in zip(types, back):
        for key in ("xyz", "obs", "hdxb") + (("error", "qc") if a["family"] == 0 else ()):
            np.testing.assert_array_equal(np.asarray(b[key]), a[key])


def test_obs_set_crosses_the_abi_as_host_memory():
    h = read_all()
    s = h.obs_set()
    assert s.memory == abi.MEM_HOST and s.n_gts == 8 and s.n_radar == 2
    assert [s.gts[e].type_id for e in range(s.n_gts)] == [1, 2, 3, 8, 9, 10, 11, 18]
    assert [s.gts[e].nvar for e in range(s.n_gts)] == [4, 5, 2, 1, 1, 5, 5, 5]


def test_metadata_comes_from_member_0(tmp_path):
    """gts_distribute / radar_distribute broadcast the root reader's arrays (member 1 of
    cwb_letkf.f90:46-57): a different position in another member's file is not used."""
    d = tmp_path / "in"
    shutil.copytree(DIR, d)
    p = d / "VR_letkf_002"
    rows = p.read_text().splitlines()
    f = rows[1].split()
    f[2] = f"{float(f[2]) + 1.0:.4f}"
    rows[1] = "".join(f"{float(v):10.4f} " for v in f)
    p.write_text("\n".join(rows) + "\n")
    a, b = read_all(), read_all(str(d))
    np.testing.assert_array_equal(a.meta(1, abi.RADAR_VR)["lon"], b.meta(1, abi.RADAR_VR)["lon"])


def test_metadata_before_member_0_is_an_error():
    """A host that has read only member 1's files has hdxb/qc but no metadata (the root
    reader's arrays): meta() must fail, not hand out pointers into empty buffers."""
    h = ingest.Ingest(3)
    h.read_radar(os.path.join(DIR, "VR_letkf_002"), "VR")
    h.read_gts(os.path.join(DIR, "gts_letkf_002"), os.path.join(DIR, "obs_gts"))
    with pytest.raises(abi.CwblError, match="no metadata"):
        h.meta(1, abi.RADAR_VR)
    with pytest.raises(abi.CwblError, match="no metadata"):
        h.meta(0, abi.GTS_SYNOP)
    h.read_radar(os.path.join(DIR, "VR_letkf_001"), "VR")
    assert h.meta(1, abi.RADAR_VR)["lon"].size > 0


def test_errors_are_reported_not_ignored(tmp_path):
    d = tmp_path / "in"
    shutil.copytree(DIR, d)
    # a station the obs_gts file does not know ("ID not found!!", :1048)
    p = d / "gts_letkf_001"
    p.write_text(p.read_text().replace("46692", "99999", 1))
    h = ingest.Ingest(3)
    with pytest.raises(abi.CwblError, match="not in"):
        h.read_gts(str(p), str(d / "obs_gts"))
    # a radar file shorter than its count (Q5, module_radar.f90:91-104)
    p = d / "VR_letkf_001"
    p.write_text("\n".join(p.read_text().splitlines()[:-2]) + "\n")
    with pytest.raises(abi.CwblError, match="ends after"):
        h.read_radar(str(p), "VR")
    # a report type the reference has no branch for, with data
    p = d / "gts_letkf_002"
    p.write_text("ssmi_rv                    1\n       1       1\n" + p.read_text())
    with pytest.raises(abi.CwblError, match="not read by the reference"):
        h.read_gts(str(p), str(d / "obs_gts"))
    # a member whose file is missing from the set
    h2 = ingest.Ingest(3)
    h2.read_radar(os.path.join(DIR, "VR_letkf_001"), "VR")
    with pytest.raises(abi.CwblError, match="lacks member 1"):
        h2.obs_set()
    with pytest.raises(abi.CwblError):
        h2.read_radar(os.path.join(DIR, "VR_letkf_001"), "XX")


def test_ingest_header_declares_the_exports():
    import re
    src = open(os.path.join(os.path.dirname(GOLDEN), "..", "include", "cwb_letkf_ingest.h")).read()
    declared = set(re.findall(r"\b(cwbl_[a-z_]+)\s*\(", src)) - {"cwbl_last_error"}  # (core)
    assert sorted(declared) == sorted(ingest.EXPORTS)
