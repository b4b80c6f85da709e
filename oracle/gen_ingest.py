#!/usr/bin/env python3
"""Generate the obs-ingest fixtures: synthetic input files in the reference's formats
(tests/golden/ingest/) and the reference's own reading of them (tests/golden/ingest.npz).

TEST INFRASTRUCTURE ONLY.  Run in the build container after oracle/ref/build_ref.sh:
    python oracle/gen_ingest.py
The reference ships no sample files, so the inputs are synthetic:
  obs_gts           WRFDA obsproc ASCII as read_alt_info reads it (module_gts_omboma.f90:
                    704-1030): count records, the INFO/SRFC/EACH formats, reports of FM-12
                    synop (incl. a repeated station id and an id longer than 5 characters),
                    FM-15 metar, FM-13 ships, FM-18 buoy, FM-35 sound, FM-32 pilot, FM-111
                    gpspw and FM-116 gpsref
  gts_letkf_00m     WRFDA gts_omboma records per member (read_gts_omboma, :48-506): synop,
                    metar, ships, buoy, sound, pilot, gpspw, gpsref and empty sections;
                    fields with many digits, no decimal point (F17.7's implied decimals), an
                    exponent, blanks and negative QC
  VR_/MR_letkf_00m  radar rows (read_radar, module_radar.f90:30-118)
and ref_harness `ingest` runs the reference's compiled read_gts_omboma / read_alt_info /
get_alt / read_radar and module_projection on them (oracle/ref/build_ref.sh), as the ranks
of cwb_letkf.f90:46-57 would: member m reads its own files, the root (member 1) provides
the metadata.  Output: tests/golden/ingest.npz.
"""
import os
import shutil
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
HARNESS = os.path.join(HERE, "_ref", "ref_harness")
OUTDIR = os.path.join(REPO, "tests", "golden", "ingest")
K = 3

INFO_FMT = "(A12,1X,A19,1X,A40,1X,I6,3(F12.3,11X),6X,A40)"
SRFC_FMT = "(F12.3,I4,F7.2,F12.3,I4,F7.3)"
EACH_FMT = "(3(F12.3,I4,F7.2),11X,3(F12.3,I4,F7.2),11X,1(F12.3,I4,F7.2))"

# obs_gts stations: (FM code, name, id (A40), lat, lon, elevation, heights per level)
STATIONS = [
    (12, "SYNOP", "46692", 25.03, 121.51, 9.0, [9.0]),
    (12, "SYNOP", "46699", 24.15, 120.68, 84.0, [84.0]),
    (12, "SYNOP", "467A1", 23.50, 120.42, 31.5, [31.5]),
    (12, "SYNOP", "C0A9", 22.99, 120.20, 14.25, [14.25]),
    (12, "SYNOP", "46692", 25.03, 121.51, 999.0, [999.0]),     # repeated id: first one wins
    (12, "SYNOP", "4669912345", 24.0, 121.0, 5.0, [5.0]),     # longer than the omboma's A5
    (15, "METAR", "RCTP", 25.08, 121.23, 33.0, [33.0]),
    (15, "METAR", "RCSS", 25.07, 121.55, 6.0, [6.0]),
    (13, "SHIP", "SHIP1", 21.5, 119.2, 0.0, [2.5]),
    (18, "BUOY", "BUOY1", 22.1, 121.9, 0.0, [1.25]),
    (35, "TEMP", "46692", 25.03, 121.51, 9.0, [9.0, 1523.7, 5870.25]),
    (35, "TEMP", "46810", 22.00, 120.75, 25.0, [25.0, 3102.125]),
    (32, "PILOT", "46750", 23.9, 121.6, 12.0, [150.5, 2975.0]),
    (111, "GPSPW", "GPS01", 24.6, 120.8, 212.75, []),
    (116, "GPSRF", "GPSR1", 23.0, 122.5, 0.0, [8000.0]),
]


def fstr(v, w, d):
    return f"{v:{w}.{d}f}"


def write_obs_gts(path):
    cnt = {}
    for fm, *_ in STATIONS:
        cnt[fm] = cnt.get(fm, 0) + 1
    c = lambda *fms: sum(cnt.get(f, 0) for f in fms)  # noqa: E731
    pair = lambda name, v: f"{name:<6}={v:7d}, "  # noqa: E731  (A6,1X,I7,2X)
    lines = [f"TOTAL ={len(STATIONS):7d}, MISS. =-888888.,",
             pair("SYNOP", c(12)) + pair("METAR", c(15, 16)) + pair("SHIP", c(13, 17)) +
             pair("BUOY", c(18, 19)) + pair("BOGUS", 0) + pair("TEMP", c(35, 36, 37, 38)),
             pair("AMDAR", 0) + pair("AIREP", 0) + pair("TAMDAR", 0) + pair("PILOT", c(32, 33, 34)) +
             pair("SATEM", 0) + pair("SATOB", 0),
             pair("GPSPW", c(111, 114)) + pair("GPSZD", 0) + pair("GPSRF", c(116)) +
             pair("GPSEP", 0) + pair("SSMT1", 0) + pair("SSMT2", 0),
             pair("TOVS", 0) + pair("QSCAT", 0) + pair("PROFL", 0) + pair("AIRSR", 0) +
             pair("OTHER", 0),
             "PHIC  =  23.76, XLONC = 120.81, TRUE1 =  10.00, TRUE2 =  40.00, XIM11 =   1.00, XJM11 =   1.00,",
             "INFO  = PLATFORM, DATE, NAME, LEVELS, LATITUDE, LONGITUDE, ELEVATION, ID.",
             "SRFC  = SLP, PW (DATA,QC,ERROR).",
             "EACH  = PRES, SPEED, DIR, HEIGHT, TEMP, DEW PT, HUMID (DATA,QC,ERROR)*LEVELS.",
             f"INFO_FMT = {INFO_FMT}",
             f"SRFC_FMT = {SRFC_FMT}",
             f"EACH_FMT = {EACH_FMT}",
             "#" + "-" * 78 + "#"]
    for fm, name, sid, lat, lon, elev, hts in STATIONS:
        plat = f"FM-{fm} {name}"
        nlev = len(hts) if hts else 1
        info = (f"{plat:<12} {'2026-10-17_00:00:00':<19} {name + ' report':<40} {nlev:6d}" +
                "".join(fstr(v, 12, 3) + " " * 11 for v in (lat, lon, elev)) + " " * 6 +
                f"{sid:<40}")
        lines.append(info)
        lines.append(fstr(101325.0, 12, 3) + "   0" + fstr(100.0, 7, 2) +
                     fstr(-888888.0, 12, 3) + " -88" + fstr(0.2, 7, 3))
        trip = lambda v: fstr(v, 12, 3) + "   0" + fstr(1.0, 7, 2)  # noqa: E731
        for ht in hts:
            lines.append(trip(92500.0) + trip(5.0) + trip(270.0) + " " * 11 + trip(ht) +
                         trip(290.0) + trip(285.0) + " " * 11 + trip(80.0))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def f17(v):
    return fstr(v, 17, 7)


# gts_omboma reports: (section, nvar, [report = [(id, lat, lon, pre_or_alt), per level]])
def gts_sections():
    return [
        ("synop", 5, [[("46692", 25.03, 121.51, 101000.5)], [("467A1", 23.5, 120.42, 100950.0)],
                      [("C0A9 ", 22.99, 120.2, 101100.25)]]),
        ("metar", 5, [[("RCTP ", 25.08, 121.23, 100800.0)], [("RCSS ", 25.07, 121.55, 100900.0)]]),
        ("ships", 5, [[("SHIP1", 21.5, 119.2, 101200.0)]]),
        ("buoy", 5, [[("BUOY1", 22.1, 121.9, 101250.0)]]),
        ("satem", 1, []),
        ("sound", 4, [[("46692", 25.03, 121.51, 100000.0), ("46692", 25.04, 121.52, 85000.0),
                       ("46692", 25.05, 121.53, 50000.0)],
                      [("46810", 22.0, 120.75, 99000.0), ("46810", 22.01, 120.76, 70000.0)]]),
        ("pilot", 2, [[("46750", 23.9, 121.6, 99500.0), ("46750", 23.91, 121.61, 70000.0)]]),
        ("gpspw", 1, [[("GPS01", 24.6, 120.8, 212.75)]]),
        ("gpsref", 1, [[("GPSR1", 23.0, 122.5, 8000.0), ("GPSR1", 23.02, 122.51, 9000.0)]]),
        ("airep", 4, []),
    ]


def write_gts_member(path, m, rng_obs, rng_m):
    out = []
    ln = 0
    for name, nvar, reports in gts_sections():
        out.append(f"{name:<20}{len(reports):8d}")
        for rep in reports:
            out.append(f"{len(rep):8d}{1:8d}")
            for (sid, lat, lon, pre) in rep:
                ln += 1
                line = f"{ln:8d}{1:8d}{sid:<5}" + fstr(lat, 9, 2) + fstr(lon, 9, 2) + f17(pre)
                for v in range(nvar):
                    obs = float(rng_obs.normal(280.0 if v == 3 else 0.0, 5.0))
                    omb = float(rng_m.normal(0.0, 1.5))
                    qc = int(rng_m.choice([0, 0, 0, 1, 2, -88, -5]))
                    err = float(abs(rng_obs.normal(1.5, 0.4)))
                    obs_s = f17(obs)
                    omb_s = f17(omb)
                    if ln == 2 and v == 0:
                        obs_s = f"{int(round(obs * 1e7)):17d}"   # no point: 7 implied decimals
                    if ln == 3 and v == 1:
                        omb_s = f"{omb:17.6E}"                  # exponent form
                    if ln == 4 and v == 2:
                        omb_s = " " * 17                          # blank: zero
                    if ln == 5 and v == 0:
                        obs_s = f17(123456.1234567)               # more digits than fp32 holds
                    line += obs_s + omb_s + f"{qc:8d}" + f17(err) + f17(obs - omb)
                out.append(line)
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")


def write_radar_member(path, rows_meta, hdxb_m):
    lines = [f"{len(rows_meta):10d}"]
    for (obs, lon, lat, alt), h in zip(rows_meta, hdxb_m):
        lines.append("".join(fstr(v, 10, 4) + " " for v in (obs, h, lon, lat, alt)))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def make_inputs(d):
    os.makedirs(d, exist_ok=True)
    write_obs_gts(os.path.join(d, "obs_gts"))
    for m in range(1, K + 1):
        # the obs, errors and positions are the same in every member's file (seed 1); omb and
        # QC are the member's own (seed 100 + m)
        write_gts_member(os.path.join(d, f"gts_letkf_{m:03d}"), m, np.random.default_rng(1),
                         np.random.default_rng(100 + m))
    rng = np.random.default_rng(7)
    for var, n in (("VR", 9), ("MR", 6)):
        rows = [(float(rng.normal(0, 8)), float(rng.uniform(119.5, 122.0)),
                 float(rng.uniform(21.8, 25.4)), float(rng.uniform(500, 12000))) for _ in range(n)]
        for m in range(1, K + 1):
            h = rng.normal(0, 8, n)
            write_radar_member(os.path.join(d, f"{var}_letkf_{m:03d}"), rows, h)


LONLAT = np.array([[120.0, 23.7644], [121.51, 25.03], [119.2, 21.5], [122.5, 23.0],
                   [118.0, 20.0], [125.0, 27.5], [120.814, 23.7644], [121.0, 24.0]], np.float32)


def run_harness(d):
    blob = (np.array([K, len(LONLAT)], np.int32).tobytes() +
            np.array([1, 1, 1, 0, 0], np.int32).tobytes() +
            LONLAT[:, 0].tobytes() + LONLAT[:, 1].tobytes())
    with tempfile.TemporaryDirectory() as td:
        for f in os.listdir(d):
            shutil.copy(os.path.join(d, f), td)
        with open(os.path.join(td, "in.bin"), "wb") as f:
            f.write(blob)
        subprocess.run([HARNESS, "ingest", "in.bin", "out.bin"], check=True, cwd=td)
        raw = open(os.path.join(td, "out.bin"), "rb").read()
    off = 0

    def take(n, dt):
        nonlocal off
        a = np.frombuffer(raw, dt, count=n, offset=off).copy()
        off += n * np.dtype(dt).itemsize
        return a
    res = {"xy": take(2 * len(LONLAT), np.float32).reshape(len(LONLAT), 2)}
    gts_types = []
    while True:
        t = int(take(1, np.int32)[0])
        if t == 0:
            break
        nv, n = (int(v) for v in take(2, np.int32))
        ids = np.frombuffer(raw, "S5", count=n, offset=off).copy()
        off += 5 * n
        res[f"g{t}_ids"] = ids
        for key in ("lat", "lon", "alt"):
            res[f"g{t}_{key}"] = take(n, np.float32)
        res[f"g{t}_xyz"] = take(3 * n, np.float32).reshape(n, 3)
        res[f"g{t}_obs"] = take(n * nv, np.float32).reshape(n, nv)
        res[f"g{t}_error"] = take(n * nv, np.float32).reshape(n, nv)
        res[f"g{t}_hdxb"] = take(K * n * nv, np.float32).reshape(K, n, nv)
        res[f"g{t}_qc"] = take(K * n * nv, np.int32).reshape(K, n, nv)
        gts_types.append(t)
    radar_types = []
    while True:
        t = int(take(1, np.int32)[0])
        if t == 0:
            break
        n = int(take(1, np.int32)[0])
        for key in ("obs", "lat", "lon", "alt"):
            res[f"r{t}_{key}"] = take(n, np.float32)
        res[f"r{t}_xyz"] = take(3 * n, np.float32).reshape(n, 3)
        res[f"r{t}_hdxb"] = take(K * n, np.float32).reshape(K, n)
        radar_types.append(t)
    assert off == len(raw)
    res.update(k=np.int32(K), lonlat=LONLAT, gts_types=np.array(gts_types, np.int32),
               radar_types=np.array(radar_types, np.int32))
    return res


def main():
    if not os.path.exists(HARNESS):
        raise SystemExit("build oracle/_ref/ref_harness first (oracle/ref/build_ref.sh)")
    make_inputs(OUTDIR)
    res = run_harness(OUTDIR)
    np.savez(os.path.join(REPO, "tests", "golden", "ingest.npz"), **res)
    print("ingest golden:", sorted(k for k in res if k.endswith("_xyz")))


if __name__ == "__main__":
    main()
