"""ctypes binding of include/cwb_letkf_ingest.h: the host-side obs readers and projection.

These replace the reference's read_gts_omboma / read_alt_info / get_alt
(module_gts_omboma.f90:48-506, 704-1049), read_radar (module_radar.f90:30-118) and
proj_type (module_projection.f90:21-50) on the ranks that read the member obs files; the
result is an abi.ObsSet for cwbl_set_obs or the one-buffer wire format of cwbl/dist.py.
Host code only (no GPU needed).
"""
import ctypes as C

import numpy as np

from . import abi

#: projection_nml defaults (module_config.f90:70-75) = input.nml:13-20
DEFAULT_PROJ = dict(sta_lon=120.0, cen_lat=23.7644, truelat1=10.0, truelat2=40.0)


class Projection(C.Structure):
    _fields_ = [("sta_lon", C.c_float), ("cen_lat", C.c_float), ("truelat1", C.c_float),
                ("truelat2", C.c_float)]


EXPORTS = ["cwbl_lonlat_to_xy", "cwbl_ingest_create", "cwbl_ingest_destroy",
           "cwbl_ingest_read_gts", "cwbl_ingest_read_radar", "cwbl_ingest_obs_set",
           "cwbl_ingest_type_meta", "cwbl_ingest_wire_words", "cwbl_ingest_pack_wire"]

_lib = None


def library():
    global _lib
    if _lib is None:
        lib = abi.load_library()
        vp, cp, fp = C.c_void_p, C.c_char_p, C.POINTER(C.c_float)
        lib.cwbl_lonlat_to_xy.argtypes = [C.POINTER(Projection), C.c_longlong, vp, vp, vp, vp]
        lib.cwbl_lonlat_to_xy.restype = C.c_int
        lib.cwbl_ingest_create.argtypes = [C.c_int, C.POINTER(Projection)]
        lib.cwbl_ingest_create.restype = vp
        lib.cwbl_ingest_destroy.argtypes = [vp]
        lib.cwbl_ingest_destroy.restype = None
        lib.cwbl_ingest_read_gts.argtypes = [vp, C.c_int, cp, cp]
        lib.cwbl_ingest_read_radar.argtypes = [vp, C.c_int, cp, cp]
        lib.cwbl_ingest_obs_set.argtypes = [vp, C.POINTER(abi.ObsSet)]
        lib.cwbl_ingest_type_meta.argtypes = [vp, C.c_int, C.c_int, C.POINTER(C.c_int),
                                              C.POINTER(C.c_int), C.POINTER(C.c_char_p),
                                              C.POINTER(fp), C.POINTER(fp), C.POINTER(fp)]
        lib.cwbl_ingest_wire_words.argtypes = [vp]
        lib.cwbl_ingest_wire_words.restype = C.c_longlong
        lib.cwbl_ingest_pack_wire.argtypes = [vp, vp, C.c_longlong]
        for fn in ("cwbl_ingest_read_gts", "cwbl_ingest_read_radar", "cwbl_ingest_obs_set",
                   "cwbl_ingest_type_meta", "cwbl_ingest_pack_wire"):
            getattr(lib, fn).restype = C.c_int
        _lib = lib
    return _lib


def _check(lib, rc):
    if rc != 0:
        msg = lib.cwbl_last_error()
        raise abi.CwblError(f"{abi.ERRORS.get(rc, rc)}: {msg.decode() if msg else ''}")


def lonlat_to_xy(lon, lat, proj=None):
    """proj_type%lonlat_to_xy (module_projection.f90:37-50) for arrays of lon, lat (degrees):
    (x, y) in metres, fp32."""
    lib = library()
    lon = np.ascontiguousarray(lon, np.float32)
    lat = np.ascontiguousarray(lat, np.float32)
    x, y = np.empty_like(lon), np.empty_like(lon)
    _check(lib, lib.cwbl_lonlat_to_xy(C.byref(Projection(**(proj or DEFAULT_PROJ))), lon.size,
                                      lon.ctypes.data, lat.ctypes.data, x.ctypes.data,
                                      y.ctypes.data))
    return x, y


class Ingest:
    """The obs set of one cycle, read member file by member file (member 0 is the root
    reader whose metadata the distribution broadcasts)."""

    def __init__(self, nmember, proj=None):
        self.lib = library()
        self.k = nmember
        self.h = self.lib.cwbl_ingest_create(nmember, C.byref(Projection(**(proj or DEFAULT_PROJ))))
        if not self.h:
            _check(self.lib, 1)

    def close(self):
        if self.h:
            self.lib.cwbl_ingest_destroy(self.h)
            self.h = None

    __del__ = close

    def read_gts(self, path, obs_gts, member=-1):
        _check(self.lib, self.lib.cwbl_ingest_read_gts(self.h, member, str(path).encode(),
                                                       str(obs_gts).encode()))

    def read_radar(self, path, varname, member=-1):
        _check(self.lib, self.lib.cwbl_ingest_read_radar(self.h, member, str(path).encode(),
                                                         varname.encode()))

    def obs_set(self):
        """abi.ObsSet (host memory) viewing the handle's arrays."""
        s = abi.ObsSet()
        _check(self.lib, self.lib.cwbl_ingest_obs_set(self.h, C.byref(s)))
        s._keep = self  # the views live as long as the handle
        return s

    def types(self):
        """The set as dist.pack_obs_set's per-type dicts (numpy copies, C-order shapes of the
        reference's Fortran layouts)."""
        s = self.obs_set()
        k, out = self.k, []

        def arr(p, n, dt=np.float32):
            return np.ctypeslib.as_array(C.cast(p, C.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                         (n,)).copy() if n else np.zeros(0, dt)
        for e in range(s.n_gts):
            g = s.gts[e]
            n, nv = g.nobs, g.nvar
            out.append(dict(family=0, type_id=g.type_id, nvar=nv, nobs=n,
                            xyz=arr(g.xyz, 3 * n).reshape(n, 3),
                            obs=arr(g.obs, n * nv).reshape(n, nv),
                            error=arr(g.error, n * nv).reshape(n, nv),
                            hdxb=arr(g.hdxb, k * n * nv).reshape(k, n, nv),
                            qc=arr(g.qc, k * n * nv, np.int32).reshape(k, n, nv)))
        for e in range(s.n_radar):
            r = s.radar[e]
            n = r.nobs
            out.append(dict(family=1, type_id=r.type_id, nvar=1, nobs=n,
                            xyz=arr(r.xyz, 3 * n).reshape(n, 3), obs=arr(r.obs, n),
                            hdxb=arr(r.hdxb, k * n).reshape(k, n)))
        return out

    def meta(self, family, type_id):
        """Station ids (GTS), lat, lon, alt of a type."""
        nv, n = C.c_int(), C.c_int()
        ids = C.c_char_p()
        fp = C.POINTER(C.c_float)
        la, lo, al = fp(), fp(), fp()
        _check(self.lib, self.lib.cwbl_ingest_type_meta(self.h, family, type_id, C.byref(nv),
                                                        C.byref(n), C.byref(ids), C.byref(la),
                                                        C.byref(lo), C.byref(al)))
        n = n.value
        cp = (lambda p: np.ctypeslib.as_array(p, (n,)).copy() if n else np.zeros(0, np.float32))
        idl = []
        if family == 0 and n:
            raw = C.string_at(C.cast(ids, C.c_void_p), 5 * n).decode("latin-1")
            idl = [raw[5 * i:5 * i + 5] for i in range(n)]
        return dict(nvar=nv.value, nobs=n, ids=idl, lat=cp(la), lon=cp(lo), alt=cp(al))

    def wire(self):
        """The packed float32 wire buffer (cwbl/dist.py layout), written by the library."""
        nw = self.lib.cwbl_ingest_wire_words(self.h)
        if nw < 0:
            _check(self.lib, 1)
        buf = np.empty(nw, np.float32)
        _check(self.lib, self.lib.cwbl_ingest_pack_wire(self.h, buf.ctypes.data, nw))
        return buf
