"""The reference's configuration surface for a non-Fortran host: `input.nml` read the way
`read_namelist` reads it (module_config.f90:97-150), and the ABI parameter blocks built from
it the way fortran/letkf_core_gpu_config.f90 builds them.

    cfg = namelist.read_namelist("input.nml")
    core = abi.Core(...) / lib.cwbl_init(byref(namelist.init_params(cfg, device)))
    vp = namelist.var_params(cfg, ivar)          # ivar = 1..16, the var_update index

Fortran namelist input (the subset module config needs): groups `&name ... /` read in the
order control, projection, observations, inflation, each searched from where the previous
one ended; `name[%comp...][(i[:j])] = values`; values separated by commas or blanks, `r*c`
repeats, `r*` and empty items leave elements unchanged; logicals T/F/.true./.false. (the
letter after an optional dot decides); quoted strings; `!` comments; names case-insensitive.
Reals are converted by the C library's strtof (correctly rounded, as the Fortran runtime).

Q6: the reference's input.nml writes `radar_nml % dbz % use_it` with blanks
around `%`.  Fujitsu's reader accepts that and amdflang's rejects it; this reader accepts it.
Errors raise NamelistError with the reference's own `stop` message where it has one."""
import ctypes as C
import re

import numpy as np

from . import abi

MAX_VARS = 16  # module_config.f90:4


class NamelistError(ValueError):
    pass


_libc = C.CDLL(None)
_libc.strtof.restype = C.c_float
_libc.strtof.argtypes = [C.c_char_p, C.POINTER(C.c_char_p)]


def _f32(tok):
    s = tok.replace("d", "e").replace("D", "e").encode()
    end = C.c_char_p()
    v = _libc.strtof(s, C.byref(end))
    if end.value:  # trailing characters: not a number
        raise NamelistError(f"bad real value {tok!r}")
    return np.float32(v)


def _int(tok):
    try:
        return int(tok)
    except ValueError:
        raise NamelistError(f"bad integer value {tok!r}") from None


def _logical(tok):
    t = tok[1:] if tok.startswith(".") else tok
    if t[:1].upper() == "T":
        return True
    if t[:1].upper() == "F":
        return False
    raise NamelistError(f"bad logical value {tok!r}")


def _string(tok):
    if len(tok) >= 2 and tok[0] in "'\"" and tok[-1] == tok[0]:
        q = tok[0]
        return tok[1:-1].replace(q + q, q)
    return tok


# ---- the state of module config, with its default initialisers (module_config.f90:7-95) ----
def _radar_var():
    return {"use_it": False, "max_lz_pts": 500, "error": np.float32(1.0),
            "err_rej": np.float32(5.0), "hclr": np.full(MAX_VARS, -1.0, np.float32),
            "vclr": np.full(MAX_VARS, -1.0, np.float32)}


def _gts_var():
    return {"err_muti": np.float32(1.0), "err_rej": np.float32(5.0),
            "is_assim": np.zeros(MAX_VARS, bool)}


def _gts():
    d = {"use_it": False, "max_lz_pts": 500, "hclr": np.full(MAX_VARS, -1.0, np.float32),
         "vclr": np.full(MAX_VARS, -1.0, np.float32)}
    for v in ("u", "v", "t", "p", "q", "tpw", "ref"):
        d[v] = _gts_var()
    return d


def default_config():
    return {
        "control": {"norain_value": np.float32(-5.0), "write_analy_mean": True,
                    "deterministic_update": False, "nt2log": False, "nt2dm": False,
                    "nt2d0": False, "nt2de": False, "nt2d6": False, "wrf_mp_physics": -1,
                    "wrf_mp_hail_opt": -1, "wrf_hypsometric_opt": 2, "nmember": -1,
                    "weight_function": 0, "var_update": [""] * MAX_VARS},
        "projection": {"cen_lon": np.float32(120.814), "cen_lat": np.float32(23.7644),
                       "truelat1": np.float32(10.0), "truelat2": np.float32(40.0),
                       "sta_lon": np.float32(120.0)},
        "observations": {"radar_nml": {v: _radar_var() for v in ("dbz", "vr", "zdr", "kdp")},
                         **{g: _gts() for g in ("synop_nml", "ships_nml", "metar_nml",
                                                "sound_nml", "gpspw_nml")}},
        "inflation": {"multi_infl": np.full(MAX_VARS, 1.0, np.float32),
                      "rtps_alpha": np.full(MAX_VARS, 0.85, np.float32),
                      "rtpp_alpha": np.full(MAX_VARS, 0.85, np.float32),
                      "use_rtps": np.zeros(MAX_VARS, bool), "use_rtpp": np.zeros(MAX_VARS, bool)},
    }


_CONV = {np.float32: _f32, int: _int, bool: _logical, str: _string}


def _kind(v):
    if isinstance(v, np.ndarray):
        return {np.dtype(np.float32): np.float32, np.dtype(bool): bool}[v.dtype]
    if isinstance(v, list):
        return str
    if isinstance(v, (bool, np.bool_)):
        return bool
    if isinstance(v, np.float32):
        return np.float32
    if isinstance(v, int):
        return int
    return str


# ---- tokens ------------------------------------------------------------------------------
_TOK = re.compile(r"""\s*(?:('(?:[^']|'')*'|"(?:[^"]|"")*")|(=)|(,)|(/)|"""
                  r"""(\d+\*(?:'(?:[^']|'')*'|"(?:[^"]|"")*")|[^\s,=/'"]+))""")


def _strip_comments(text):
    out = []
    for line in text.splitlines():
        q, cut = None, len(line)
        for i, ch in enumerate(line):
            if q:
                if ch == q:
                    q = None
            elif ch in "'\"":
                q = ch
            elif ch == "!":
                cut = i
                break
        out.append(line[:cut])
    return "\n".join(out)


def _tokens(body):
    toks, pos = [], 0
    while pos < len(body):
        m = _TOK.match(body, pos)
        if not m or m.end() == pos:
            if body[pos:].strip() == "":
                break
            raise NamelistError(f"cannot read {body[pos:pos + 20]!r}")
        pos = m.end()
        s, eq, comma, slash, word = m.groups()
        toks.append(("str", s) if s else ("=", "=") if eq else (",", ",") if comma else
                    ("/", "/") if slash else ("w", word))
    return toks


def _groups(text):
    """(name, body) of each group in file order; a group ends at a '/' outside strings."""
    text = _strip_comments(text)
    out, pos = [], 0
    start = re.compile(r"[&$]([A-Za-z][A-Za-z0-9_]*)")
    while True:
        m = start.search(text, pos)
        if not m:
            return out
        name = m.group(1).lower()
        i, q = m.end(), None
        while i < len(text):
            ch = text[i]
            if q:
                if ch == q:
                    q = None
            elif ch in "'\"":
                q = ch
            elif ch == "/":
                break
            elif ch in "&$" and text[i + 1:i + 4].lower() == "end":
                break
            i += 1
        out.append((name, text[m.end():i]))
        pos = i + 1


def _assignments(body):
    """[(designator parts, subscript or None, [value tokens or None for null])]."""
    toks = _tokens(body)
    # Q6: join `a % b % c` (and `a(1) % b`) into one designator word
    joined = []
    for t in toks:
        if joined and t[0] == "w" and joined[-1][0] == "w" and (
                t[1].startswith("%") or joined[-1][1].endswith("%")):
            joined[-1] = ("w", joined[-1][1] + t[1])
        else:
            joined.append(t)
    out, i = [], 0
    n = len(joined)
    while i < n:
        if joined[i][0] == ",":
            i += 1
            continue
        if joined[i][0] != "w" or i + 1 >= n or joined[i + 1][0] != "=":
            raise NamelistError(f"expected `name =` at {joined[i][1]!r}")
        des = joined[i][1]
        i += 2
        vals = []
        last_sep = True  # a value may start here
        while i < n:
            kind, tok = joined[i]
            if kind == "w" and i + 1 < n and joined[i + 1][0] == "=":
                break  # the next designator
            if kind == ",":
                if last_sep:
                    vals.append(None)  # null value
                last_sep = True
            else:
                vals.append(tok)
                last_sep = False
            i += 1
        if vals and vals[-1] is None:
            vals.pop()  # the separator before the next designator
        m = re.fullmatch(r"([A-Za-z0-9_%]+?)(?:\((\s*\d+\s*(?::\s*\d+\s*)?)\))?", des)
        if not m:
            raise NamelistError(f"bad designator {des!r}")
        parts = m.group(1).lower().split("%")
        sub = None
        if m.group(2):
            lo, _, hi = m.group(2).partition(":")
            sub = (int(lo), int(hi) if hi else int(lo))
        out.append((parts, sub, vals))
    return out


def _expand(vals):
    out = []
    for v in vals:
        if v is None:
            out.append(None)
            continue
        m = re.fullmatch(r"(\d+)\*(.*)", v)
        if m:
            out.extend([m.group(2) if m.group(2) != "" else None] * int(m.group(1)))
        else:
            out.append(v)
    return out


def _assign(group, parts, sub, vals, gname):
    node = group
    for p in parts[:-1]:
        if not isinstance(node, dict) or p not in node:
            raise NamelistError(f"{'%'.join(parts)} is not in namelist group {gname}")
        node = node[p]
    leaf = parts[-1]
    if not isinstance(node, dict) or leaf not in node or isinstance(node[leaf], dict):
        raise NamelistError(f"{'%'.join(parts)} is not an item of namelist group {gname}")
    cur = node[leaf]
    conv = _CONV[_kind(cur)]
    vals = _expand(vals)
    if isinstance(cur, (np.ndarray, list)):
        lo = sub[0] if sub else 1
        hi = sub[1] if sub else len(cur)
        if lo < 1 or hi > len(cur) or len(vals) > hi - lo + 1:
            raise NamelistError(f"too many values or subscript out of range for {'%'.join(parts)}")
        for k, v in enumerate(vals):
            if v is not None:
                cur[lo - 1 + k] = conv(v)
    else:
        if sub or len(vals) > 1:
            raise NamelistError(f"{'%'.join(parts)} is a scalar")
        if vals and vals[0] is not None:
            node[leaf] = conv(vals[0])


def read_namelist(path_or_text, is_text=False):
    """module config's state after read_namelist (module_config.f90:97-150)."""
    if is_text:
        text = path_or_text
    else:
        try:
            with open(path_or_text) as f:
                text = f.read()
        except OSError:
            raise NamelistError("input.nml doesn't exist...") from None
    cfg = default_config()
    groups = _groups(text)
    pos = 0
    for gname, msg in (("control", "control_nml"), ("projection", "projection_nml"),
                       ("observations", "observations_nml"), ("inflation", "inflation_nml")):
        j = next((i for i in range(pos, len(groups)) if groups[i][0] == gname), None)
        if j is None:
            raise NamelistError(f"read namelist of {msg} fail!")
        try:
            for parts, sub, vals in _assignments(groups[j][1]):
                # the names of a group are matched case-insensitively
                _assign(cfg[gname], parts, sub, vals, gname)
        except NamelistError as e:
            raise NamelistError(f"read namelist of {msg} fail! ({e})") from None
        pos = j + 1
    if cfg["control"]["nmember"] == -1:
        raise NamelistError("Please input ensemble size in control_nml: nmember")
    return cfg


# ---- the ABI blocks (fortran/letkf_core_gpu_config.f90) ------------------------------------
_TUNE_Q = {"QVAPOR", "QRAIN", "QSNOW", "QGRAUP", "QHAIL", "QNRAIN", "QNSNOW", "QNGRAUPEL",
           "QNHAIL"}  # letkf_driver's select case calling letkf_tune_q (:253-278)


def init_params(cfg, device=0):
    c = cfg["control"]
    return abi.InitParams(int(c["nmember"]), int(device), int(c["weight_function"]),
                          float(c["norain_value"]), 0, 0, 0)


def projection(cfg):
    from .ingest import Projection
    p = cfg["projection"]
    return Projection(float(p["sta_lon"]), float(p["cen_lat"]), float(p["truelat1"]),
                      float(p["truelat2"]))


def var_params(cfg, ivar):
    """cwbl_var_params of var_update entry ivar (1-based, as letkf_driver's ivar)."""
    if not 1 <= ivar <= MAX_VARS:
        raise NamelistError(f"ivar {ivar} outside 1..{MAX_VARS}")
    i = ivar - 1
    inf, obs = cfg["inflation"], cfg["observations"]
    vp = abi.VarParams()
    vp.multi_infl = float(inf["multi_infl"][i])
    vp.use_rtpp, vp.rtpp_alpha = int(inf["use_rtpp"][i]), float(inf["rtpp_alpha"][i])
    vp.use_rtps, vp.rtps_alpha = int(inf["use_rtps"][i]), float(inf["rtps_alpha"][i])
    vp.tune_q = int(cfg["control"]["var_update"][i].strip() in _TUNE_Q)
    for t in list(vp.gts) + list(vp.radar):  # `off` in the Fortran glue
        t.use_it, t.max_lz_pts, t.hclr, t.vclr = 0, 0, -1.0, -1.0
        for e in range(abi.MAX_NVAR):
            t.err_muti[e], t.err_rej[e], t.is_assim[e] = 1.0, 5.0, 0

    def common(g, t):
        t.use_it, t.max_lz_pts = int(g["use_it"]), int(g["max_lz_pts"])
        t.hclr, t.vclr = float(g["hclr"][i]), float(g["vclr"][i])

    def put(t, e, v):
        t.err_muti[e], t.err_rej[e] = float(v["err_muti"]), float(v["err_rej"])
        t.is_assim[e] = int(v["is_assim"][i])

    for name, tid in (("synop_nml", abi.GTS_SYNOP), ("metar_nml", abi.GTS_METAR),
                      ("ships_nml", abi.GTS_SHIPS)):
        t = vp.gts[tid - 1]
        common(obs[name], t)
        for e, v in enumerate(("u", "v", "t", "p", "q")):
            put(t, e, obs[name][v])
    t = vp.gts[abi.GTS_SOUND - 1]
    common(obs["sound_nml"], t)
    for e, v in enumerate(("u", "v", "t", "q")):
        put(t, e, obs["sound_nml"][v])
    t = vp.gts[abi.GTS_GPSPW - 1]
    common(obs["gpspw_nml"], t)
    put(t, 0, obs["gpspw_nml"]["tpw"])
    for name, tid in (("dbz", abi.RADAR_DBZ), ("vr", abi.RADAR_VR), ("zdr", abi.RADAR_ZDR),
                      ("kdp", abi.RADAR_KDP)):
        r, t = obs["radar_nml"][name], vp.radar[tid - 1]
        common(r, t)
        t.err_muti[0], t.err_rej[0] = float(r["error"]), float(r["err_rej"])
    return vp


def var_names(cfg):
    """The var_update entries up to the first blank one, 1-based position = ivar: letkf_driver
    leaves its variable loop at the first blank entry (module_letkf_core.f90:59-60,
    `if(len_trim(var_update(ivar)) == 0) exit`), so names after a gap are never analysed."""
    out = []
    for v in cfg["control"]["var_update"]:
        if not v.strip():
            break
        out.append(v.strip())
    return out
