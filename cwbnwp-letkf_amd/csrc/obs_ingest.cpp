// obs_ingest.cpp — host-side observation ingest and Lambert projection (cwb_letkf_ingest.h).
//
// The reference reads its observations with Fortran formatted I/O (module_gts_omboma.f90:
// 48-506, 704-1049; module_radar.f90:30-118) and projects them with proj_type
// (module_projection.f90:21-50).  This file restates those readers in C++:
//   - a Fortran edit-descriptor reader (A, I, F, X, repeat groups) for the fixed record
//     formats and for the INFO/EACH formats that obs_gts carries in its own header
//     (read_alt_info, :767-770); input conversion is the standard's: blanks ignored, an
//     all-blank field is zero, F fields without a decimal point take d implied decimals,
//     values rounded to nearest (strtof / strtol);
//   - get_alt (:1032-1049) as one hash map per report type (first station of an id wins, as
//     the reference's linear scan returns the first match), so a report costs O(1) instead of
//     O(stations);
//   - lonlat_to_xy in fp32 with the same libm calls and operation order (cotan(x) as
//     1./tan(x), the definition the reference's own compiled check uses, oracle/ref).
// Host code only; compiled with -ffp-contract=off like the rest of the library.
#include "../../include/cwb_letkf_ingest.h"
#include "cwbl_internal.h"

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

namespace cwbl {
namespace {

// ---- Fortran formatted input ------------------------------------------------------------
struct Desc {
  char kind;  // 'A', 'I', 'F', 'X'
  int w, d;   // w < 0: A without a width (the item's length)
};

// Parses a format like "(3(F12.3,I4,F7.2),11X,A40)" into a flat descriptor list (repeat
// counts expanded).  Returns false on anything outside A/I/F/E/X and groups.
bool parse_format(const std::string &f, std::vector<Desc> &out) {
  size_t i = 0;
  std::vector<std::pair<size_t, int>> stack;  // (start index in out, repeat)
  auto skip = [&]() { while (i < f.size() && (f[i] == ' ' || f[i] == ',')) ++i; };
  auto num = [&](int def) {
    if (i >= f.size() || !isdigit((unsigned char)f[i])) return def;
    int v = 0;
    while (i < f.size() && isdigit((unsigned char)f[i])) v = 10 * v + (f[i++] - '0');
    return v;
  };
  skip();
  if (i >= f.size() || f[i] != '(') return false;
  ++i;
  stack.push_back({0, 1});
  while (true) {
    skip();
    if (i >= f.size()) return false;
    if (f[i] == ')') {
      ++i;
      auto [start, rep] = stack.back();
      stack.pop_back();
      std::vector<Desc> grp(out.begin() + start, out.end());
      for (int r = 1; r < rep; ++r) out.insert(out.end(), grp.begin(), grp.end());
      if (stack.empty()) return true;
      continue;
    }
    const int rep = num(1);
    skip();
    if (i >= f.size()) return false;
    const char c = (char)toupper((unsigned char)f[i]);
    if (c == '(') {
      ++i;
      stack.push_back({out.size(), rep});
      continue;
    }
    ++i;
    if (c == 'X') {
      out.push_back({'X', rep, 0});
    } else if (c == 'A') {
      const int w = num(-1);
      for (int r = 0; r < rep; ++r) out.push_back({'A', w, 0});
    } else if (c == 'I') {
      const int w = num(-1);
      if (w <= 0) return false;
      for (int r = 0; r < rep; ++r) out.push_back({'I', w, 0});
    } else if (c == 'F' || c == 'E' || c == 'D') {
      const int w = num(-1);
      if (w <= 0 || i >= f.size() || f[i] != '.') return false;
      ++i;
      const int d = num(-1);
      if (d < 0) return false;
      for (int r = 0; r < rep; ++r) out.push_back({'F', w, d});
    } else {
      return false;
    }
  }
}

// Fortran numeric input conversion of one field (BLANK='NULL': blanks are ignored).
bool conv_int(const std::string &fld, int &v) {
  std::string s;
  for (char c : fld)
    if (c != ' ') s += c;
  if (s.empty()) { v = 0; return true; }
  char *end = nullptr;
  const long x = std::strtol(s.c_str(), &end, 10);
  if (*end != '\0') return false;
  v = (int)x;
  return true;
}

bool conv_real(const std::string &fld, int d, float &v) {
  std::string s;
  for (char c : fld)
    if (c != ' ') s += c;
  if (s.empty()) { v = 0.0f; return true; }
  // mantissa [sign] digits [. digits], then an optional exponent: E/D [sign] digits, or a
  // bare signed integer
  size_t i = 0;
  std::string sign, digs;
  int point = -1;
  if (s[i] == '+' || s[i] == '-') sign = s[i++];
  for (; i < s.size() && (isdigit((unsigned char)s[i]) || s[i] == '.'); ++i) {
    if (s[i] == '.') {
      if (point >= 0) return false;
      point = (int)digs.size();
    } else {
      digs += s[i];
    }
  }
  if (digs.empty()) return false;
  long exp10 = 0;
  if (i < s.size()) {
    if (s[i] == 'E' || s[i] == 'e' || s[i] == 'D' || s[i] == 'd') ++i;
    if (i >= s.size()) return false;
    char *end = nullptr;
    exp10 = std::strtol(s.c_str() + i, &end, 10);
    if (*end != '\0' || end == s.c_str() + i) return false;
  }
  // value = 0.digs-with-point * 10^..: point absent -> d implied decimals
  const long frac = point >= 0 ? (long)digs.size() - point : d;
  const std::string norm = sign + digs + "e" + std::to_string(exp10 - frac);
  char *end = nullptr;
  v = std::strtof(norm.c_str(), &end);
  return *end == '\0';
}

// One record under a parsed format: items are consumed in order, X descriptors move the
// position; past the end of the record the line reads as blanks (PAD='YES').
struct RecordReader {
  const std::string &rec;
  const std::vector<Desc> &fmt;
  size_t pos = 0, di = 0;
  RecordReader(const std::string &r, const std::vector<Desc> &f) : rec(r), fmt(f) {}
  std::string take(int w) {
    std::string s = pos < rec.size() ? rec.substr(pos, (size_t)w) : std::string();
    s.resize((size_t)w, ' ');
    pos += (size_t)w;
    return s;
  }
  const Desc *next() {
    while (di < fmt.size() && fmt[di].kind == 'X') pos += (size_t)fmt[di++].w;
    return di < fmt.size() ? &fmt[di++] : nullptr;
  }
  bool a(std::string &out, int len) {  // character(len=len) item
    const Desc *e = next();
    if (!e || e->kind != 'A') return false;
    const int w = e->w < 0 ? len : e->w;
    const std::string f = take(w);
    out = w >= len ? f.substr((size_t)(w - len)) : f + std::string((size_t)(len - w), ' ');
    return true;
  }
  bool i(int &v) {
    const Desc *e = next();
    return e && e->kind == 'I' && conv_int(take(e->w), v);
  }
  bool f(float &v) {
    const Desc *e = next();
    return e && e->kind == 'F' && conv_real(take(e->w), e->d, v);
  }
};

std::string rtrim(const std::string &s) {
  size_t e = s.size();
  while (e > 0 && s[e - 1] == ' ') --e;
  return s.substr(0, e);
}
std::string strip(const std::string &s) {
  size_t b = 0;
  while (b < s.size() && s[b] == ' ') ++b;
  return rtrim(s.substr(b));
}

bool getline_rec(std::istream &in, std::string &line) {
  if (!std::getline(in, line)) return false;
  if (!line.empty() && line.back() == '\r') line.pop_back();
  return true;
}

// ---- projection (module_projection.f90) --------------------------------------------------
struct Proj {
  float lon0, n, f, rh0;
};
constexpr float kPi = 3.14159274101257324f;  // acos(-1.) in real(4) (module_param.f90:105)
constexpr float kD2r = kPi / 180.0f;         // :106
constexpr float kEarthRadius = 6.37122e6f;   // :108
inline float cotan(float x) { return 1.0f / tanf(x); }

Proj proj_init(const cwbl_projection &p) {  // proj_init, :21-35
  Proj q;
  const float lat0 = p.cen_lat * kD2r, lat1 = p.truelat1 * kD2r, lat2 = p.truelat2 * kD2r;
  q.lon0 = p.sta_lon * kD2r;
  q.n = logf(cosf(lat1) / cosf(lat2)) /
        logf(tanf(0.5f * (0.5f * kPi + lat2)) * cotan(0.5f * (0.5f * kPi + lat1)));
  q.f = cosf(lat1) * expf(q.n * logf(tanf(0.5f * (0.5f * kPi + lat1)))) / q.n;
  q.rh0 = kEarthRadius * q.f * expf(q.n * logf(cotan(0.5f * (0.5f * kPi + lat0))));
  return q;
}

inline void lonlat_to_xy(const Proj &q, float lon, float lat, float &x, float &y) {  // :37-50
  const float rh = kEarthRadius * q.f * expf(q.n * logf(cotan(0.5f * (0.5f * kPi + lat * kD2r))));
  const float dlon = q.n * (lon * kD2r - q.lon0);
  x = rh * sinf(dlon);
  y = q.rh0 - rh * cosf(dlon);
}

// ---- the obs set --------------------------------------------------------------------------
struct GtsType {
  int nvar = 0, nobs = -1;  // nobs < 0: no file has had this type yet
  bool meta = false;        // member 0's arrays are in
  std::string ids;          // 5 characters per obs
  std::vector<float> lat, lon, alt, xyz, obs, error, hdxb;
  std::vector<int> qc;
  std::vector<char> have;   // member slices filled
};
struct RadarType {
  int nobs = -1;
  bool meta = false;
  std::vector<float> lat, lon, alt, xyz, obs, hdxb;
  std::vector<char> have;
};

// read_alt_info (:704-1030): per report type, station id -> altitude per level
struct AltTable {
  struct Station { std::vector<float> alt; };
  std::vector<Station> stations;
  std::unordered_map<std::string, int> index;  // rtrim(id(1:20)) -> first station
};

}  // namespace
}  // namespace cwbl

using namespace cwbl;

struct cwbl_ingest {
  int k = 0;
  Proj proj{};
  GtsType gts[CWBL_NUM_GTS_TYPES + 1];
  RadarType radar[CWBL_NUM_RADAR_TYPES + 1];
  std::string alt_path;                       // the obs_gts the tables below come from
  AltTable alt[CWBL_NUM_GTS_TYPES + 1];
  std::vector<cwbl_gts_obs> gview;
  std::vector<cwbl_radar_obs> rview;
};

namespace cwbl {
namespace {

int ifail(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return set_last_error(CWBL_ERR_ARG, buf);
}

constexpr int SOUND = 1, SYNOP = 2, PILOT = 3, SATEM = 4, GEOAMV = 5, POLARAMV = 6, AIREP = 7,
              GPSPW = 8, GPSREF = 9, METAR = 10, SHIPS = 11, SSMT1 = 14, SSMT2 = 15,
              QSCAT = 16, PROFILER = 17, BUOY = 18, BOGUS = 19, AIRSR = 23, SONDE_SFC = 24,
              MTGIRS = 25, TAMDAR = 26, TAMDAR_SFC = 27;

int read_alt_info(cwbl_ingest &h, const std::string &path) {
  if (h.alt_path == path) return CWBL_OK;  // parsed once per obs_gts file
  for (auto &t : h.alt) t = AltTable{};
  h.alt_path.clear();
  std::ifstream in(path);
  if (!in) return ifail("read_alt_info: cannot open %s", path.c_str());
  std::string line;
  // five count records (:727-749); the counts size the reference's arrays, here only checked
  std::vector<Desc> f1, f6;
  parse_format("(A6,1X,I7,2X,A6,1X,F8.0)", f1);
  parse_format("(6(A6,1X,I7,2X))", f6);
  {
    if (!getline_rec(in, line)) return ifail("read_alt_info: %s is empty", path.c_str());
    RecordReader r(line, f1);
    std::string s;
    int total;
    float missing;
    if (!r.a(s, 160) || !r.i(total) || !r.a(s, 160) || !r.f(missing))
      return ifail("read_alt_info: bad TOTAL record in %s", path.c_str());
  }
  for (int rec = 0; rec < 4; ++rec) {
    if (!getline_rec(in, line)) return ifail("read_alt_info: short header in %s", path.c_str());
    RecordReader r(line, f6);
    const int items = rec == 3 ? 4 : 6;
    for (int it = 0; it < items; ++it) {
      std::string s;
      int c;
      if (!r.a(s, 160) || !r.i(c))
        return ifail("read_alt_info: bad count record %d in %s", rec + 2, path.c_str());
    }
  }
  while (true) {  // skip to the EACH line (:762-765)
    if (!getline_rec(in, line)) return ifail("read_alt_info: no EACH line in %s", path.c_str());
    if (line.compare(0, 6, "EACH  ") == 0) break;
  }
  // read(11,'(A,1X,A)') fmt_name(10), info_fmt(45), .. srfc_fmt(29), .. each_fmt(60)
  std::string info_fmt, each_fmt;
  const int flen[3] = {45, 29, 60};
  for (int q = 0; q < 3; ++q) {
    if (!getline_rec(in, line)) return ifail("read_alt_info: missing *_FMT line in %s", path.c_str());
    std::string body = line.size() > 11 ? line.substr(11) : std::string();
    body.resize((size_t)flen[q], ' ');
    if (q == 0) info_fmt = body;
    if (q == 2) each_fmt = body;
  }
  std::vector<Desc> finfo, feach;
  if (!parse_format(info_fmt, finfo) || !parse_format(each_fmt, feach))
    return ifail("read_alt_info: unreadable INFO/EACH format in %s", path.c_str());
  if (!getline_rec(in, line)) return ifail("read_alt_info: no data in %s", path.c_str());
  auto each_alt = [&](float &alt) {  // 9 items (3 x value, qc, error), then the height
    if (!getline_rec(in, line)) return false;
    RecordReader r(line, feach);
    float fr;
    int ir;
    for (int q = 0; q < 3; ++q)
      if (!r.f(fr) || !r.i(ir) || !r.f(fr)) return false;
    return r.f(alt);
  };
  while (getline_rec(in, line)) {
    RecordReader r(line, finfo);
    std::string plat, date, source, id;
    int level;
    float lat, lon, elev;
    if (!r.a(plat, 160) || !r.a(date, 19) || !r.a(source, 40) || !r.i(level) || !r.f(lat) ||
        !r.f(lon) || !r.f(elev) || !r.a(id, 40))
      return ifail("read_alt_info: bad report line in %s: '%s'", path.c_str(), line.c_str());
    int fm = 0;
    if (!conv_int(plat[5] == ' ' ? plat.substr(3, 2) : plat.substr(3, 3), fm))
      return ifail("read_alt_info: bad platform '%s' in %s", plat.substr(0, 12).c_str(), path.c_str());
    int type = 0, levels = 1;
    bool has_each = true;
    switch (fm) {
      case 12: type = SYNOP; break;
      case 13: case 17: type = SHIPS; break;
      case 15: case 16: type = METAR; break;
      case 32: case 33: case 34: type = PILOT; levels = level; break;
      case 35: case 36: case 37: case 38: type = SOUND; levels = level; break;
      case 101: type = TAMDAR; levels = level; break;
      case 161: type = MTGIRS; levels = level; break;
      case 86: type = SATEM; levels = level; break;
      case 42: case 96: case 97: type = AIREP; levels = level; break;
      case 111: case 114: type = GPSPW; has_each = false; break;
      case 116: type = GPSREF; break;
      case 121: type = SSMT1; levels = level; break;
      case 122: type = SSMT2; levels = level; break;
      case 281: type = QSCAT; levels = level; break;
      case 132: type = PROFILER; levels = level; break;
      case 135: type = BOGUS; levels = level; break;
      case 18: case 19: type = BUOY; break;
      case 133: type = AIRSR; levels = level; break;
      default:
        // the reference has no branch here and would read the next record as a report
        return ifail("read_alt_info: report type FM-%d is not read by the reference (%s)", fm,
                     path.c_str());
    }
    std::string srfc;
    if (!getline_rec(in, srfc)) return ifail("read_alt_info: missing SRFC record in %s", path.c_str());
    AltTable &t = h.alt[type];
    AltTable::Station st;
    if (!has_each) {
      st.alt.push_back(elev);  // gpspw: the report's elevation (:915)
    } else {
      st.alt.resize((size_t)std::max(levels, 0));
      for (int q = 0; q < levels; ++q)
        if (!each_alt(st.alt[(size_t)q]))
          return ifail("read_alt_info: bad EACH record (FM-%d, '%s') in %s", fm,
                       rtrim(id).c_str(), path.c_str());
    }
    // gtsalt(type)%id(n) = trim(id): character(len=20), so the first 20 characters
    const std::string key = rtrim(id.substr(0, 20));
    t.index.emplace(key, (int)t.stations.size());  // first station of an id wins (:1041-1045)
    t.stations.push_back(std::move(st));
  }
  h.alt_path = path;
  return CWBL_OK;
}

int get_alt(const cwbl_ingest &h, int type, const std::string &id5, int level, float &alt) {
  const AltTable &t = h.alt[type];
  const auto it = t.index.find(rtrim(id5));
  if (it == t.index.end())
    return ifail("get_alt: station '%s' (type %d) not in %s (\"ID not found!!\")",
                 rtrim(id5).c_str(), type, h.alt_path.c_str());
  const auto &a = t.stations[(size_t)it->second].alt;
  if (level < 1 || level > (int)a.size())
    return ifail("get_alt: station '%s' (type %d) has %zu levels, level %d requested",
                 rtrim(id5).c_str(), type, a.size(), level);
  alt = a[(size_t)(level - 1)];
  return CWBL_OK;
}

int member_of(const char *file, int member) {
  if (member >= 0) return member;
  const size_t n = std::strlen(file);
  int v = 0;
  if (n < 3 || !conv_int(std::string(file + n - 3, 3), v)) return -1;
  return v - 1;  // read(filename(l-2:l), '(i3)') iproc; iproc = iproc - 1 (:82-84)
}

// One report line of gts_omboma, '(2i8,a5,2f9.2,f17.7,5(2f17.7,i8,2f17.7))' (:135)
struct GtsLine {
  std::string id;
  float lat = 0, lon = 0, pre = 0;
  float obs[5] = {}, omb[5] = {}, err[5] = {};
  int qc[5] = {};
};
bool read_gts_line(std::istream &in, int nvar, GtsLine &g) {
  // parsed once, thread-safely (a magic static): hosts may read member files concurrently
  static const std::vector<Desc> fmt = [] {
    std::vector<Desc> f;
    parse_format("(2i8,a5,2f9.2,f17.7,5(2f17.7,i8,2f17.7))", f);
    return f;
  }();
  std::string line;
  if (!getline_rec(in, line)) return false;
  RecordReader r(line, fmt);
  int kk, l;
  float oma;
  if (!r.i(kk) || !r.i(l) || !r.a(g.id, 5) || !r.f(g.lat) || !r.f(g.lon) || !r.f(g.pre))
    return false;
  for (int v = 0; v < nvar; ++v)
    if (!r.f(g.obs[v]) || !r.f(g.omb[v]) || !r.i(g.qc[v]) || !r.f(g.err[v]) || !r.f(oma))
      return false;
  return true;
}

}  // namespace

// set_last_error is defined in cwbl_abi.hip (cwbl_last_error)

}  // namespace cwbl

extern "C" {

int cwbl_lonlat_to_xy(const cwbl_projection *p, long long n, const float *lon, const float *lat,
                      float *x, float *y) {
  if (!p || n < 0 || (n > 0 && (!lon || !lat || !x || !y)))
    return ifail("cwbl_lonlat_to_xy: bad arguments");
  const Proj q = proj_init(*p);
  for (long long i = 0; i < n; ++i) lonlat_to_xy(q, lon[i], lat[i], x[i], y[i]);
  return CWBL_OK;
}

cwbl_ingest *cwbl_ingest_create(int nmember, const cwbl_projection *p) {
  if (nmember < 1 || nmember > CWBL_MAX_MEMBERS || !p) {
    ifail("cwbl_ingest_create: bad arguments (nmember %d)", nmember);
    return nullptr;
  }
  auto *h = new cwbl_ingest;
  h->k = nmember;
  h->proj = proj_init(*p);
  return h;
}

void cwbl_ingest_destroy(cwbl_ingest *h) { delete h; }

int cwbl_ingest_read_gts(cwbl_ingest *h, int member, const char *gts_file,
                         const char *obs_gts_file) {
  if (!h || !gts_file || !obs_gts_file) return ifail("cwbl_ingest_read_gts: null argument");
  const int m = member_of(gts_file, member);
  if (m < 0 || m >= h->k)
    return ifail("cwbl_ingest_read_gts: member %d of %s outside 0..%d", m, gts_file, h->k - 1);
  if (int rc = read_alt_info(*h, obs_gts_file)) return rc;
  std::ifstream in(gts_file);
  if (!in) return ifail("open gts_omboma error: %s", gts_file);
  const size_t k = (size_t)h->k;
  std::string line;
  std::vector<Desc> fhdr, f2i;
  parse_format("(a20,i8)", fhdr);
  parse_format("(2i8)", f2i);
  while (getline_rec(in, line)) {  // report: do (:92-502)
    RecordReader rh(line, fhdr);
    std::string iv_type;
    int nobs;
    if (!rh.a(iv_type, 20) || !rh.i(nobs)) return ifail("read gts_omboma error: %s", gts_file);
    const std::string name = strip(iv_type);
    int type = 0, nvar = 0;
    bool vertical = false;
    if (name == "synop") { type = SYNOP; nvar = 5; }
    else if (name == "ships") { type = SHIPS; nvar = 5; }
    else if (name == "buoy") { type = BUOY; nvar = 5; }
    else if (name == "metar") { type = METAR; nvar = 5; }
    else if (name == "sonde_sfc") { type = SONDE_SFC; nvar = 5; }
    else if (name == "tamdar_sfc") { type = TAMDAR_SFC; nvar = 5; }
    else if (name == "pilot") { type = PILOT; nvar = 2; vertical = true; }
    else if (name == "profiler") { type = PROFILER; nvar = 2; vertical = true; }
    else if (name == "geoamv") { type = GEOAMV; nvar = 2; vertical = true; }
    else if (name == "qscat") { type = QSCAT; nvar = 2; vertical = true; }
    else if (name == "polaramv") { type = POLARAMV; nvar = 2; vertical = true; }
    else if (name == "gpspw") { type = GPSPW; nvar = 1; }
    else if (name == "sound") { type = SOUND; nvar = 4; vertical = true; }
    else if (name == "tamdar") { type = TAMDAR; nvar = 4; vertical = true; }
    else if (name == "airep") { type = AIREP; nvar = 4; vertical = true; }
    else if (name == "gpsref") { type = GPSREF; nvar = 1; vertical = true; }
    if (nobs <= 0) continue;  // `if(nobs > 0)` of every branch
    if (type == 0)
      return ifail("gts_omboma %s: '%s' has %d reports but is not read by the reference",
                   gts_file, name.c_str(), nobs);
    // reports -> rows (vertical types: one row per level, :189-270)
    std::vector<GtsLine> rows;
    std::vector<float> alts;
    for (int n = 0; n < nobs; ++n) {
      if (!getline_rec(in, line)) return ifail("gts_omboma %s: short %s section", gts_file, name.c_str());
      RecordReader rr(line, f2i);
      int nlev, nreq;
      if (!rr.i(nlev) || !rr.i(nreq)) return ifail("gts_omboma %s: bad report line", gts_file);
      const int nl = vertical ? nlev : 1;  // surface types read one line per report (:131-147)
      std::vector<GtsLine> lv((size_t)std::max(nl, 0));
      for (int q = 0; q < nl; ++q)
        if (!read_gts_line(in, nvar, lv[(size_t)q]))
          return ifail("gts_omboma %s: bad data line (%s report %d)", gts_file, name.c_str(), n + 1);
      for (int q = 0; q < nl; ++q) {
        float a = 0.0f;
        if (type == GPSPW || type == GPSREF) {
          a = lv[(size_t)q].pre;  // the f17.7 after lon holds alt for these (:295-299, :445-449)
        } else if (!vertical) {
          if (int rc = get_alt(*h, type, lv[(size_t)q].id, 1, a)) return rc;  // :149
        } else {
          if (int rc = get_alt(*h, type, lv[(size_t)q].id, q + 1, a)) return rc;  // :218, :361
        }
        alts.push_back(a);
      }
      // vert(n)%id is one scalar per report: every level takes the last line's id (:256)
      if (vertical)
        for (int q = 0; q < nl; ++q) lv[(size_t)q].id = lv[(size_t)nl - 1].id;
      rows.insert(rows.end(), lv.begin(), lv.end());
    }
    GtsType &t = h->gts[type];
    const int total = (int)rows.size();
    if (t.nobs >= 0 && (t.nobs != total || t.nvar != nvar))
      return ifail("gts_omboma %s: %s has %d obs, another member's file had %d", gts_file,
                   name.c_str(), total, t.nobs);
    if (t.nobs < 0) {
      t.nobs = total;
      t.nvar = nvar;
      const size_t nv = (size_t)nvar * (size_t)total;
      t.hdxb.assign(nv * k, 0.0f);
      t.qc.assign(nv * k, 0);
      t.have.assign(k, 0);
    }
    const size_t nv = (size_t)nvar * (size_t)total;
    if (m == 0) {  // the root reader's arrays (gts_distribute broadcasts them)
      t.ids.clear();
      t.lat.resize((size_t)total); t.lon.resize((size_t)total); t.alt.resize((size_t)total);
      t.xyz.resize(3 * (size_t)total); t.obs.resize(nv); t.error.resize(nv);
      for (int i = 0; i < total; ++i) {
        const GtsLine &g = rows[(size_t)i];
        t.ids += g.id;
        t.lat[(size_t)i] = g.lat;
        t.lon[(size_t)i] = g.lon;
        t.alt[(size_t)i] = alts[(size_t)i];
        lonlat_to_xy(h->proj, g.lon, g.lat, t.xyz[3 * (size_t)i], t.xyz[3 * (size_t)i + 1]);
        t.xyz[3 * (size_t)i + 2] = alts[(size_t)i];
        for (int v = 0; v < nvar; ++v) {
          t.obs[(size_t)i * nvar + v] = g.obs[v];
          t.error[(size_t)i * nvar + v] = g.err[v];
        }
      }
      t.meta = true;
    }
    for (int i = 0; i < total; ++i)  // hdxb = obs - omb of this member's file (:171)
      for (int v = 0; v < nvar; ++v) {
        const GtsLine &g = rows[(size_t)i];
        t.hdxb[(size_t)m * nv + (size_t)i * nvar + v] = g.obs[v] - g.omb[v];
        t.qc[(size_t)m * nv + (size_t)i * nvar + v] = g.qc[v];
      }
    t.have[(size_t)m] = 1;
  }
  return CWBL_OK;
}

int cwbl_ingest_read_radar(cwbl_ingest *h, int member, const char *file, const char *varname) {
  if (!h || !file || !varname) return ifail("cwbl_ingest_read_radar: null argument");
  const int m = member_of(file, member);
  if (m < 0 || m >= h->k)
    return ifail("cwbl_ingest_read_radar: member %d of %s outside 0..%d", m, file, h->k - 1);
  int type = 0;  // :70-79
  const std::string vn(varname);
  if (vn == "VR") type = CWBL_RADAR_VR;
  else if (vn == "MR") type = CWBL_RADAR_DBZ;
  else if (vn == "MD") type = CWBL_RADAR_ZDR;
  else if (vn == "MK") type = CWBL_RADAR_KDP;
  else return ifail("read_radar: unknown variable '%s'", varname);
  std::ifstream in(file);
  if (!in) return ifail("open %s_letkf error: %s", varname, file);
  std::string line;
  std::vector<Desc> fn, frow;
  parse_format("(i10)", fn);
  parse_format("(5(f10.4,1x))", frow);
  if (!getline_rec(in, line)) return CWBL_OK;  // EOF before the count: no data (:53-57)
  int nobs;
  {
    RecordReader r(line, fn);
    if (!r.i(nobs)) return ifail("read %s_letkf nobs error: %s", varname, file);
  }
  if (nobs <= 0) return CWBL_OK;
  RadarType &t = h->radar[type];
  if (t.nobs >= 0 && t.nobs != nobs)
    return ifail("read_radar %s: %d obs, another member's file had %d", file, nobs, t.nobs);
  const size_t n = (size_t)nobs, k = (size_t)h->k;
  if (t.nobs < 0) {
    t.nobs = nobs;
    t.hdxb.assign(n * k, 0.0f);
    t.have.assign(k, 0);
  }
  std::vector<float> obs(n), hd(n), lon(n), lat(n), alt(n);
  for (size_t i = 0; i < n; ++i) {
    // Q5: the reference uses the record before checking iostat; a short file is an error here
    if (!getline_rec(in, line))
      return ifail("read %s_letkf data error: %s ends after %zu of %d rows", varname, file, i, nobs);
    RecordReader r(line, frow);
    if (!r.f(obs[i]) || !r.f(hd[i]) || !r.f(lon[i]) || !r.f(lat[i]) || !r.f(alt[i]))
      return ifail("read %s_letkf data error: %s row %zu", varname, file, i + 1);
  }
  if (m == 0) {  // the root reader's arrays (radar_distribute broadcasts them)
    t.obs = obs; t.lon = lon; t.lat = lat; t.alt = alt;
    t.xyz.resize(3 * n);
    for (size_t i = 0; i < n; ++i) {
      lonlat_to_xy(h->proj, lon[i], lat[i], t.xyz[3 * i], t.xyz[3 * i + 1]);  // :96-98
      t.xyz[3 * i + 2] = alt[i];
    }
    t.meta = true;
  }
  std::memcpy(&t.hdxb[(size_t)m * n], hd.data(), n * sizeof(float));  // hdxb(n, iproc)
  t.have[(size_t)m] = 1;
  return CWBL_OK;
}

int cwbl_ingest_obs_set(cwbl_ingest *h, cwbl_obs_set *out) {
  if (!h || !out) return ifail("cwbl_ingest_obs_set: null argument");
  h->gview.clear();
  h->rview.clear();
  for (int t = 1; t <= CWBL_NUM_GTS_TYPES; ++t) {
    GtsType &g = h->gts[t];
    if (g.nobs <= 0) continue;
    for (int m = 0; m < h->k; ++m)
      if (!g.have[(size_t)m] || !g.meta)
        return ifail("cwbl_ingest_obs_set: GTS type %d lacks member %d's file", t, g.meta ? m : 0);
    cwbl_gts_obs o{};
    o.type_id = t; o.nvar = g.nvar; o.nobs = g.nobs;
    o.xyz = g.xyz.data(); o.obs = g.obs.data(); o.error = g.error.data();
    o.hdxb = g.hdxb.data(); o.qc = g.qc.data();
    h->gview.push_back(o);
  }
  for (int t = 1; t <= CWBL_NUM_RADAR_TYPES; ++t) {
    RadarType &r = h->radar[t];
    if (r.nobs <= 0) continue;
    for (int m = 0; m < h->k; ++m)
      if (!r.have[(size_t)m] || !r.meta)
        return ifail("cwbl_ingest_obs_set: radar type %d lacks member %d's file", t, r.meta ? m : 0);
    cwbl_radar_obs o{};
    o.type_id = t; o.nobs = r.nobs;
    o.xyz = r.xyz.data(); o.obs = r.obs.data(); o.hdxb = r.hdxb.data();
    h->rview.push_back(o);
  }
  std::memset(out, 0, sizeof *out);
  out->n_gts = (int)h->gview.size();
  out->n_radar = (int)h->rview.size();
  out->gts = h->gview.empty() ? nullptr : h->gview.data();
  out->radar = h->rview.empty() ? nullptr : h->rview.data();
  out->memory = CWBL_MEM_HOST;
  return CWBL_OK;
}

int cwbl_ingest_type_meta(cwbl_ingest *h, int family, int type_id, int *nvar, int *nobs,
                          const char **ids, const float **lat, const float **lon,
                          const float **alt) {
  if (!h) return ifail("cwbl_ingest_type_meta: null handle");
  if (family == 0 && type_id >= 1 && type_id <= CWBL_NUM_GTS_TYPES) {
    const GtsType &g = h->gts[type_id];
    if (g.nobs > 0 && !g.meta)  // only member 0's file carries ids/lat/lon/alt (:508-611)
      return ifail("cwbl_ingest_type_meta: GTS type %d has no metadata until member 0's file "
                   "is read", type_id);
    if (nvar) *nvar = g.nvar;
    if (nobs) *nobs = std::max(g.nobs, 0);
    if (ids) *ids = g.ids.data();
    if (lat) *lat = g.lat.data();
    if (lon) *lon = g.lon.data();
    if (alt) *alt = g.alt.data();
    return CWBL_OK;
  }
  if (family == 1 && type_id >= 1 && type_id <= CWBL_NUM_RADAR_TYPES) {
    const RadarType &r = h->radar[type_id];
    if (r.nobs > 0 && !r.meta)  // only member 0's file carries lat/lon/alt (:120-186)
      return ifail("cwbl_ingest_type_meta: radar type %d has no metadata until member 0's "
                   "file is read", type_id);
    if (nvar) *nvar = 1;
    if (nobs) *nobs = std::max(r.nobs, 0);
    if (ids) *ids = nullptr;
    if (lat) *lat = r.lat.data();
    if (lon) *lon = r.lon.data();
    if (alt) *alt = r.alt.data();
    return CWBL_OK;
  }
  return ifail("cwbl_ingest_type_meta: bad family %d / type %d", family, type_id);
}

// cwbl/dist.py pack_obs_set: [magic, ntypes, k] + (family, type_id, nvar, nobs) per type, then
// per type  GTS: xyz (n,3) | obs (n,nvar) | error (n,nvar) | hdxb (k,n,nvar) | qc (k,n,nvar)
//           radar: xyz (n,3) | obs (n,) | hdxb (k,n)
long long cwbl_ingest_wire_words(cwbl_ingest *h) {
  cwbl_obs_set s;
  if (!h || cwbl_ingest_obs_set(h, &s)) return -1;
  const long long k = h->k;
  long long w = 3 + 4LL * (s.n_gts + s.n_radar);
  for (int e = 0; e < s.n_gts; ++e) {
    const long long n = s.gts[e].nobs, nv = s.gts[e].nvar;
    w += 3 * n + 2 * n * nv + 2 * k * n * nv;
  }
  for (int e = 0; e < s.n_radar; ++e) w += 3LL * s.radar[e].nobs + s.radar[e].nobs * (1 + k);
  return w;
}

int cwbl_ingest_pack_wire(cwbl_ingest *h, float *buf, long long cap) {
  const long long need = cwbl_ingest_wire_words(h);
  if (need < 0) return CWBL_ERR_ARG;
  if (!buf || cap < need)
    return ifail("cwbl_ingest_pack_wire: buffer of %lld words, %lld needed", cap, need);
  cwbl_obs_set s;
  cwbl_ingest_obs_set(h, &s);
  const int32_t kMagic = 0x4C4B4631;  // "LKF1" (cwbl/dist.py WIRE_MAGIC)
  auto put_i = [](float *p, int32_t v) { std::memcpy(p, &v, 4); };
  put_i(buf, kMagic);
  put_i(buf + 1, s.n_gts + s.n_radar);
  put_i(buf + 2, h->k);
  float *p = buf + 3;
  for (int e = 0; e < s.n_gts; ++e) {
    put_i(p++, 0); put_i(p++, s.gts[e].type_id); put_i(p++, s.gts[e].nvar); put_i(p++, s.gts[e].nobs);
  }
  for (int e = 0; e < s.n_radar; ++e) {
    put_i(p++, 1); put_i(p++, s.radar[e].type_id); put_i(p++, 1); put_i(p++, s.radar[e].nobs);
  }
  auto copy = [&p](const void *src, size_t words) {
    std::memcpy(p, src, words * 4);
    p += words;
  };
  const size_t k = (size_t)h->k;
  for (int e = 0; e < s.n_gts; ++e) {
    const cwbl_gts_obs &g = s.gts[e];
    const size_t n = (size_t)g.nobs, nv = (size_t)g.nvar;
    copy(g.xyz, 3 * n); copy(g.obs, n * nv); copy(g.error, n * nv);
    copy(g.hdxb, k * n * nv); copy(g.qc, k * n * nv);
  }
  for (int e = 0; e < s.n_radar; ++e) {
    const cwbl_radar_obs &r = s.radar[e];
    const size_t n = (size_t)r.nobs;
    copy(r.xyz, 3 * n); copy(r.obs, n); copy(r.hdxb, k * n);
  }
  return CWBL_OK;
}

}  // extern "C"
