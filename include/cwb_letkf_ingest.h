/* cwb_letkf_ingest.h — host-side observation ingest and map projection of the LETKF core.
 *
 * the readers a Fortran or C++ host calls on the ranks that
 * own the member obs files, in place of the reference's
 *   read_gts_omboma + read_alt_info + get_alt   (module_gts_omboma.f90:48-506, 704-1049)
 *   read_radar                                  (module_radar.f90:30-118)
 *   proj_type%init / %lonlat_to_xy              (module_projection.f90:21-50)
 * They fill the cwbl_obs_set of cwb_letkf_core.h (host memory, the reference's Fortran
 * layouts) and the one-buffer wire format that replaces gts_distribute / radar_distribute
 * (module_gts_omboma.f90:508-611, module_radar.f90:120-186; cwbl/dist.py).  Host code only:
 * nothing here touches the GPU.
 *
 * Semantics follow the reference, with three deliberate differences:
 *   - the station-altitude lookup get_alt is a hash map, not a linear scan per report
 *     (module_gts_omboma.f90:1041-1048); the first station of an id still wins;
 *   - every malformed field, short file (Q5, module_radar.f90:91-104) and unknown report
 *     type with data is an error, where the reference ignores iostat or misreads on;
 *   - the member index may be given explicitly (the reference always takes it from the
 *     file name's last three characters, module_gts_omboma.f90:82-84).
 * Errors return nonzero with the message in cwbl_last_error(); the library never exits.
 */
#ifndef CWB_LETKF_INGEST_H
#define CWB_LETKF_INGEST_H

#include "cwb_letkf_core.h"

#ifdef __cplusplus
extern "C" {
#endif

/* projection_nml (module_config.f90:70-75); the defaults there are 120.0, 23.7644, 10.0, 40.0 */
typedef struct cwbl_projection {
  float sta_lon;   /* reference longitude of the Lambert conformal map (degrees) */
  float cen_lat;   /* latitude of the map origin (degrees) */
  float truelat1;  /* true latitudes (degrees) */
  float truelat2;
} cwbl_projection;

/* proj_type%init + %lonlat_to_xy for n points (module_projection.f90:21-50), in fp32 in the
 * reference's operation order: x = rh sin(dlon), y = rh0 - rh cos(dlon), metres. */
int cwbl_lonlat_to_xy(const cwbl_projection *proj, long long n, const float *lon,
                      const float *lat, float *x, float *y);

typedef struct cwbl_ingest cwbl_ingest; /* opaque: the obs set of one cycle on the host */

/* An empty obs set for `nmember` members projected with `proj`; NULL on a bad argument. */
cwbl_ingest *cwbl_ingest_create(int nmember, const cwbl_projection *proj);
void         cwbl_ingest_destroy(cwbl_ingest *h);

/* read_gts_omboma(filename = gts_file, obascii = obs_gts_file) of one member: the WRFDA
 * gts_omboma records ('(a20,i8)' headers, '(2i8)' report lines and
 * '(2i8,a5,2f9.2,f17.7,5(2f17.7,i8,2f17.7))' data lines) with hdxb = obs - omb, station
 * altitudes from the obs_gts file (read_alt_info: its INFO/EACH formats are read from the file
 * itself) and x, y by lonlat_to_xy.  member: 0-based (the reference's iproc), or -1 for the
 * file name's last three digits minus one.  Member 0's file (the root reader of
 * gts_distribute) provides every array but hdxb and qc; each member provides its own
 * hdxb(:,:,member) and qc(:,:,member). */
int cwbl_ingest_read_gts(cwbl_ingest *h, int member, const char *gts_file,
                         const char *obs_gts_file);

/* read_radar of one member: '(i10)' count, then '(5(f10.4,1x))' rows obs, hdxb, lon, lat, alt.
 * varname "MR" (dbz), "VR" (vr), "MD" (zdr) or "MK" (kdp), as module_radar.f90:70-79. */
int cwbl_ingest_read_radar(cwbl_ingest *h, int member, const char *file, const char *varname);

/* Views of the set read so far as a host-memory cwbl_obs_set, valid until the next read or
 * destroy: every type with data, GTS types then radar types by type id.  Fails if a type
 * lacks a member's hdxb. */
int cwbl_ingest_obs_set(cwbl_ingest *h, cwbl_obs_set *out);

/* Per-type metadata the obs set does not carry: station ids (5 characters per obs, not NUL
 * terminated) and lat, lon, alt (degrees, degrees, metres).  family 0 GTS, 1 radar (ids NULL).
 * Only member 0's file fills them (the root reader, module_gts_omboma.f90:508-611): a type
 * read from other members' files alone returns CWBL_ERR_ARG here. */
int cwbl_ingest_type_meta(cwbl_ingest *h, int family, int type_id, int *nvar, int *nobs,
                          const char **ids, const float **lat, const float **lon,
                          const float **alt);

/* The one-buffer wire format of the set (cwbl/dist.py pack_obs_set): words needed, and the
 * packed float32 buffer (integers as int32 bit patterns). */
long long cwbl_ingest_wire_words(cwbl_ingest *h);
int       cwbl_ingest_pack_wire(cwbl_ingest *h, float *buf, long long cap_words);

#ifdef __cplusplus
}
#endif

#endif /* CWB_LETKF_INGEST_H */
