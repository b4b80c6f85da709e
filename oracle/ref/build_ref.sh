#!/bin/bash
# Build oracle/_ref/ref_harness from the reference sources where they lie.
#
# TEST INFRASTRUCTURE ONLY.  Compiles, unmodified apart from the reference Makefile's own
# preprocessing (`cpp -C -P -traditional ... -DREAL64`, Makefile:4,9,66-67):
#   module_param.f90, module_config.f90, module_eigen.f90, module_kdtree2.f90
# and the source text of
#   letkf_solve        (module_letkf_core.f90:598-700)
#   letkf_tune_q       (module_letkf_core.f90:702-733)
#   Gaspari_Cohn_1999  (module_localization.f90:333-364)
#   read_gts_omboma, read_alt_info, get_alt and the gts_structure / alt_* types
#                      (module_gts_omboma.f90:13-22,36-44,48-506,704-1049)
#   read_radar and radar_structure (module_radar.f90:13-16,30-118)
# cut out at build time into wrapper modules (their home modules cannot be compiled here:
# module_letkf_core/module_localization `use` grid/gts_omboma/radar, whose chain needs the
# NetCDF-Fortran library and an MPI Fortran module, neither of which exists for amdflang in
# this image — see DESIGN.md "Oracle").  Intermediate sources live in a temp dir that is
# deleted; only the executable is written to oracle/_ref/.
#
# module_projection.f90 compiles with one preprocessor definition, cotan(x) = 1./tan(x)
# (cotan is a Fujitsu extension flang rejects, module_projection.f90:32-34,45).
#
# LAPACK/BLAS: MKL (libmkl_rt from /opt/conda/lib), sequential, MKL_CBWR=COMPATIBLE at run
# time (the reference production build links Fujitsu SSL2, Makefile:11).
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=$(cd "$HERE/.." && pwd)/_ref
FC=${FC:-amdflang}
MKLDIR=${MKLDIR:-/opt/conda/lib}

if [ ! -d "$REF" ]; then echo "build_ref: $REF not present, skipping"; exit 0; fi
command -v "$FC" >/dev/null || { echo "build_ref: $FC not found"; exit 1; }
[ -e "$MKLDIR/libmkl_rt.so" ] || { echo "build_ref: MKL not found in $MKLDIR"; exit 1; }

mkdir -p "$OUT"
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
CPP="cpp -C -P -traditional -Wno-invalid-pp-token -ffreestanding -DREAL64"

for f in module_param module_config module_eigen module_kdtree2; do
  $CPP "$REF/$f.f90" > "$TMP/$f.F90"
done
{
  echo "module ref_extract"
  echo "    use param"
  echo "    use config"
  echo "    use eigen"
  echo "    implicit none"
  echo "contains"
  awk '/^    function letkf_solve\(/,/end function letkf_solve/' "$REF/module_letkf_core.f90"
  # letkf_tune_q's loop bounds read the MPI decomposition (cpu(myid)%loc_nx/loc_ny, from
  # module_mpi_util, which cannot be compiled here).  The harness passes q allocated as
  # (loc_nx, loc_ny, nz, k), as letkf_driver does for the mass-grid Q species (:85), so
  # the bounds are replaced by size(q,1) / size(q,2); the body is otherwise unchanged.
  awk '/^    subroutine letkf_tune_q\(/,/end subroutine letkf_tune_q/' "$REF/module_letkf_core.f90" \
    | sed -e 's/cpu(myid) *% *loc_ny/size(q, 2)/' -e 's/cpu(myid) *% *loc_nx/size(q, 1)/'
  awk '/pure function Gaspari_Cohn_1999\(/,/end function Gaspari_Cohn_1999/' "$REF/module_localization.f90"
  echo "end module ref_extract"
} > "$TMP/ref_extract.f90"
grep -q "end function letkf_solve" "$TMP/ref_extract.f90"
grep -q "end function Gaspari_Cohn_1999" "$TMP/ref_extract.f90"
grep -q "end subroutine letkf_tune_q" "$TMP/ref_extract.f90"
if grep -q "cpu(myid)" "$TMP/ref_extract.f90"; then echo "build_ref: tune_q bounds not replaced"; exit 1; fi
$CPP "$TMP/ref_extract.f90" > "$TMP/ref_extract.F90"
$CPP -D'cotan(x)=(1./tan(x))' "$REF/module_projection.f90" > "$TMP/module_projection.F90"
# the obs readers (the types their dummies use are restated without the type-bound
# procedures, whose targets — distribute / write_data — need MPI)
{
  echo "module ref_ingest"
  echo "    use projection, only : proj_type"
  echo "    use config,     only : nmember"
  echo "    use param"
  echo "    implicit none"
  echo "    integer :: myid = 0   ! module_mpi_util's rank (read_radar's error messages)"
  awk '/^    type, extends\(obs_structure\) :: gts_structure/,/^    end type gts_structure/' "$REF/module_gts_omboma.f90"
  echo "    type wrfda_gts"
  echo "        type(gts_structure), dimension(:), allocatable :: platform"
  echo "    end type wrfda_gts"
  awk '/^    type alt_info/,/^    end type alt_structure/' "$REF/module_gts_omboma.f90"
  awk '/^    type, extends\(obs_structure\) +:: radar_structure/,/^    end type radar_structure/' "$REF/module_radar.f90"
  echo "    type cwb_radar"
  echo "        type(radar_structure), dimension(:), allocatable :: radarobs"
  echo "    end type cwb_radar"
  echo "contains"
  awk '/^    subroutine read_gts_omboma\(/,/^    end subroutine read_gts_omboma/' "$REF/module_gts_omboma.f90"
  awk '/^    subroutine read_alt_info\(/,/^    end subroutine read_alt_info/' "$REF/module_gts_omboma.f90"
  awk '/^    real function get_alt\(/,/^    end function get_alt/' "$REF/module_gts_omboma.f90"
  awk '/^    subroutine read_radar\(/,/^    end subroutine read_radar/' "$REF/module_radar.f90"
  echo "end module ref_ingest"
} > "$TMP/ref_ingest.f90"
for pat in "end type gts_structure" "end type alt_structure" "end type radar_structure" \
           "end subroutine read_gts_omboma" "end subroutine read_alt_info" "end function get_alt" \
           "end subroutine read_radar"; do
  grep -q "$pat" "$TMP/ref_ingest.f90" || { echo "build_ref: extraction of '$pat' failed"; exit 1; }
done
$CPP "$TMP/ref_ingest.f90" > "$TMP/ref_ingest.F90"

cd "$TMP"
FFLAGS="-O2"
for f in module_param module_config module_eigen module_kdtree2 ref_extract module_projection \
         ref_ingest; do
  $FC $FFLAGS -c "$f.F90"
done
$FC $FFLAGS -I"$HERE" -c "$HERE/ref_harness.f90"
$FC $FFLAGS -o "$OUT/ref_harness" module_param.o module_config.o module_eigen.o \
  module_kdtree2.o ref_extract.o module_projection.o ref_ingest.o ref_harness.o \
  -L"$MKLDIR" -lmkl_rt -Wl,-rpath,"$MKLDIR"
echo "build_ref: built $OUT/ref_harness"
