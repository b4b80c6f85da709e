#!/bin/bash
# Build oracle/_ref/ref_harness from the reference sources where they lie.
#
# TEST INFRASTRUCTURE ONLY.  Compiles, unmodified apart from the reference Makefile's own
# preprocessing (`cpp -C -P -traditional ... -DREAL64`, Makefile:4,9,66-67):
#   module_param.f90, module_config.f90, module_eigen.f90,
#   module_localization.f90 (build_tree, get_lz, destroy_tree, Gaspari_Cohn_1999),
#   module_kdtree2.f90 (one array section of kdtree2_create made explicit: Q7 below)
# against two type-only modules with the reference's module names, gts_omboma and
# simulated_radar: the reference's own gts_structure / alt_* / radar_structure type
# definitions cut out of module_gts_omboma.f90:13-22,36-44 and module_radar.f90:13-16, plus
# the container types wrfda_gts / cwb_radar without their type-bound procedures (read_data,
# write_data, distribute: their targets need MPI).  And the source text of
#   letkf_yoyb         (module_letkf_core.f90:300-595)
#   letkf_solve        (module_letkf_core.f90:598-700)
#   letkf_tune_q       (module_letkf_core.f90:702-733)
#   read_gts_omboma, read_alt_info, get_alt (module_gts_omboma.f90:48-506,704-1049)
#   read_radar         (module_radar.f90:30-118)
# cut out at build time into wrapper modules (their home modules cannot be compiled here:
# module_letkf_core `use`s grid / mpi_util, and module_gts_omboma / module_radar `use`
# mpi_util; that chain needs the NetCDF-Fortran library and an MPI Fortran module, neither
# of which exists for amdflang in this image — see DESIGN.md "Oracle").  Intermediate
# sources live in a temp dir that is deleted; only the executable is written to oracle/_ref/.
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

for f in module_param module_config module_eigen module_localization; do
  $CPP "$REF/$f.f90" > "$TMP/$f.F90"
done
# Q7: with dim=2, kdtree2_create assigns the_data(:,ind(i)) (3 rows, as
# build_tree passes them, module_localization.f90:151-160) to rearranged_data(:,i) (2 rows,
# module_kdtree2.f90:670-675).  Fujitsu's compiler copies silently (rows 1..2 land where the
# search reads them, the third one float past the column); flang's runtime aborts on the
# element-count mismatch.  The one statement's source section becomes the_data(1:dimen, ...),
# the rows the reference keeps; for dim=3 it is the same section.  Nothing else is changed.
$CPP "$REF/module_kdtree2.f90" \
  | sed 's/^\( *mr%rearranged_data(:,i) = mr%the_data(\):, &$/\11:mr%dimen, \&/' \
  > "$TMP/module_kdtree2.F90"
[ "$(grep -c 'mr%the_data(1:mr%dimen, &' "$TMP/module_kdtree2.F90")" = 1 ] || \
  { echo "build_ref: Q7 substitution in module_kdtree2 not applied exactly once"; exit 1; }
# type-only modules under the reference's module names (module_localization `use`s them)
{
  echo "module gts_omboma"
  echo "    use param"
  echo "    implicit none"
  awk '/^    type, extends\(obs_structure\) :: gts_structure/,/^    end type gts_structure/' "$REF/module_gts_omboma.f90"
  echo "    type wrfda_gts"
  echo "        type(gts_structure), dimension(:), allocatable :: platform"
  echo "    end type wrfda_gts"
  awk '/^    type alt_info/,/^    end type alt_structure/' "$REF/module_gts_omboma.f90"
  echo "end module gts_omboma"
} > "$TMP/gts_omboma_types.f90"
{
  echo "module simulated_radar"
  echo "    use param"
  echo "    implicit none"
  awk '/^    type, extends\(obs_structure\) +:: radar_structure/,/^    end type radar_structure/' "$REF/module_radar.f90"
  echo "    type cwb_radar"
  echo "        type(radar_structure), dimension(:), allocatable :: radarobs"
  echo "    end type cwb_radar"
  echo "end module simulated_radar"
} > "$TMP/radar_types.f90"
for pat in "end type gts_structure" "end type alt_structure"; do
  grep -q "$pat" "$TMP/gts_omboma_types.f90" || { echo "build_ref: extraction of '$pat' failed"; exit 1; }
done
grep -q "end type radar_structure" "$TMP/radar_types.f90" || { echo "build_ref: radar_structure"; exit 1; }
$CPP "$TMP/gts_omboma_types.f90" > "$TMP/gts_omboma_types.F90"
$CPP "$TMP/radar_types.f90" > "$TMP/radar_types.F90"
{
  echo "module ref_extract"
  echo "    use param"
  echo "    use config"
  echo "    use eigen"
  echo "    use localization,    only : lz_structure, Gaspari_Cohn_1999"
  echo "    use gts_omboma,      only : wrfda_gts"
  echo "    use simulated_radar, only : cwb_radar"
  echo "    implicit none"
  echo "contains"
  awk '/^    subroutine letkf_yoyb\(/,/end subroutine letkf_yoyb/' "$REF/module_letkf_core.f90"
  awk '/^    function letkf_solve\(/,/end function letkf_solve/' "$REF/module_letkf_core.f90"
  # letkf_tune_q's loop bounds read the MPI decomposition (cpu(myid)%loc_nx/loc_ny, from
  # module_mpi_util, which cannot be compiled here).  The harness passes q allocated as
  # (loc_nx, loc_ny, nz, k), as letkf_driver does for the mass-grid Q species (:85), so
  # the bounds are replaced by size(q,1) / size(q,2); the body is otherwise unchanged.
  awk '/^    subroutine letkf_tune_q\(/,/end subroutine letkf_tune_q/' "$REF/module_letkf_core.f90" \
    | sed -e 's/cpu(myid) *% *loc_ny/size(q, 2)/' -e 's/cpu(myid) *% *loc_nx/size(q, 1)/'
  echo "end module ref_extract"
} > "$TMP/ref_extract.f90"
grep -q "end subroutine letkf_yoyb" "$TMP/ref_extract.f90"
grep -q "end function letkf_solve" "$TMP/ref_extract.f90"
grep -q "end subroutine letkf_tune_q" "$TMP/ref_extract.f90"
if grep -q "cpu(myid)" "$TMP/ref_extract.f90"; then echo "build_ref: tune_q bounds not replaced"; exit 1; fi
$CPP "$TMP/ref_extract.f90" > "$TMP/ref_extract.F90"
$CPP -D'cotan(x)=(1./tan(x))' "$REF/module_projection.f90" > "$TMP/module_projection.F90"
# the obs readers, on the type-only modules above
{
  echo "module ref_ingest"
  echo "    use projection,      only : proj_type"
  echo "    use config,          only : nmember"
  echo "    use param"
  echo "    use gts_omboma"
  echo "    use simulated_radar"
  echo "    implicit none"
  echo "    integer :: myid = 0   ! module_mpi_util's rank (read_radar's error messages)"
  echo "contains"
  awk '/^    subroutine read_gts_omboma\(/,/^    end subroutine read_gts_omboma/' "$REF/module_gts_omboma.f90"
  awk '/^    subroutine read_alt_info\(/,/^    end subroutine read_alt_info/' "$REF/module_gts_omboma.f90"
  awk '/^    real function get_alt\(/,/^    end function get_alt/' "$REF/module_gts_omboma.f90"
  awk '/^    subroutine read_radar\(/,/^    end subroutine read_radar/' "$REF/module_radar.f90"
  echo "end module ref_ingest"
} > "$TMP/ref_ingest.f90"
for pat in "end subroutine read_gts_omboma" "end subroutine read_alt_info" "end function get_alt" \
           "end subroutine read_radar"; do
  grep -q "$pat" "$TMP/ref_ingest.f90" || { echo "build_ref: extraction of '$pat' failed"; exit 1; }
done
$CPP "$TMP/ref_ingest.f90" > "$TMP/ref_ingest.F90"

cd "$TMP"
FFLAGS="-O2"
OBJS=""
for f in module_param module_config module_eigen module_kdtree2 gts_omboma_types radar_types \
         module_localization ref_extract module_projection ref_ingest; do
  $FC $FFLAGS -c "$f.F90"
  OBJS="$OBJS $f.o"
done
$FC $FFLAGS -I"$HERE" -c "$HERE/ref_harness.f90"
$FC $FFLAGS -o "$OUT/ref_harness" $OBJS ref_harness.o -L"$MKLDIR" -lmkl_rt -Wl,-rpath,"$MKLDIR"
echo "build_ref: built $OUT/ref_harness"
