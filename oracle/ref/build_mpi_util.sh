#!/bin/bash
# Build oracle/_ref/mpi_util_harness from the reference's module_mpi_util.f90 where it lies.
#
# TEST INFRASTRUCTURE ONLY.  Compiles, with the reference Makefile's own preprocessing
# (`cpp -C -P -traditional ... -DREAL64`, Makefile:4,9,66-67) and nothing else changed:
#   module_param.f90, module_config.f90, module_mpi_util.f90
# against MPICH (/opt/conda: mpif.h, libmpifort, libmpi) and MKL (sgemv, sequential).
# The one build shim is SURVEY.md §8(c) shim 1: the image's `mpi.mod` was written by gfortran
# and cannot be read by amdflang, so `use mpi` is served by a three-line module that
# `include`s MPICH's own mpif.h (the MPI-1 Fortran interface the module would export; every
# routine is MPICH's).  Intermediate files live in a temp dir that is deleted; only the
# executable is written to oracle/_ref/.  Run it with oracle/gen_mpi_util_goldens.py.
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=$(cd "$HERE/.." && pwd)/_ref
FC=${FC:-amdflang}
MPIDIR=${MPIDIR:-/opt/conda}
MKLDIR=${MKLDIR:-/opt/conda/lib}

if [ ! -d "$REF" ]; then echo "build_mpi_util: $REF not present, skipping"; exit 0; fi
command -v "$FC" >/dev/null || { echo "build_mpi_util: $FC not found"; exit 1; }
[ -e "$MPIDIR/include/mpif.h" ] || { echo "build_mpi_util: no mpif.h under $MPIDIR"; exit 1; }
[ -e "$MPIDIR/lib/libmpifort.so" ] || { echo "build_mpi_util: no libmpifort under $MPIDIR"; exit 1; }
[ -e "$MKLDIR/libmkl_rt.so" ] || { echo "build_mpi_util: MKL not found in $MKLDIR"; exit 1; }

mkdir -p "$OUT"
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
CPP="cpp -C -P -traditional -Wno-invalid-pp-token -ffreestanding -DREAL64"
for f in module_param module_config module_mpi_util; do
  $CPP "$REF/$f.f90" > "$TMP/$f.F90"
done
printf 'module mpi\n    include "mpif.h"\nend module mpi\n' > "$TMP/mpi_shim.f90"

cd "$TMP"
FFLAGS="-O2 -I$MPIDIR/include"
OBJS=""
for f in mpi_shim.f90 module_param.F90 module_config.F90 module_mpi_util.F90; do
  $FC $FFLAGS -c "$f"
  OBJS="$OBJS ${f%.*}.o"
done
$FC $FFLAGS -c "$HERE/mpi_util_harness.f90"
$FC $FFLAGS -o "$OUT/mpi_util_harness" $OBJS mpi_util_harness.o \
  -L"$MPIDIR/lib" -lmpifort -lmpi -L"$MKLDIR" -lmkl_rt \
  -Wl,-rpath,"$MPIDIR/lib" -Wl,-rpath,"$MKLDIR"
echo "build_mpi_util: built $OUT/mpi_util_harness"
