#!/usr/bin/env bash
# oracle/build_ref.sh -- compile the REFERENCE's own sources, in place under /root/reference,
# into oracle/_ref/ (git-ignored; travels to the GPU box with the snapshot). Test infrastructure only.
#
#   _ref/photonmap_strict.hsaco  reference photonmap.cl for gfx950 with ROCm's OpenCL device
#                                libraries; IEEE div/sqrt (-cl-fp32-correctly-rounded-divide-sqrt),
#                                no FMA contraction -- the oracle's arithmetic contract.
#   _ref/photonmap_fast.hsaco    same source with the flags the reference itself passes to
#                                clBuildProgram (global_illumination_cl.c:196: -cl-fast-relaxed-math).
#   _ref/dump_geometry           reference parseLayout.c/image.c/png_helper.c/rectangle.c/... +
#                                oracle/dump_geometry.c; turns a layout PNG into a geometry fixture.
#   _ref/ao_ref                  reference photonmap.c/rectangle.c/vector3_cl.c/geoSphere.c + oracle/ao_ref_main.c:
#                                performAmbientOcclusionNative on a geometry fixture (AO fixtures).
#   _ref/photon_ref              reference photonmap.o/rectangle.o/vector3_cl.o + oracle/photon_ref_main.c:
#                                performPhotonMappingNative timed on a geometry fixture (bench CPU baseline).
#   _ref/rad_ref                 reference radiosityNative.o/rectangle.o/vector3_cl.o + oracle/rad_ref_main.c:
#                                performRadiosityNative on a geometry fixture (radiosity fixtures).
#   _ref/out_ref                 main.c:66-79 normalisation + the reference's saveAs()/read_png_file()
#                                (output-step fixtures: RGB8 tile bytes).
#   _ref/globalIllumination_fmgi reference main.c + its layout/IO objects linked against OUR
#                                libflatmatch_gi.so instead of global_illumination_cl.o (drop-in check).
#
# No reference file is copied into the repository; nothing here is needed at run time on the GPU box
# except the built artefacts themselves.
set -euo pipefail
REF=${FMGI_REFERENCE:-/root/reference}
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
REPO="$(dirname "$HERE")"
OUT="$HERE/_ref"
CLANG=${CLANG:-/opt/rocm/lib/llvm/bin/clang}
mkdir -p "$OUT/obj"

if [ ! -f "$REF/photonmap.cl" ]; then
    echo "build_ref: $REF not present; skipping reference builds" >&2
    exit 0
fi

CLFLAGS="-x cl -cl-std=CL1.2 -Xclang -finclude-default-header -target amdgcn-amd-amdhsa -mcpu=gfx950 -O3"
$CLANG $CLFLAGS -Wno-nan-infinity-disabled -cl-fp32-correctly-rounded-divide-sqrt -ffp-contract=off "$REF/photonmap.cl" -o "$OUT/photonmap_strict.hsaco"
# The reference's own flag (-cl-fast-relaxed-math) implies finite-math-only, under which ROCm's clang
# folds photonmap.cl:208 `dist_out == INFINITY` away: an escaping photon then dereferences hitObj == 0
# and the kernel faults (observed on MI355X, gpurun_out/s1/ref.log). It is built for inspection only and
# must not be launched; "relaxed" keeps every other fast-math relaxation and stays well defined.
$CLANG $CLFLAGS -Wno-nan-infinity-disabled -cl-fast-relaxed-math "$REF/photonmap.cl" -o "$OUT/photonmap_fast.hsaco"
$CLANG $CLFLAGS -Wno-nan-infinity-disabled -cl-unsafe-math-optimizations "$REF/photonmap.cl" -o "$OUT/photonmap_relaxed.hsaco"

# Host C objects of the reference (flags as in the reference Makefile:21,26 minus -flto/-g).
PNG_INC=${PNG_INC:-/opt/conda/include}
PNG_SO=${PNG_SO:-/usr/lib/x86_64-linux-gnu/libpng16.so.16}  # system libpng (same 1.6.37 ABI as the conda headers)
CFLAGS="-O2 -msse3 -std=c99 -DNDEBUG -DCL_TARGET_OPENCL_VERSION=120 -I$REF -I/opt/rocm/include -I$PNG_INC -w"
for f in parseLayout image png_helper rectangle geometry vector3_cl helpers photonmap geoSphere radiosityNative main; do
    gcc $CFLAGS -c "$REF/$f.c" -o "$OUT/obj/$f.o"
done
gcc $CFLAGS -c "$HERE/dump_geometry.c" -o "$OUT/obj/dump_geometry.o"
COMMON="$OUT/obj/parseLayout.o $OUT/obj/image.o $OUT/obj/png_helper.o $OUT/obj/rectangle.o $OUT/obj/geometry.o $OUT/obj/vector3_cl.o $OUT/obj/helpers.o"
gcc -o "$OUT/dump_geometry" "$OUT/obj/dump_geometry.o" $COMMON "$PNG_SO" -lm

# Ambient-occlusion reference: the reference's performAmbientOcclusionNative on a geometry fixture.
gcc $CFLAGS -c "$HERE/ao_ref_main.c" -o "$OUT/obj/ao_ref_main.o"
gcc -o "$OUT/ao_ref" "$OUT/obj/ao_ref_main.o" "$OUT/obj/photonmap.o" "$OUT/obj/geoSphere.o" $COMMON "$PNG_SO" -lm

# CPU photon-mapping reference (bench.py's cpu_baseline): the reference's performPhotonMappingNative, timed.
gcc $CFLAGS -c "$HERE/photon_ref_main.c" -o "$OUT/obj/photon_ref_main.o"
gcc -o "$OUT/photon_ref" "$OUT/obj/photon_ref_main.o" "$OUT/obj/photonmap.o" "$OUT/obj/geoSphere.o" $COMMON "$PNG_SO" -lm

# Radiosity reference: the reference's performRadiosityNative on a geometry fixture, seeded rand().
gcc $CFLAGS -c "$HERE/rad_ref_main.c" -o "$OUT/obj/rad_ref_main.o"
gcc -o "$OUT/rad_ref" "$OUT/obj/rad_ref_main.o" "$OUT/obj/radiosityNative.o" $COMMON "$PNG_SO" -lm

# Output-step reference: main.c:66-79 normalisation + the reference's saveAs() per wall, read back.
gcc $CFLAGS -c "$HERE/out_ref_main.c" -o "$OUT/obj/out_ref_main.o"
gcc -o "$OUT/out_ref" "$OUT/obj/out_ref_main.o" $COMMON "$PNG_SO" -lm

# Drop-in link check: the reference CLI against our C-ABI library (needs the product .so built).
LIB="$REPO/flatmatch-global-illumination_amd/libflatmatch_gi.so"
if [ -f "$LIB" ]; then
    g++ -o "$OUT/globalIllumination_fmgi" "$OUT/obj/main.o" $COMMON "$OUT/obj/photonmap.o" \
        "$OUT/obj/geoSphere.o" "$OUT/obj/radiosityNative.o" \
        -L"$(dirname "$LIB")" -Wl,-rpath,'$ORIGIN/../../flatmatch-global-illumination_amd' -lflatmatch_gi \
        "$PNG_SO" -lm
fi
echo "build_ref: OK -> $OUT"
