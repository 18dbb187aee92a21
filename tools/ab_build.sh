#!/bin/bash
# A/B builds of libhip_raytrace.so with extra compile definitions (device and host code), for HRT_LIB=... experiments:
#   bash tools/ab_build.sh <name> -DHRT_WQ_DEEP=0u ...   -> epq_raytracer_amd/build/ab_<name>/libhip_raytrace.so
# HIP_EXTRA=<flags>: device/HIP compile only (e.g. -fslp-vectorize).  EXP_PATCH=<file.patch>: build from a copy of the sources with that patch applied (EXP_PATCH=1:
# tools/exp/phase_experiments.patch) -- e.g. the
# timing-only phase experiments (-DHRT_EXP_TWICE=<phase>: a phase run twice on opaque copies of its inputs;
# -DHRT_EXP_ONE_NORMALIZE: wrong frames; -DHRT_IEEE_DIV: the compiler's division sequences), which the
# product sources do not carry.  The patch is against the sources of its commit.
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/epq_raytracer_amd/build/ab_$NAME
mkdir -p $OUT/obj
SRC=$ROOT/epq_raytracer_amd/csrc
if [ -n "$EXP_PATCH" ]; then
  TMP=$OUT/src; rm -rf $TMP; mkdir -p $TMP/epq_raytracer_amd
  cp -r $SRC $TMP/epq_raytracer_amd/csrc
  PATCH=$EXP_PATCH; [ "$PATCH" == "1" ] && PATCH=$ROOT/tools/exp/phase_experiments.patch
  (cd $TMP && patch -s -p1 < $PATCH)
  SRC=$TMP/epq_raytracer_amd/csrc
fi
make -s -C $SRC OUT=$OUT OBJDIR=$OUT/obj ROOT=$ROOT \
  HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wall -Wno-bitwise-instead-of-logical -mllvm -amdgpu-schedule-relaxed-occupancy=1 -I$ROOT/include -I$SRC $* $HIP_EXTRA" \
  CXXFLAGS="-O2 -std=c++17 -fPIC -pthread -ffp-contract=off -fno-fast-math -Wall -Wextra -I$ROOT/include -I$SRC $*"
echo $OUT/libhip_raytrace.so
