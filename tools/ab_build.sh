#!/bin/bash
# A/B builds of libhip_raytrace.so with extra compile definitions (device and host code), for HRT_LIB=... experiments:
#   bash tools/ab_build.sh <name> -DHRT_WQ_DEEP=0u ...   -> epq_raytracer_amd/build/ab_<name>/libhip_raytrace.so
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/epq_raytracer_amd/build/ab_$NAME
mkdir -p $OUT/obj
make -s -C $ROOT/epq_raytracer_amd/csrc OUT=$OUT OBJDIR=$OUT/obj \
  HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wall -Wno-bitwise-instead-of-logical -mllvm -amdgpu-schedule-relaxed-occupancy=1 -I$ROOT/include -I$ROOT/epq_raytracer_amd/csrc $*" \
  CXXFLAGS="-O2 -std=c++17 -fPIC -pthread -ffp-contract=off -fno-fast-math -Wall -Wextra -I$ROOT/include -I$ROOT/epq_raytracer_amd/csrc $*"
echo $OUT/libhip_raytrace.so
