#!/bin/bash
# Round-6 A/B helper: interleaved tools/ab.sh rounds of the production library against A/B builds, on
# island and cave at bench.py's launch shape (20-frame launches).  Usage (via gpurun):
#   bash tools/r06_ab.sh <tag> <rounds> <ab name> ...      (ab name: epq_raytracer_amd/build/ab_<name>)
set -o pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
LIBS=(epq_raytracer_amd/lib/libhip_raytrace.so)
for n in "$@"; do LIBS+=(epq_raytracer_amd/build/ab_$n/libhip_raytrace.so); done
for scene in ${AB_SCENES:-island cave}; do
  AB_BATCH=${AB_BATCH:-20} timeout -k 10 900 bash tools/ab.sh $R "${LIBS[@]}" -- --scene $scene > $OUT/ab_$scene.jsonl 2>&1 || { echo "ab $scene failed"; tail -5 $OUT/ab_$scene.jsonl; exit 1; }
  python3 tools/ab_summary.py $OUT/ab_$scene.jsonl 2>/dev/null || tail -${#LIBS[@]} $OUT/ab_$scene.jsonl
done
