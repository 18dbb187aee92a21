#!/bin/bash
# r04g: marginal phase costs (timing-only builds running one phase a second time on opaque copies,
# tools/exp/r04_phase_twice_timing.patch): bounce traversal, primary list, shading.
set -o pipefail
OUT=gpurun_out/r04g; mkdir -p $OUT
B=epq_raytracer_amd/build
L=epq_raytracer_amd/lib/libhip_raytrace.so
AB_BATCH=20 timeout -k 10 900 bash tools/ab.sh 2 $L $B/ab_bx2/libhip_raytrace.so $B/ab_px2/libhip_raytrace.so $B/ab_sx2/libhip_raytrace.so > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 2 $L $B/ab_bx2/libhip_raytrace.so $B/ab_px2/libhip_raytrace.so $B/ab_sx2/libhip_raytrace.so -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
