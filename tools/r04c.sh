#!/bin/bash
# r04c: GPU suite + smoke on the product build (sky zero-component raygen, light-item frame runs), then
# A/B of the frame-run policy, the grab size, primary batching and the sky micro-variants.
set -o pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT
[ -z "$SKIP_SUITE" ] && { bash tools/r04.sh r04c || exit 1; }
B=epq_raytracer_amd/build
L=epq_raytracer_amd/lib/libhip_raytrace.so
AB_BATCH=20 timeout -k 10 1000 bash tools/ab.sh 3 $L $B/ab_norun/libhip_raytrace.so $B/ab_runheavy/libhip_raytrace.so $B/ab_g8/libhip_raytrace.so $B/ab_g6/libhip_raytrace.so $B/ab_g2/libhip_raytrace.so $B/ab_pb8/libhip_raytrace.so $B/ab_nosky0/libhip_raytrace.so > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 2 $L $B/ab_norun/libhip_raytrace.so $B/ab_runheavy/libhip_raytrace.so $B/ab_g8/libhip_raytrace.so $B/ab_pb8/libhip_raytrace.so -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
