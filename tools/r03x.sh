#!/bin/bash
# r03x: band width tau_g 1.5e-3 / 2e-3 (256 and 512 cells) against 4.5e-3 and 3e-3 with 512 cells
set -o pipefail
OUT=gpurun_out/r03x; mkdir -p $OUT
L=epq_raytracer_amd/build
LIBS="$L/ab_cur/libhip_raytrace.so $L/ab_t3d512/libhip_raytrace.so $L/ab_t2/libhip_raytrace.so $L/ab_t15/libhip_raytrace.so $L/ab_t2d512/libhip_raytrace.so $L/ab_t15d512/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 2 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
