#!/bin/bash
# r04j: position-bias check of r04i (a copy of the product library first and last in each round).
set -o pipefail
OUT=gpurun_out/r04j; mkdir -p $OUT
B=epq_raytracer_amd/build
L=epq_raytracer_amd/lib/libhip_raytrace.so
AB_BATCH=20 timeout -k 10 900 bash tools/ab.sh 4 $B/ab_lib2/libhip_raytrace.so $B/ab_u1/libhip_raytrace.so $B/ab_gt32/libhip_raytrace.so $L > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
