#!/bin/bash
# r04ad2: the singly-grabbed tail at 8 / 16 / 24 / 32 items per resident wave (default 64) against the
# final build (ab_head).
set -o pipefail
OUT=gpurun_out/r04ad2; mkdir -p $OUT
B=epq_raytracer_amd/build
L="$B/ab_head/libhip_raytrace.so $B/ab_tail8/libhip_raytrace.so $B/ab_tail16/libhip_raytrace.so $B/ab_tail24/libhip_raytrace.so $B/ab_tail32/libhip_raytrace.so"
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $L > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $L -- --scene cave --node-r 2 > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
