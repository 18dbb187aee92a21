#!/bin/bash
# r04ad: the persistent loop's grab size (HRT_GRAB 2 / 8, default 4) and singly-grabbed tail
# (HRT_GRAB_TAIL 32 / 128 items per resident wave, default 64) against the final build (ab_head).
set -o pipefail
OUT=gpurun_out/r04ad; mkdir -p $OUT
B=epq_raytracer_amd/build
L="$B/ab_head/libhip_raytrace.so $B/ab_tail32/libhip_raytrace.so $B/ab_tail128/libhip_raytrace.so $B/ab_grab8/libhip_raytrace.so $B/ab_grab2/libhip_raytrace.so"
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $L > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $L -- --scene cave --node-r 2 > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
