#!/bin/bash
# r04z2: bounce-phase priority variants: prio3 (items 1, sky 0, bounce 2), prio5 (items 1, sky 0, bounce 3),
# prio6 (items 0, bounce 1) against the final r04 build (ab_base2).
set -o pipefail
OUT=gpurun_out/r04z2; mkdir -p $OUT
B=epq_raytracer_amd/build
L="$B/ab_base2/libhip_raytrace.so $B/ab_prio3/libhip_raytrace.so $B/ab_prio5/libhip_raytrace.so $B/ab_prio6/libhip_raytrace.so"
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 4 $L > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 4 $L -- --scene cave --node-r 2 > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
