#!/bin/bash
# r04z: wave issue priority -- light items' waves at 1 or 2 with the sky loop's pure-ALU waves at 0
# (HRT_ITEM_PRIO, HRT_SKY_PRIO0; heavy items stay at 3), and a light wave raised (prio3: 1 -> 2) or lowered
# (prio4: 2 -> 1) during its bounce traversal (HRT_BOUNCE_PRIO), against the final r04 build (ab_base2).
set -o pipefail
OUT=gpurun_out/r04z; mkdir -p $OUT
B=epq_raytracer_amd/build
L="$B/ab_base2/libhip_raytrace.so $B/ab_prio1/libhip_raytrace.so $B/ab_prio2/libhip_raytrace.so $B/ab_prio3/libhip_raytrace.so $B/ab_prio4/libhip_raytrace.so"
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 4 $L > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 4 $L -- --scene cave --node-r 2 > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
