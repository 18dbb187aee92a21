#!/bin/bash
# r04b: GPU suite + smoke, then A/B of frame runs, the handoff fences, the list-loop pairs, the sky
# loop, and the sky / non-sky split timing (timing-only builds, tools/exp/r04_sky_split_timing.patch).
set -o pipefail
OUT=gpurun_out/r04b; mkdir -p $OUT
bash tools/r04.sh r04b || exit 1
B=epq_raytracer_amd/build
L=epq_raytracer_amd/lib/libhip_raytrace.so
timeout -k 10 900 bash tools/ab.sh 2 $L $B/ab_norun/libhip_raytrace.so $B/ab_nofence/libhip_raytrace.so $B/ab_pairs/libhip_raytrace.so $B/ab_nosky/libhip_raytrace.so $B/ab_nonsky/libhip_raytrace.so $B/ab_skyonly/libhip_raytrace.so > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
timeout -k 10 600 bash tools/ab.sh 2 $L $B/ab_norun/libhip_raytrace.so $B/ab_nofence/libhip_raytrace.so $B/ab_pairs/libhip_raytrace.so -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
