#!/bin/bash
# r03k: two-stage band pipeline (band2p2) vs one-stage (band2p) vs 8-byte entries (cur3); the band scan's
# whole cost (noband: no band pairs, wrong frames, timing only).
set -o pipefail
OUT=gpurun_out/r03k; mkdir -p $OUT
L=epq_raytracer_amd/build
LIBS="$L/ab_cur3/libhip_raytrace.so $L/ab_band2p/libhip_raytrace.so $L/ab_band2p2/libhip_raytrace.so $L/ab_noband/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 2 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl $OUT/ab_cave.jsonl
