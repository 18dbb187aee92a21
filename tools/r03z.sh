#!/bin/bash
# r03z: band cells 256 / 384 / 512 per face edge (tau 3e-3; 256 also at 2e-3): ms per frame and counter
# bytes (FETCH_SIZE, one 64-frame launch) on island and cave.
set -o pipefail
OUT=gpurun_out/r03z; mkdir -p $OUT
L=epq_raytracer_amd/build
LIBS="$L/ab_cur/libhip_raytrace.so $L/ab_c256t3/libhip_raytrace.so $L/ab_c256t2/libhip_raytrace.so $L/ab_c384t3/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 2 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
PMC="FETCH_SIZE" bash tools/pmc_ab.sh r03z/fetch_island $LIBS || exit 1
PMC="FETCH_SIZE" FRAMES_ARGS="--scene cave" bash tools/pmc_ab.sh r03z/fetch_cave $LIBS || exit 1
