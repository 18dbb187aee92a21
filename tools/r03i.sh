#!/bin/bash
# r03i: 2-byte grazing-band entries + per-prim normal table (band2) against the 8-byte entries (cur3),
# and band2 at 128^2 direction cells: time (island, cave), fetched bytes (FETCH_SIZE), then the GPU suite
# on the product library (band2).
set -o pipefail
OUT=gpurun_out/r03i; mkdir -p $OUT
L=epq_raytracer_amd/build
LIBS="$L/ab_cur3/libhip_raytrace.so $L/ab_band2/libhip_raytrace.so $L/ab_band2r128/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 2 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl $OUT/ab_cave.jsonl
PMC="FETCH_SIZE" bash tools/pmc_ab.sh r03i/fetch_island $LIBS || exit 1
PMC="FETCH_SIZE" FRAMES_ARGS="--scene cave" bash tools/pmc_ab.sh r03i/fetch_cave $LIBS || exit 1
bash tools/pmc_ab.sh r03i/insts_island $L/ab_cur3/libhip_raytrace.so $L/ab_band2/libhip_raytrace.so || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
