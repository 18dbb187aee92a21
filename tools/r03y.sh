#!/bin/bash
# r03y: the r03x defaults (band tau 3e-3, 512 cells) -- GPU suite, PMC passes, bench (island, cave) and
# kernel trace (tools/gpu_round.sh); A/B of the triangle pre-test as one predicate; bounce batch on cave.
set -o pipefail
OUT=gpurun_out/r03y; mkdir -p $OUT
L=epq_raytracer_amd/build
timeout -k 10 600 bash tools/ab.sh 2 $L/ab_cur/libhip_raytrace.so $L/ab_trisel/libhip_raytrace.so > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
timeout -k 10 600 bash tools/ab.sh 2 $L/ab_cur/libhip_raytrace.so $L/ab_trisel/libhip_raytrace.so -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
timeout -k 10 600 bash tools/knobs.sh 1 cave "" "--sec-batch 24" "--sec-batch 36" "--leaf 4" > $OUT/knobs_cave.jsonl 2>&1 || { echo "knobs failed"; exit 1; }
python3 tools/ab_summary.py $OUT/knobs_cave.jsonl
bash tools/gpu_round.sh r03y_main || exit 1
SKIP_TESTS=1 bash tools/gpu_round.sh r03y_cave --scene cave || exit 1
