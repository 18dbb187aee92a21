#!/bin/bash
# r03m: two-stage band pipeline (pipe2) and 512^2 direction cells (r512) against the current build (cur4).
set -o pipefail
OUT=gpurun_out/r03m; mkdir -p $OUT
L=epq_raytracer_amd/build
LIBS="$L/ab_cur4/libhip_raytrace.so $L/ab_pipe2/libhip_raytrace.so $L/ab_r512/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 2 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl $OUT/ab_cave.jsonl
