#!/bin/bash
# r03c: A/B of the r03 kernel changes (kargs: phase constants read from the kernel arguments; lean: fewer
# node-step shuffles; nocone_nr: no back-face cone test in the per-node-radius kernel) on island and cave.
set -o pipefail
OUT=gpurun_out/r03c; mkdir -p $OUT
L=epq_raytracer_amd/build
LIBS="$L/ab_base/libhip_raytrace.so $L/ab_kargs2/libhip_raytrace.so $L/ab_lean/libhip_raytrace.so $L/ab_nocone_nr/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 3 $LIBS > $OUT/island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/island.jsonl; exit 1; }
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/island.jsonl $OUT/cave.jsonl
