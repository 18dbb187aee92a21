#!/bin/bash
# r03ap: compiler scheduler options on the committed sources -- f1 no unclustered high-RP reschedule,
# f2 no clustered low-occupancy reschedule, f3 schedule-metric bias 0, f4 no loop alignment -- vs lib.
set -o pipefail
OUT=gpurun_out/r03ap; mkdir -p $OUT
L=epq_raytracer_amd/build
LIBS="epq_raytracer_amd/lib/libhip_raytrace.so $L/ab_f1/libhip_raytrace.so $L/ab_f2/libhip_raytrace.so $L/ab_f3/libhip_raytrace.so $L/ab_f4/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
timeout -k 10 600 bash tools/ab.sh 2 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
