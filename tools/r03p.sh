#!/bin/bash
# r03p: raygen shortcuts one at a time (rg_zero: signed-zero jitter components; rg_unit: normalize_unit;
# rg_both; rg_none), time and instruction counts on island.
set -o pipefail
OUT=gpurun_out/r03p; mkdir -p $OUT
L=epq_raytracer_amd/build
LIBS="$L/ab_rg_none/libhip_raytrace.so $L/ab_rg_zero/libhip_raytrace.so $L/ab_rg_unit/libhip_raytrace.so $L/ab_rg_both/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 3 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
bash tools/pmc_ab.sh r03p/insts $LIBS || exit 1
