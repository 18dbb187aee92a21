#!/bin/bash
# r03u: kept leaves pushed by one flat loop (flat), triangle pre-test rejections as one predicate
# (trisel), both; GPU parity suite against flat_trisel.
set -o pipefail
OUT=gpurun_out/r03u; mkdir -p $OUT
L=epq_raytracer_amd/build
LIBS="$L/ab_cur/libhip_raytrace.so $L/ab_flat/libhip_raytrace.so $L/ab_trisel/libhip_raytrace.so $L/ab_flat_trisel/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 2 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
HRT_LIB=$L/ab_flat_trisel/libhip_raytrace.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || { echo "parity failed"; tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
