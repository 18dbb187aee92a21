#!/bin/bash
# r03ao: the step after a triangle step composed and its stack entries read while the triangle step
# waits on its records (pref; p0 = the same source without it) vs the committed build.
set -o pipefail
OUT=gpurun_out/r03ao; mkdir -p $OUT
L=epq_raytracer_amd/build
LIBS="epq_raytracer_amd/lib/libhip_raytrace.so $L/ab_p0/libhip_raytrace.so $L/ab_pref/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
timeout -k 10 600 bash tools/ab.sh 2 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
HRT_LIB=$L/ab_pref/libhip_raytrace.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || { echo "parity failed"; tail -30 $OUT/parity.log; exit 1; }
tail -n 2 $OUT/parity.log
