#!/bin/bash
# r03ad: packed FP32 (v_pk_*) in the node step's member test (pk: with the packed sincos; pkn: without;
# sc: packed sincos alone) against the current build; parity suite on the candidate.
set -o pipefail
OUT=gpurun_out/r03ad; mkdir -p $OUT
L=epq_raytracer_amd/build
NAMES=${NAMES:-"cur pk pkn sc"}
LIBS=""; for B in $NAMES; do LIBS="$LIBS $L/ab_$B/libhip_raytrace.so"; done
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
timeout -k 10 600 bash tools/ab.sh 2 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
HRT_LIB=$L/ab_${CAND:-pk}/libhip_raytrace.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || { echo "parity failed"; tail -30 $OUT/parity.log; exit 1; }
tail -n 2 $OUT/parity.log
