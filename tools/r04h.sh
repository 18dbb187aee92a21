#!/bin/bash
# r04h: a node step's first member pair read before the (atomic) slot read; parity subset first.
set -o pipefail
OUT=gpurun_out/r04h; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_boundary.py -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
B=epq_raytracer_amd/build
L=epq_raytracer_amd/lib/libhip_raytrace.so
AB_BATCH=20 timeout -k 10 900 bash tools/ab.sh 3 $L $B/ab_noearly/libhip_raytrace.so > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $L $B/ab_noearly/libhip_raytrace.so -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
