#!/bin/bash
# r04i: sky-loop unroll (1 / 2 / 3 / 4 samples per trip) and the grab tail threshold (32 / 64 / 128 items
# per resident wave taken singly at the end); sky parity subset first for the unroll variants.
set -o pipefail
OUT=gpurun_out/r04i; mkdir -p $OUT
B=epq_raytracer_amd/build
L=epq_raytracer_amd/lib/libhip_raytrace.so
for v in u1 u3; do
HRT_LIB=$B/ab_$v/libhip_raytrace.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "sky" -q -x --timeout 200 --timeout-method thread > $OUT/parity_$v.log 2>&1 || { echo "parity $v failed"; tail -30 $OUT/parity_$v.log; exit 1; }
tail -1 $OUT/parity_$v.log
done
AB_BATCH=20 timeout -k 10 900 bash tools/ab.sh 3 $L $B/ab_u1/libhip_raytrace.so $B/ab_u3/libhip_raytrace.so $B/ab_u4/libhip_raytrace.so $B/ab_gt32/libhip_raytrace.so $B/ab_gt128/libhip_raytrace.so > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 2 $L $B/ab_u4/libhip_raytrace.so $B/ab_gt32/libhip_raytrace.so $B/ab_gt128/libhip_raytrace.so -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
