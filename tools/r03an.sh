#!/bin/bash
# r03an: per-member R of trace_bundle_wq_nr bounded as (sum + max) / 2 of the farthest-corner offsets (no
# square root) vs the committed build: ms per frame on cave, traversal counters, parity suite.
set -o pipefail
OUT=gpurun_out/r03an; mkdir -p $OUT
L=epq_raytracer_amd/build
LIBS="epq_raytracer_amd/lib/libhip_raytrace.so $L/ab_nrl1/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 3 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
for B in $LIBS; do
  HRT_LIB=$B timeout -k 10 300 python3 tools/kbench.py --variants 0 --diag --scene cave --rounds 1 --no-ref > $OUT/diag.jsonl 2>&1 || { echo "diag failed"; tail -5 $OUT/diag.jsonl; exit 1; }
  python3 -c "
import json
for l in open('$OUT/diag.jsonl'):
    if l.startswith('{') and 'bvh_band_per_lane' in l:
        d=json.loads(l); print('$B'.split('/')[-2], {k: round(d[k],3) for k in ('bvh_visits_per_lane','bvh_prims_per_lane','bvh_trips_per_iter')})
"
done
HRT_LIB=$L/ab_nrl1/libhip_raytrace.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || { echo "parity failed"; tail -30 $OUT/parity.log; exit 1; }
tail -n 2 $OUT/parity.log
