#!/bin/bash
# r03aa: plane-side filter of band entries (plane) vs current; parity suite on the candidate; diag on cave.
set -o pipefail
OUT=gpurun_out/r03aa; mkdir -p $OUT
L=epq_raytracer_amd/build
LIBS="$L/ab_cur/libhip_raytrace.so $L/ab_plane/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 2 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
for B in cur plane; do
  HRT_LIB=$L/ab_$B/libhip_raytrace.so timeout -k 10 300 python3 tools/kbench.py --variants 0 --diag --scene cave --rounds 1 --no-ref > $OUT/diag_cave_$B.jsonl 2>&1 || { echo "diag $B failed"; tail -5 $OUT/diag_cave_$B.jsonl; exit 1; }
  python3 -c "
import json
for l in open('$OUT/diag_cave_$B.jsonl'):
    if l.startswith('{') and 'bvh_band_per_lane' in l:
        d=json.loads(l); print('$B', {k: round(d[k],3) for k in ('bvh_visits_per_lane','bvh_prims_per_lane','bvh_band_per_lane','band_len_per_lane','bvh_trips_per_iter')})
"
done
HRT_LIB=$L/ab_plane/libhip_raytrace.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || { echo "parity failed"; tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
