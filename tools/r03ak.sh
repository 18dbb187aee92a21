#!/bin/bash
# r03ak: a node step's first member pair (early) or both pairs (early2) read before the node-only shuffles
# vs the current build (e0): ms per frame on cave and island, traversal counters, and
# the parity suite on the candidate.
set -o pipefail
OUT=gpurun_out/r03ak; mkdir -p $OUT
L=epq_raytracer_amd/build
NAMES=${NAMES:-"cur e0 early early2"}
LIBS="epq_raytracer_amd/lib/libhip_raytrace.so"; for B in $NAMES; do LIBS="$LIBS $L/ab_$B/libhip_raytrace.so"; done
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
timeout -k 10 600 bash tools/ab.sh 2 $LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
for S in cave island; do for B in $NAMES; do
  HRT_LIB=$L/ab_$B/libhip_raytrace.so timeout -k 10 300 python3 tools/kbench.py --variants 0 --diag --scene $S --rounds 1 --no-ref > $OUT/diag_${S}_$B.jsonl 2>&1 || { echo "diag $S $B failed"; tail -5 $OUT/diag_${S}_$B.jsonl; exit 1; }
  python3 -c "
import json
for l in open('$OUT/diag_${S}_$B.jsonl'):
    if l.startswith('{') and 'bvh_band_per_lane' in l:
        d=json.loads(l); print('$S $B', {k: round(d[k],3) for k in ('bvh_visits_per_lane','bvh_prims_per_lane','bvh_band_per_lane','bvh_trips_per_iter','bounce_cycle_share','primary_cycle_share','shade_cycle_share')})
"
done; done
HRT_LIB=$L/ab_${CAND:-early}/libhip_raytrace.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || { echo "parity failed"; tail -30 $OUT/parity.log; exit 1; }
tail -n 2 $OUT/parity.log
