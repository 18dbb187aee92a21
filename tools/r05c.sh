#!/bin/bash
# r05c: per-item timelines of the 20-frame launch at bench.py's shape (ab_timeline = the in-tree kernel +
# HRT_TIMELINE records): the whole frame and one rank of 8; then the same with a grab tail of 8 items per
# wave (ab_tlgrab: frame runs of up to 4 frames while more than 8 items per wave remain).
set -o pipefail
OUT=gpurun_out/r05c; mkdir -p $OUT
B=epq_raytracer_amd/build
for L in timeline tlgrab; do
  export HRT_LIB=$B/ab_$L/libhip_raytrace.so
  timeout -k 10 120 python3 tools/timeline.py --json $OUT/tl_${L}_whole.json > $OUT/tl.log 2>&1 || { echo "whole failed"; tail -5 $OUT/tl.log; exit 1; }
  timeout -k 10 120 python3 tools/timeline.py --partition 8,6,8 --json $OUT/tl_${L}_rank6.json > $OUT/tl.log 2>&1 || { echo "rank6 failed"; tail -5 $OUT/tl.log; exit 1; }
  for f in whole rank6; do python3 -c "
import json; d=json.load(open('$OUT/tl_${L}_$f.json')); [d.pop(k) for k in ('last_items','busy_frac_curve')]; print('$L $f', json.dumps(d))"; done
done
