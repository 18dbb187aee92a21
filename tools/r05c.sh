#!/bin/bash
# r05c: per-item timelines of the 20-frame launch at bench.py's shape (ab_timeline = the in-tree kernel +
# HRT_TIMELINE records): the whole frame, one rank of 8, and one rank of 8 with 64 frames.
set -o pipefail
OUT=gpurun_out/r05c; mkdir -p $OUT
export HRT_LIB=epq_raytracer_amd/build/ab_timeline/libhip_raytrace.so
timeout -k 10 120 python3 tools/timeline.py --json $OUT/tl_whole.json > $OUT/tl_whole.log 2>&1 || { echo "whole failed"; tail -5 $OUT/tl_whole.log; exit 1; }
timeout -k 10 120 python3 tools/timeline.py --partition 8,6,8 --json $OUT/tl_rank6.json > $OUT/tl_rank6.log 2>&1 || { echo "rank6 failed"; tail -5 $OUT/tl_rank6.log; exit 1; }
timeout -k 10 120 python3 tools/timeline.py --partition 8,6,8 --steps 64 --json $OUT/tl_rank6_64.json > $OUT/tl_rank6_64.log 2>&1 || { echo "rank6 64 failed"; tail -5 $OUT/tl_rank6_64.log; exit 1; }
timeout -k 10 120 python3 tools/timeline.py --scene cave --json $OUT/tl_cave.json > $OUT/tl_cave.log 2>&1 || { echo "cave failed"; tail -5 $OUT/tl_cave.log; exit 1; }
for f in whole rank6 rank6_64 cave; do python3 -c "
import json; d=json.load(open('$OUT/tl_$f.json')); [d.pop(k) for k in ('last_items',)]; print('$f', json.dumps(d))"; done
