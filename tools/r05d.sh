#!/bin/bash
# r05d: raw per-item timelines (ab_timeline) of the whole frame and rank 6 of 8 at bench.py's shape, plus the
# warm-up launch's plan inputs are implied by the records' order.
set -o pipefail
OUT=gpurun_out/r05d; mkdir -p $OUT
export HRT_LIB=epq_raytracer_amd/build/ab_timeline/libhip_raytrace.so
timeout -k 10 120 python3 tools/timeline.py --raw $OUT/whole.npy --json $OUT/whole.json > $OUT/tl.log 2>&1 || { echo "whole failed"; tail -5 $OUT/tl.log; exit 1; }
timeout -k 10 120 python3 tools/timeline.py --partition 8,6,8 --raw $OUT/rank6.npy --json $OUT/rank6.json > $OUT/tl.log 2>&1 || { echo "rank6 failed"; tail -5 $OUT/tl.log; exit 1; }
timeout -k 10 120 python3 tools/timeline.py --partition 8,6,8 --warmup 25 --raw $OUT/rank6_w25.npy --json $OUT/rank6_w25.json > $OUT/tl.log 2>&1 || { echo "rank6 w25 failed"; tail -5 $OUT/tl.log; exit 1; }
ls -la $OUT
