#!/bin/bash
# r06j: per-item timelines (ab_timeline, -DHRT_TIMELINE=1) of the whole frame and ranks 3 and 6 of 8 at bench.py's
# shape on this round's kernel (band records, pool, tile lists).
set -o pipefail
OUT=gpurun_out/r06j; mkdir -p $OUT
export HRT_LIB=epq_raytracer_amd/build/ab_timeline/libhip_raytrace.so
timeout -k 10 120 python3 tools/timeline.py --raw $OUT/whole.npy --json $OUT/whole.json > $OUT/tl_whole.log 2>&1 || { echo "whole failed"; tail -5 $OUT/tl_whole.log; exit 1; }
for p in 3 6; do
timeout -k 10 120 python3 tools/timeline.py --partition 8,$p,8 --raw $OUT/rank$p.npy --json $OUT/rank$p.json > $OUT/tl_rank$p.log 2>&1 || { echo "rank$p failed"; tail -5 $OUT/tl_rank$p.log; exit 1; }
done
tail -3 $OUT/tl_*.log
