#!/bin/bash
# r06n: BUNDLE_WQ planned from work counts (product) against shader clocks (ab_clockcost): ranks 3 and 6 of 8 and
# the whole frame at bench.py's shape, island and cave, two rounds each.
set -o pipefail
OUT=gpurun_out/r06n; mkdir -p $OUT
for scene in island cave; do
for r in 1 2; do
for v in work clockcost; do
  L=epq_raytracer_amd/build/ab_$v/libhip_raytrace.so; [ $v == work ] && L=epq_raytracer_amd/lib/libhip_raytrace.so
  HRT_LIB=$L timeout -k 10 200 python3 tools/rank_shape.py --scene $scene --rounds 1 --parts 3 6 > $OUT/${scene}_${v}_$r.jsonl 2>&1 || { echo "$v failed"; tail -3 $OUT/${scene}_${v}_$r.jsonl; exit 1; }
  echo "== $scene $v $r"; grep -v summary $OUT/${scene}_${v}_$r.jsonl | cut -c1-70
done; done; done
