#!/bin/bash
# r06l: planner cost buckets per octave 2 (product) / 4 / 8 (HRT_PLAN_SUB A/B builds): ranks 3 and 6 of 8 and the
# whole frame at bench.py's shape (tools/rank_shape.py), island then cave.
set -o pipefail
OUT=gpurun_out/r06l; mkdir -p $OUT
for scene in island cave; do
for r in 1 2; do
for v in base psub2 psub3; do
  L=epq_raytracer_amd/build/ab_$v/libhip_raytrace.so; [ $v == base ] && L=epq_raytracer_amd/lib/libhip_raytrace.so
  HRT_LIB=$L timeout -k 10 200 python3 tools/rank_shape.py --scene $scene --rounds 1 --parts 3 6 > $OUT/${scene}_${v}_$r.jsonl 2>&1 || { echo "$v failed"; tail -3 $OUT/${scene}_${v}_$r.jsonl; exit 1; }
  echo "== $scene $v $r"; grep -v summary $OUT/${scene}_${v}_$r.jsonl | cut -c1-90
done; done; done
