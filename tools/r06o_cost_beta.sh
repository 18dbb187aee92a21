#!/bin/bash
# r06o: persistent-kernel item costs scaled to full contention ((16 / active waves)^beta, HRT_COST_BETA A/B
# builds; beta066p3 also with eighth-octave plan buckets): ranks 3 and 6 of 8 and the whole frame at bench.py's
# shape, island (2 rounds) and cave (1 round).
set -o pipefail
OUT=gpurun_out/r06o; mkdir -p $OUT
for scene in island cave; do
R=2; [ $scene == cave ] && R=1
for r in $(seq 1 $R); do
for v in base beta05 beta066 beta085 beta066p3; do
  L=epq_raytracer_amd/build/ab_$v/libhip_raytrace.so; [ $v == base ] && L=epq_raytracer_amd/lib/libhip_raytrace.so
  HRT_LIB=$L timeout -k 10 200 python3 tools/rank_shape.py --scene $scene --rounds 1 --parts 3 6 > $OUT/${scene}_${v}_$r.jsonl 2>&1 || { echo "$v failed"; tail -3 $OUT/${scene}_${v}_$r.jsonl; exit 1; }
  echo "== $scene $v $r $(grep -v summary $OUT/${scene}_${v}_$r.jsonl | python3 -c 'import sys,json; print([json.loads(l)["kernel_ms"] for l in sys.stdin])')"
done; done; done
