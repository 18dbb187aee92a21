#!/bin/bash
# r06p: r06o's candidates again, more rounds (island 4, cave 2): base, beta066, beta066p3, psub3.
set -o pipefail
OUT=gpurun_out/r06p; mkdir -p $OUT
for scene in island cave; do
R=4; [ $scene == cave ] && R=2
for r in $(seq 1 $R); do
for v in base beta066 beta066p3 psub3; do
  L=epq_raytracer_amd/build/ab_$v/libhip_raytrace.so; [ $v == base ] && L=epq_raytracer_amd/lib/libhip_raytrace.so
  HRT_LIB=$L timeout -k 10 200 python3 tools/rank_shape.py --scene $scene --rounds 1 --parts 3 6 > $OUT/${scene}_${v}_$r.jsonl 2>&1 || { echo "$v failed"; tail -3 $OUT/${scene}_${v}_$r.jsonl; exit 1; }
  echo "== $scene $v $r $(grep -v summary $OUT/${scene}_${v}_$r.jsonl | python3 -c 'import sys,json; print([json.loads(l)["kernel_ms"] for l in sys.stdin])')"
done; done; done
