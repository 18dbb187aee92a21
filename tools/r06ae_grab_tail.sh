#!/bin/bash
# r06ae: HRT_GRAB_TAIL (items per resident wave taken singly at a launch's end; fewer = more frame runs) at 64
# (today) / 16 / 8 / 4 -- ranks of 8 and 4 at bench.py's shape, island and cave (whole frames in the same runs).
# builds: bash tools/ab_build.sh gtN -DHRT_GRAB_TAIL=Nu
set -o pipefail
OUT=gpurun_out/r06ae; mkdir -p $OUT
for g in 8 4; do
for s in island cave; do
for v in gt64 gt16 gt8 gt4; do
  HRT_LIB=epq_raytracer_amd/build/ab_$v/libhip_raytrace.so timeout -k 10 280 python3 tools/rank_shape.py --gpus $g --scene $s --rounds 1 > $OUT/${s}_g${g}_$v.jsonl 2>&1 || { echo "$s $g $v failed"; tail -3 $OUT/${s}_g${g}_$v.jsonl; exit 1; }
  echo "== $s g$g $v"; tail -1 $OUT/${s}_g${g}_$v.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['whole_kernel_ms'], [r['slowest_over_fair'] for r in d['runs']], [r['slowest_ms'] for r in d['runs']], {k: v[0] for k, v in d['part_kernel_ms'].items()})"
done
done
done
