#!/bin/bash
# r04af: the grab tail 64 vs 24 through bench.py itself (the driver's shape: 5 warm-up, 20 timed frames
# in one launch), alternating builds, and one rank of 8 (64-frame launches) with each.
set -o pipefail
OUT=gpurun_out/r04af; mkdir -p $OUT
B=epq_raytracer_amd/build
for r in 1 2 3; do
  for L in t64 t24; do
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 300 python3 bench.py --cpu-seconds 0 --realtime-frames 0 > $OUT/b.json 2> $OUT/b.err || { echo "bench $L failed"; tail -5 $OUT/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$r $L island', d['ms_per_step'], d['roofline']['kernel_ms'])"
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 300 python3 bench.py --scene cave --cpu-seconds 0 --realtime-frames 0 > $OUT/b.json 2> $OUT/b.err || { echo "bench cave $L failed"; tail -5 $OUT/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$r $L cave', d['ms_per_step'], d['roofline']['kernel_ms'])"
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 120 python3 tools/frames.py --batch 64 --frames 2 --partition 8,3,8 > $OUT/p.log 2>&1 || { echo "rank $L failed"; exit 1; }
    echo "$r $L rank3of8 $(tail -1 $OUT/p.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms"])')"
  done
done
