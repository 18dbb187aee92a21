#!/bin/bash
# r04ag: bounce-phase issue priority 0 / 1 (default) / 2 through bench.py's own shape, alternating builds.
set -o pipefail
OUT=gpurun_out/r04ag; mkdir -p $OUT
B=epq_raytracer_amd/build
for r in 1 2 3; do
  for L in bp0 bp1 bp2; do
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 300 python3 bench.py --cpu-seconds 0 --realtime-frames 0 > $OUT/b.json 2> $OUT/b.err || { echo "bench $L failed"; tail -5 $OUT/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$r $L island', d['ms_per_step'], d['roofline']['kernel_ms'])"
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 300 python3 bench.py --scene cave --cpu-seconds 0 --realtime-frames 0 > $OUT/b.json 2> $OUT/b.err || { echo "bench cave $L failed"; tail -5 $OUT/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$r $L cave', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
