#!/bin/bash
# r03f: the GPU suite on the current library (per-triangle margins, margin-aware SAH, per-scene band
# width, kargs), then band-width / node-radius A/Bs on cave and island.
set -o pipefail
OUT=gpurun_out/r03f; mkdir -p $OUT
L=epq_raytracer_amd/build
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
LIBS="$L/ab_cur/libhip_raytrace.so $L/ab_tw45/libhip_raytrace.so $L/ab_tw9/libhip_raytrace.so"
timeout -k 10 600 bash tools/ab.sh 2 $LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
for nr in 0 1 2; do
  timeout -k 10 120 python3 tools/frames.py --scene cave --batch 64 --frames 2 --node-r $nr 2>&1 | tail -1
  timeout -k 10 120 python3 tools/frames.py --batch 64 --frames 3 --node-r $nr 2>&1 | tail -1
done > $OUT/node_r.jsonl || { echo "node_r sweep failed"; exit 1; }
cat $OUT/node_r.jsonl
