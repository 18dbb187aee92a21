#!/bin/bash
# Repeated bench.py runs of one build on one box (the spread the driver's single run sits in):
#   bash tools/bench_repeat.sh <tag> [island runs] [cave runs]
set -o pipefail
TAG=${1:?usage: bench_repeat.sh <tag> [n_island] [n_cave]}; NI=${2:-5}; NC=${3:-3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $NI); do
  timeout -k 10 300 python3 bench.py --cpu-seconds 0 > $OUT/b.json 2> $OUT/b.err || { echo "bench failed"; tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); print('island', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['per_frame_dispatch_ms'])" | tee -a $OUT/repeat.txt
done
for i in $(seq 1 $NC); do
  timeout -k 10 300 python3 bench.py --scene cave --cpu-seconds 0 --realtime-frames 0 > $OUT/b.json 2> $OUT/b.err || { echo "bench cave failed"; tail -5 $OUT/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); print('cave', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" | tee -a $OUT/repeat.txt
done
