#!/bin/bash
# r06af: the N = 4 and N = 8 bench paths rehearsed on one GPU (bench.py self-spawns the ranks, gloo all-gather):
# the row-tile partition, each rank's 16-frame launch and the gathered frames' check (gather_check) at the
# driver's N values. Every rank shares the one GPU, so the times say nothing about scaling.
set -o pipefail
OUT=gpurun_out/r06af; mkdir -p $OUT
for n in 4 8; do
timeout -k 10 400 python3 bench.py --gpus $n --dist-backend gloo --steps 16 --warmup 2 --cpu-seconds 0 --realtime-frames 0 > $OUT/bench_n${n}_gloo.json 2> $OUT/bench_n${n}_gloo.err || { echo "n$n failed"; tail -30 $OUT/bench_n${n}_gloo.err; exit 1; }
# (gloo's own C++ log lines share stdout with the JSON line: take the last line that is one)
python3 -c "import json; L = [l for l in open('$OUT/bench_n${n}_gloo.json') if l.startswith('{')]; d = json.loads(L[-1]); print($n, d['config']['parallelism'], d['gather_check'], d['ranks']['kernel_ms'], d['ranks']['segments'])"
done
