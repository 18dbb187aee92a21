#!/bin/bash
# r03n: camera lists kept across traces from one position; GPU suite, realtime loop, bench (island, cave).
set -o pipefail
OUT=gpurun_out/r03n; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_boundary.py -q -x -k camera_lists --timeout 120 --timeout-method thread > $OUT/cam_test.log 2>&1 || { echo "camera test failed"; tail -30 $OUT/cam_test.log; exit 1; }
tail -1 $OUT/cam_test.log
timeout -k 10 300 python3 tools/realtime.py --lanes 1 3 --busy-split 2 --defer 0 --rounds 2 --frames 32 > $OUT/realtime.jsonl 2>&1 || { echo "realtime failed"; tail -5 $OUT/realtime.jsonl; exit 1; }
cat $OUT/realtime.jsonl
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 300 python3 bench.py --scene cave > $OUT/bench_cave.json 2> $OUT/bench_cave.err || { echo "bench cave failed"; tail -20 $OUT/bench_cave.err; exit 1; }
python3 -c "
import json
for f in ('bench', 'bench_cave'):
    d = json.load(open('$OUT/%s.json' % f)); r = d['roofline']
    print(f, d['value'], d['unit'], 'ms/step', d['ms_per_step'], 'kernel_ms', r['kernel_ms'], 'rt', d['per_frame_dispatch_ms'], 'parity', d.get('parity_sample'))
"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
