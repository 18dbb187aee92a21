#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench (N=1), rocprofv3 kernel-trace summary of the same bench,
# PMC passes (traffic + executed FLOPs).  Usage (repo root, via gpurun): bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r01}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
bash tools/pmc.sh $TAG/pmc 0 > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $OUT/pmc.log; exit 1; }
cp $OUT/pmc/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 600 python3 bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --cpu-seconds 0 --steps 20 "$@" > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \;
timeout -k 10 300 python3 tools/tile_profile.py > $OUT/tile_profile.json 2>&1 || { echo "tile profile failed"; tail -20 $OUT/tile_profile.json; exit 1; }
timeout -k 10 300 python3 tools/frames.py --frames 8 > $OUT/frames.json 2>&1 || { echo "frames failed"; tail -20 $OUT/frames.json; exit 1; }
for n in 2 4 8; do timeout -k 10 300 python3 tools/frames.py --frames 6 --partition 8,0,$n >> $OUT/frames.json 2>&1 || { echo "frames failed"; exit 1; }; done
cat $OUT/frames.json
for v in 9 7; do timeout -k 10 300 python3 tools/frames.py --scene cave --variant $v --frames 5 >> $OUT/frames.json 2>&1 || { echo "cave frames failed"; exit 1; }; done
tail -2 $OUT/frames.json
