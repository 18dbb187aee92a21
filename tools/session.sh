#!/bin/bash
# GPU session step: the GPU suite (unless SKIP_TESTS=1), smoke, optional interleaved A/B of library
# builds (AB_LIBS="libA libB ...", island and cave, AB_ROUNDS rounds), optional cull diagnostics of the
# product library (DIAG=1) and the N=1 bench line (BENCH=1).
# Usage (repo root, via gpurun): bash tools/session.sh <tag>
set -o pipefail
TAG=${1:?usage: session.sh <tag>}
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
fi
if [ -n "$AB_LIBS" ]; then
  timeout -k 10 600 bash tools/ab.sh ${AB_ROUNDS:-2} $AB_LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
  python3 tools/ab_summary.py $OUT/ab_island.jsonl
  if [ -z "$AB_NO_CAVE" ]; then
  timeout -k 10 600 bash tools/ab.sh ${AB_ROUNDS:-2} $AB_LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
  python3 tools/ab_summary.py $OUT/ab_cave.jsonl
  fi
fi
if [ -n "$DIAG" ]; then
  timeout -k 10 300 python3 tools/kbench.py --variants 0 --rounds 1 --no-ref --diag > $OUT/diag_island.jsonl 2>&1 || { echo "diag failed"; tail -5 $OUT/diag_island.jsonl; exit 1; }
  timeout -k 10 300 python3 tools/kbench.py --variants 0 --rounds 1 --no-ref --diag --scene cave > $OUT/diag_cave.jsonl 2>&1 || { echo "diag cave failed"; tail -5 $OUT/diag_cave.jsonl; exit 1; }
  grep -h primary_iters $OUT/diag_island.jsonl $OUT/diag_cave.jsonl | python3 -c "import sys,json; [print({k: d.get(k) for k in ('primary_iters','sky_items','sky_cycles','primary_cycles','bounce_cycles','shade_cycles','primary_lane_use','live_lane_use','loop_iters','bounce_lanes_per_iter')}) for d in map(json.loads, sys.stdin)]"
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python3 bench.py --cpu-seconds 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
