#!/bin/bash
# r03 GPU check: the GPU suite, the self-spawned 2-rank rehearsal (gloo gather on one GPU, --verify on by
# default), the RCCL 2-rank refusal on a 1-GPU box, and the N=1 bench line.
# Usage (repo root, via gpurun): bash tools/r03_check.sh <tag> [SKIP_TESTS=1]
set -o pipefail
TAG=${1:-r03a}
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
fi
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 16 --warmup 2 --cpu-seconds 0 --realtime-frames 0 > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err || { echo "n2 gloo failed"; tail -30 $OUT/bench_n2_gloo.err; exit 1; }
cat $OUT/bench_n2_gloo.json
timeout -k 10 120 python3 bench.py --gpus 2 --steps 4 > $OUT/bench_n2_nccl.json 2> $OUT/bench_n2_nccl.err
echo "rccl --gpus 2 on one GPU: exit $? ($(tail -1 $OUT/bench_n2_nccl.err))"
timeout -k 10 600 python3 bench.py --cpu-seconds 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
# optional A/B of library builds (AB_LIBS="libA libB ..."): interleaved per-frame times, island and cave
if [ -n "$AB_LIBS" ]; then
  timeout -k 10 600 bash tools/ab.sh ${AB_ROUNDS:-2} $AB_LIBS -- --scene cave > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
  timeout -k 10 600 bash tools/ab.sh ${AB_ROUNDS:-2} $AB_LIBS > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
  python3 tools/ab_summary.py $OUT/ab_cave.jsonl $OUT/ab_island.jsonl
fi
