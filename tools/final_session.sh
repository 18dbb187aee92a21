#!/bin/bash
# Final GPU session for a build: GPU suite + smoke, PMC passes + bench line + rocprof kernel trace of
# the driver's shape (tools/gpu_round.sh), the cave line with its own PMC record, the self-spawned 2-rank
# gloo rehearsal (the N > 1 line's "ranks" object), and the BASELINE configs' per-frame times.
# Usage (via gpurun): bash tools/final_session.sh <tag>
set -o pipefail
TAG=${1:?usage: final_session.sh <tag>}
ROUND=${ROUND:-${TAG:0:3}}  # profiles/<round>/
OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/gpu_round.sh $TAG || exit 1
PMC=profiles/$ROUND/${TAG}_cave_pmc; mkdir -p $PMC
bash tools/pmc.sh $TAG/cave_pmc --scene cave > $OUT/cave_pmc.log 2>&1 || { echo "cave pmc failed"; tail -20 $OUT/cave_pmc.log; exit 1; }
cp $OUT/cave_pmc/pmc_traffic.json $PMC/pmc_traffic.json
timeout -k 10 600 python3 bench.py --scene cave --pmc-json $PMC/pmc_traffic.json > $OUT/bench_cave.json 2> $OUT/bench_cave.err || { echo "cave bench failed"; tail -20 $OUT/bench_cave.err; exit 1; }
cat $OUT/bench_cave.json
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 16 --warmup 2 --cpu-seconds 0 --realtime-frames 0 > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err || { echo "n2 gloo failed"; tail -30 $OUT/bench_n2_gloo.err; exit 1; }
cat $OUT/bench_n2_gloo.json
timeout -k 10 600 bash tools/configs_round.sh > $OUT/configs.txt 2>&1 || { echo "configs failed"; tail -5 $OUT/configs.txt; exit 1; }
cat $OUT/configs.txt
timeout -k 10 300 python3 tools/rank_shape.py --rounds 2 > $OUT/rank8_bench_shape.jsonl 2>&1 || { echo "rank shape failed"; tail -5 $OUT/rank8_bench_shape.jsonl; exit 1; }
tail -1 $OUT/rank8_bench_shape.jsonl
timeout -k 10 300 python3 tools/rank_shape.py --rounds 1 --scene cave > $OUT/rank8_bench_shape_cave.jsonl 2>&1 || { echo "cave rank shape failed"; tail -5 $OUT/rank8_bench_shape_cave.jsonl; exit 1; }
tail -1 $OUT/rank8_bench_shape_cave.jsonl
