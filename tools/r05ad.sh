#!/bin/bash
# r05ad: bounce batch thresholds (HRT_OPT_SECONDARY_BATCH = 3) re-checked with the pixel pool: whole
# frame + rank 6 at bench.py's shape, island (default 28) and cave (default 36), x2.
set -o pipefail
OUT=gpurun_out/r05ad; mkdir -p $OUT
run() {  # scene tag options...
  local S=$1 T=$2; shift 2
  timeout -k 10 150 python3 tools/rank_shape.py --rounds 1 --parts 6 --scene $S "$@" > $OUT/rs.jsonl 2>&1 || { echo "rank shape $S $T failed"; tail -5 $OUT/rs.jsonl; exit 1; }
  echo "$r $T $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/knobs.txt
}
for r in 1 2; do
  run island def
  run island sb20 --option 3=20
  run island sb24 --option 3=24
  run island sb32 --option 3=32
  run cave def
  run cave sb28 --option 3=28
  run cave sb32 --option 3=32
  run cave sb44 --option 3=44
done
