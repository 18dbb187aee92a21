#!/bin/bash
# r06ab: ranks of 8 at bench.py's shape with the heavy threshold at 1 x a wave's share (HRT_OPT_SPLIT_FACTOR=1)
# against auto (2 x at these shapes): cave (one tile of part 3 takes 18 ms a frame against a 15 ms share,
# profiles/r06/r06aa/) and island.
set -o pipefail
OUT=gpurun_out/r06ab; mkdir -p $OUT
for s in cave island; do
for f in auto 1; do
  OPT=""; [ $f != auto ] && OPT="--option 6=$f"
  timeout -k 10 280 python3 tools/rank_shape.py --scene $s --rounds 2 $OPT > $OUT/${s}_$f.jsonl 2>&1 || { echo "$s $f failed"; tail -3 $OUT/${s}_$f.jsonl; exit 1; }
  echo "== $s $f"; tail -1 $OUT/${s}_$f.jsonl | cut -c1-600
done
done
