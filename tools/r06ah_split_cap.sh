#!/bin/bash
# r06ah: ranks of 8 at bench.py's shape with the heavy split capped at 2 or 4 items (HRT_OPT_SPLIT) and the
# threshold at 1 x a wave's share (HRT_OPT_SPLIT_FACTOR = 1) against auto (8 items, 1.25 x), island and cave.
set -o pipefail
OUT=gpurun_out/r06ah; mkdir -p $OUT
for s in island cave; do
for cfg in auto s2 s2f1 s4f1; do
  case $cfg in auto) OPT="";; s2) OPT="--option 5=2";; s2f1) OPT="--option 5=2 --option 6=1";; s4f1) OPT="--option 5=4 --option 6=1";; esac
  timeout -k 10 280 python3 tools/rank_shape.py --scene $s --rounds 2 $OPT > $OUT/${s}_$cfg.jsonl 2>&1 || { echo "$s $cfg failed"; tail -3 $OUT/${s}_$cfg.jsonl; exit 1; }
  echo "== $s $cfg"; tail -1 $OUT/${s}_$cfg.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['whole_kernel_ms'], [r['slowest_over_fair'] for r in d['runs']], [r['slowest_ms'] for r in d['runs']])"
done
done
