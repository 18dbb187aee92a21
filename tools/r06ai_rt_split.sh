#!/bin/bash
# r06ai: the realtime loop (3 lanes, busy split 2) with fewer heavy splits: HRT_OPT_SPLIT_FACTOR 3 / 4 and
# HRT_OPT_SPLIT 1 (never split) against auto; island, 2 rounds.
set -o pipefail
OUT=gpurun_out/r06ai; mkdir -p $OUT
timeout -k 10 400 python3 tools/realtime.py --lanes 3 --busy-split 2 --rounds 2 --split 0 1 --factor -1 3 4 > $OUT/island.jsonl 2>&1 || { echo "failed"; tail -3 $OUT/island.jsonl; exit 1; }
cat $OUT/island.jsonl
