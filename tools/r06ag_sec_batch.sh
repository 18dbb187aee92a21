#!/bin/bash
# r06ag: the bounce-batch threshold (HRT_OPT_SECONDARY_BATCH, auto 28 island / 36 cave since r02) re-swept on this
# round's kernel: whole frames at bench.py's shape (5 warm-up + 20 in one launch), 2 rounds, interleaved.
set -o pipefail
OUT=gpurun_out/r06ag; mkdir -p $OUT
for r in 0 1; do
for v in 20 24 28 32 36; do
  timeout -k 10 120 python3 tools/rank_shape.py --scene island --rounds 1 --parts --option 3=$v > $OUT/island_${v}_$r.jsonl 2>&1 || { echo "island $v failed"; tail -3 $OUT/island_${v}_$r.jsonl; exit 1; }
  echo "island $v $r $(tail -1 $OUT/island_${v}_$r.jsonl | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["whole_kernel_ms"])')"
done
for v in 28 32 36 40 44; do
  timeout -k 10 120 python3 tools/rank_shape.py --scene cave --rounds 1 --parts --option 3=$v > $OUT/cave_${v}_$r.jsonl 2>&1 || { echo "cave $v failed"; tail -3 $OUT/cave_${v}_$r.jsonl; exit 1; }
  echo "cave $v $r $(tail -1 $OUT/cave_${v}_$r.jsonl | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["whole_kernel_ms"])')"
done
done
