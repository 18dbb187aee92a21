#!/bin/bash
# Per-frame times of the BASELINE configs on one GPU with the current library (64-frame hrt_compute_n
# launches): C5 per frame, the row-tile partitions of 2 / 4 / 8 ranks (each rendered alone: what one
# rank of an N-GPU run does), cave.  Usage (via gpurun): bash tools/configs_round.sh > gpurun_out/configs.txt
set -o pipefail
f() { timeout -k 10 120 python3 tools/frames.py --batch 64 --frames 2 "$@" 2>&1 | tail -1 | \
      python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms"])'; }
echo "C5 island 3840x2160 16spp 12b: $(f --size 3840x2160 --spp 16 --bounces 12)" || exit 1
for n in 2 4 8; do
  line="island 1080p 64spp 8b, ranks of $n (8-row tiles):"
  for r in $(seq 0 $((n - 1))); do line="$line rank$r $(f --partition 8,$r,$n | tr -d '[] ' )" || exit 1; done
  echo "$line"
done
echo "island 1080p 64spp 8b whole frame: $(f)"
echo "C3 cave 1080p 64spp 8b: $(f --scene cave)"
