#!/bin/bash
# Rehearse bench.py's N>1 path on a 1-GPU box: 2 ranks share cuda:0, gloo (host-staged) gather,
# rank 0 verifies the gathered frame against a full-frame render.  Never used for the N=8 case.
set -o pipefail
OUT=gpurun_out/${1:-rehearsal}; mkdir -p $OUT
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --dist-backend gloo --verify --spp 16 \
  > $OUT/n2.json 2> $OUT/n2.err || { echo "rehearsal failed"; tail -30 $OUT/n2.err; exit 1; }
cat $OUT/n2.json
