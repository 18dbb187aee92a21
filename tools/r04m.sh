set -o pipefail
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 300 python3 tools/realtime.py --lanes 2 3 --busy-split 1 2 --defer 0 1 --rounds 2 --frames 32 > $O/rt_acc.jsonl 2> $O/rt_acc.err &&
timeout -k 10 300 python3 tools/realtime.py --lanes 1 2 3 --busy-split 1 2 --defer 0 --rounds 2 --frames 32 --no-accumulate > $O/rt_noacc.jsonl 2> $O/rt_noacc.err
