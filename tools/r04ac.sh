#!/bin/bash
# r04ac: the scheduler's GCN register-pressure trackers (-mllvm -amdgpu-use-amdgpu-trackers=1: scratch
# 92 -> 60 B, VGPR spills 18 -> 6, SGPR spills 54 -> 58) against the final build (ab_head): parity of
# the tracker build, then timing.
set -o pipefail
OUT=gpurun_out/r04ac; mkdir -p $OUT
B=epq_raytracer_amd/build
HRT_LIB=$B/ab_trk/libhip_raytrace.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
L="$B/ab_head/libhip_raytrace.so $B/ab_trk/libhip_raytrace.so"
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 4 $L > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 4 $L -- --scene cave --node-r 2 > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
