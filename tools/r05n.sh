#!/bin/bash
# r05n: the tile-list cache tests (camera direction / jitter / regenerated rays) and the camera-list tests
set -o pipefail
OUT=gpurun_out/r05n; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_boundary.py -q -x -k "tile_lists or camera_lists" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
