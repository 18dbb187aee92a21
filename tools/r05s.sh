#!/bin/bash
# r05s: grazing-band cells per face edge x band width tau_g (HRT_DIR_RES_SMALL / HRT_BAND_TAU): base (256,
# 3e-3), ndr1024 (1024, 3e-3; multi-level band build), t2_1024 (2e-3), t15_1024 (1.5e-3), dr1536, t15_2048:
# parity subset for the tau variants, then whole frame + rank 6 of 8 at bench.py's shape, island and cave x2.
set -o pipefail
OUT=gpurun_out/r05s; mkdir -p $OUT
B=epq_raytracer_amd/build
LIBS="base ndr1024 t2_1024 t15_1024 dr1536 t15_2048"
for L in t15_1024 t15_2048; do
  HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -x -k "headline or golden or grazing or wq_node_radius or degenerate" --timeout 200 --timeout-method thread > $OUT/tests_$L.log 2>&1 || { echo "tests $L failed"; tail -30 $OUT/tests_$L.log; exit 1; }
  echo "$L $(tail -1 $OUT/tests_$L.log)"
done
for r in 1 2; do
  for S in island cave; do
    for L in $LIBS; do
      HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 150 python3 tools/rank_shape.py --rounds 1 --parts 6 --scene $S > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L $S failed"; tail -5 $OUT/rs.jsonl; exit 1; }
      echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_ab.txt
    done
  done
done
