#!/bin/bash
# r05t: the full GPU suite on the 1024-cell build (ab_n2dr1024: multi-level band build, flat task buffers;
# duration against the product's ~93 s), then cells x tau_g A/B: base, n2dr1024, n2dr1536, n2dr2048,
# t4_1024 (4e-3), t5_1024 (5e-3): whole frame + rank 6 of 8 at bench.py's shape, island and cave x2.
set -o pipefail
OUT=gpurun_out/r05t; mkdir -p $OUT
B=epq_raytracer_amd/build
HRT_LIB=$B/ab_n2dr1024/libhip_raytrace.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread --durations=15 > $OUT/tests_n2dr1024.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests_n2dr1024.log; exit 1; }
grep -E "passed|failed" $OUT/tests_n2dr1024.log | tail -1
for L in t4_1024 t5_1024; do
  HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -x -k "headline or golden or grazing or wq_node_radius or degenerate" --timeout 200 --timeout-method thread > $OUT/tests_$L.log 2>&1 || { echo "tests $L failed"; tail -30 $OUT/tests_$L.log; exit 1; }
  echo "$L $(tail -1 $OUT/tests_$L.log)"
done
LIBS="base n2dr1024 n2dr1536 n2dr2048 t4_1024 t5_1024"
for r in 1 2; do
  for S in island cave; do
    for L in $LIBS; do
      HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 150 python3 tools/rank_shape.py --rounds 1 --parts 6 --scene $S > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L $S failed"; tail -5 $OUT/rs.jsonl; exit 1; }
      echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_ab.txt
    done
  done
done
