#!/bin/bash
# r04v: (1) the RNG-domain self-check, which now counts the bare hardware square root's misses on u01
# draws and on -2 log(u01) over all 2^32 states, with the library built both ways (in-tree: corrected
# roots; ab_sul: bare roots, whose own check must then count no sqrt mismatch); (2) the parity suite on
# the in-tree build (inv_det by rcp_rn, the sky's fixed octant); (3) timing: r04t build (ab_cone2), + rcp_rn (ab_rcp), + bare
# roots (ab_sul), the SLP vectoriser on (ab_slp: v_pk_* packed f32); the sky's fixed octant (ab_oct = in-tree; ab_rcp without it).
set -o pipefail
OUT=gpurun_out/r04v; mkdir -p $OUT
B=epq_raytracer_amd/build
timeout -k 10 60 ./tools/probe/valu_rate > $OUT/valu_rate.jsonl 2>&1 || { echo "valu_rate failed"; tail -5 $OUT/valu_rate.jsonl; exit 1; }
cat $OUT/valu_rate.jsonl
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_boundary.py -k "rng_domain or math" -q -s --timeout 250 --timeout-method thread > $OUT/check.log 2>&1 || { echo "check failed"; tail -30 $OUT/check.log; exit 1; }
grep -a "bare hardware" $OUT/check.log; tail -1 $OUT/check.log
HRT_LIB=$B/ab_sul/libhip_raytrace.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_boundary.py -k "rng_domain" -q -s --timeout 250 --timeout-method thread > $OUT/check_sul.log 2>&1; echo "bare-root build self-check rc=$? $(tail -1 $OUT/check_sul.log)"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
HRT_LIB=$B/ab_slp/libhip_raytrace.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread > $OUT/tests_slp.log 2>&1 || { echo "slp tests failed"; tail -30 $OUT/tests_slp.log; exit 1; }
echo "slp build: $(tail -1 $OUT/tests_slp.log)"
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $B/ab_cone2/libhip_raytrace.so $B/ab_rcp/libhip_raytrace.so $B/ab_oct/libhip_raytrace.so $B/ab_sul/libhip_raytrace.so $B/ab_slp/libhip_raytrace.so > $OUT/ab_island.jsonl 2>&1 || { echo "ab island failed"; tail -5 $OUT/ab_island.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_island.jsonl
AB_BATCH=20 timeout -k 10 600 bash tools/ab.sh 3 $B/ab_cone2/libhip_raytrace.so $B/ab_rcp/libhip_raytrace.so $B/ab_oct/libhip_raytrace.so $B/ab_sul/libhip_raytrace.so $B/ab_slp/libhip_raytrace.so -- --scene cave --node-r 2 > $OUT/ab_cave.jsonl 2>&1 || { echo "ab cave failed"; tail -5 $OUT/ab_cave.jsonl; exit 1; }
python3 tools/ab_summary.py $OUT/ab_cave.jsonl
