#!/bin/bash
# r05l: the rgba8 combiner with a UNORM8 table and a shared reciprocal (HRT_COMBINE_FAST, ab_combfast) against
# the reference spelling (ab_base): GPU suite subset on the in-tree build, then bench.py itself (ms per step,
# per_frame_dispatch_ms) alternating, and the accumulate kernels' times from a rocprofv3 kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/r05l; mkdir -p $OUT
B=epq_raytracer_amd/build
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_checkpoint.py -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2 3; do
  for L in base combfast; do
    HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 300 python3 bench.py --cpu-seconds 0 > $OUT/b.json 2> $OUT/b.err || { echo "bench $L failed"; tail -5 $OUT/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$r $L', d['ms_per_step'], d['roofline']['kernel_ms'], d['per_frame_dispatch_ms'])" | tee -a $OUT/bench_ab.txt
  done
done
for L in base combfast; do
  HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$L -o run --output-format csv -- python3 bench.py --cpu-seconds 0 > $OUT/prof_$L.log 2>&1 || { echo "prof $L failed"; tail -5 $OUT/prof_$L.log; exit 1; }
  find $OUT/prof_$L -name '*kernel_stats.csv' -exec grep -h accumulate {} \; | sed "s/^/$L /"
done
